"""GPU LDA sampler vs the exact sequential CPU sampler (likelihood trajectories)."""
import pytest
import torch

from harp_amd.models.lda import LDAConfig, run_lda, synthetic_corpus
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K", [20, 300, 1000])
def test_lda_gpu_matches_cpu_quality(cuda, K):
    toks = synthetic_corpus(2000, 3000, 20, 60, seed=4)
    cfg = LDAConfig(num_topics=K, alpha=50.0 / K, beta=0.01, iterations=20, print_interval=20)
    g = run_lda(Communicator(None, cuda), cfg, 2000, 3000, toks)
    c = run_lda(Communicator(None, torch.device("cpu")), cfg, 2000, 3000, toks)
    n = toks[0].numel()
    lg, lc = g["loglik"][-1][1], c["loglik"][-1][1]
    assert abs(lg - lc) / n < 0.1, (lg, lc)
