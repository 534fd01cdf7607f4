"""Diagnostic: final log-likelihood per token of the LDA samplers on the small synthetic
corpus of tests/test_lda_gpu.py (dense GPU, sparse GPU at several workgroup sizes, CPU)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from harp_amd.models.lda import LDAConfig, run_lda, synthetic_corpus
from harp_amd.ops import lda as L
from harp_amd.parallel.comm import Communicator

K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
toks = synthetic_corpus(2000, 3000, 20, 60, seed=4)
n = toks[0].numel()
cfg = LDAConfig(num_topics=K, alpha=50.0 / K, beta=0.01, iterations=12, print_interval=12)
out = {"K": K}
dev = torch.device("cuda")
if K <= 1024:
    L.SAMPLER = "dense"
    out["dense"] = run_lda(Communicator(None, dev), cfg, 2000, 3000, toks)["loglik"][-1][1] / n
L.SAMPLER = "sparse"
for w in (1, 2, 4, 8, 16):
    L.SPARSE_WAVES = w
    out[f"sparse_w{w}"] = run_lda(Communicator(None, dev), cfg, 2000, 3000, toks)["loglik"][-1][1] / n
out["cpu"] = run_lda(Communicator(None, torch.device("cpu")), cfg, 2000, 3000, toks)["loglik"][-1][1] / n
print(json.dumps(out), flush=True)
