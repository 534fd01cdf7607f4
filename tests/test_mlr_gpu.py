"""GPU MLR SGD pass (csrc/mlr.hip, one launch per pass) vs the fp64 torch mini-batch pass."""
import pytest
import torch

from harp_amd.models import mlr as M
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch", [1, 64, 300, 1024])
def test_sgd_pass_matches_torch(cuda, batch):
    X, Y = M.synthetic_multilabel(1500, 400, 7, density=0.05, seed=batch)
    Xc = M.CSRRows.from_dense(X.double())
    g = torch.Generator().manual_seed(3)
    W0 = torch.randn(7, 401, generator=g, dtype=torch.float64) * 0.1
    Wc = W0.clone()
    M._sgd_pass(Wc, Xc, Y, 0.5, batch)
    Wg = W0.to(cuda)
    Yg = torch.zeros(1500, 9, device=cuda)
    Yg[:, 1:8] = Y.to(cuda)  # strided label view like the rotation slab's column block
    M._sgd_pass(Wg, Xc.to(cuda), Yg[:, 1:8], 0.5, batch)
    assert torch.allclose(Wg.cpu(), Wc, rtol=1e-9, atol=1e-11)


def test_mlr_train_gpu_equals_cpu(cuda):
    X, Y = M.synthetic_multilabel(800, 120, 5, density=0.08, seed=9)
    cfg = M.MLRConfig(alpha=1.0, iterations=3, batch_size=16)
    ref = M.train(Communicator(None, torch.device("cpu")), M.CSRRows.from_dense(X), Y, cfg, 5, 120)
    out = M.train(Communicator(None, cuda), M.CSRRows.from_dense(X), Y, cfg, 5, 120)
    assert torch.allclose(out["W"].cpu(), ref["W"], rtol=1e-9, atol=1e-11)
    ev = M.evaluate(Communicator(None, cuda), M.CSRRows.from_dense(X), Y, out["W"])
    ev_ref = M.evaluate(Communicator(None, torch.device("cpu")), M.CSRRows.from_dense(X), Y, ref["W"])
    assert abs(ev["micro_f1"] - ev_ref["micro_f1"]) < 1e-6 and ev["micro_f1"] > 0.3
