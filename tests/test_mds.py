"""WDA-MDS (deterministic-annealing weighted SMACOF): recovers a 3-D point cloud's
geometry (low normalised stress), honours zero weights, and the P=2 gloo run equals
the single-worker run."""
import torch

from harp_amd.models import mds as MD
from harp_amd.parallel.comm import Communicator
from harp_amd.runtime.launcher import launch


def _problem(n=40, seed=0):
    g = torch.Generator().manual_seed(seed)
    Y = torch.rand(n, 3, generator=g, dtype=torch.float64)
    D = MD.quantize_distances(torch.cdist(Y, Y))
    W = torch.ones(n, n, dtype=torch.float64)
    return D, W


def test_wdamds_recovers_geometry():
    D, W = _problem()
    out = MD.wda_mds(Communicator(), D, W, 0, 40, MD.MDSConfig(d=3, alpha=0.9, threshold=1e-7))
    assert out["stress"] < 1e-3
    X = out["X"]
    assert torch.allclose(torch.cdist(X, X), D, atol=0.05)
    # annealing stages ran and the stress at T=0 is the last entry
    assert len(out["history"]) > 3 and out["history"][-1]["T"] == 0.0


def test_wdamds_zero_weights_ignored():
    D, W = _problem()
    D2 = D.clone()
    D2[0, 1] = D2[1, 0] = 1.0  # corrupted entry ...
    W[0, 1] = W[1, 0] = 0.0  # ... with zero weight
    out = MD.wda_mds(Communicator(), D2, W, 0, 40, MD.MDSConfig(d=3, alpha=0.9, threshold=1e-7))
    assert out["stress"] < 1e-3


def _job(comm, D, W):
    n = D.shape[0]
    a, b = comm.rank * n // comm.world_size, (comm.rank + 1) * n // comm.world_size
    return MD.wda_mds(comm, D[a:b], W[a:b], a, n, MD.MDSConfig(d=3, alpha=0.9, threshold=1e-6))


def test_wdamds_distributed_equals_single():
    D, W = _problem(30, 1)
    single = MD.wda_mds(Communicator(), D, W, 0, 30, MD.MDSConfig(d=3, alpha=0.9, threshold=1e-6))
    res = launch(_job, 2, args=(D, W), timeout=300)
    for r in res:
        assert r["smacof_iters"] == single["smacof_iters"]
        assert torch.allclose(r["X"], single["X"], atol=1e-4)  # fp reduction order only
        assert abs(r["stress"] - single["stress"]) < 1e-12
