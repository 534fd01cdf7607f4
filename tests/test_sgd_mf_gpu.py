"""GPU MF-SGD kernels vs the native sequential CPU reference / torch."""
import pytest
import torch

from harp_amd.ops import mf as MF
from harp_amd.models.sgd_mf import SGDConfig, run_sgd, synthetic_ratings
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("r", [16, 48, 128])
def test_sse_matches_torch(cuda, r):
    n, nu, ni = 50000, 1000, 300
    g = torch.Generator().manual_seed(r)
    rows = torch.randint(0, nu, (n,), generator=g, dtype=torch.int32)
    cols = torch.randint(0, ni, (n,), generator=g, dtype=torch.int32)
    vals = torch.rand(n, generator=g) * 4 + 1
    W = torch.rand(nu, r, generator=g) * 0.3
    H = torch.rand(ni, r, generator=g) * 0.3
    ref = ((vals.double() - (W[rows.long()].double() * H[cols.long()].double()).sum(1)) ** 2).sum()
    got = MF.sse(rows.to(cuda), cols.to(cuda), vals.to(cuda), W.to(cuda), H.to(cuda))
    assert abs(got.item() - ref.item()) <= 1e-5 * ref.item()


def test_sgd_single_stream_matches_sequential(cuda):
    """chunk >= n -> one stream -> exactly the sequential order of the CPU reference."""
    n, nu, ni, r = 3000, 40, 30, 16
    g = torch.Generator().manual_seed(0)
    rows = torch.sort(torch.randint(0, nu, (n,), generator=g, dtype=torch.int32)).values
    cols = torch.randint(0, ni, (n,), generator=g, dtype=torch.int32)
    vals = torch.rand(n, generator=g) * 4 + 1
    W0 = torch.rand(nu, r, generator=g) * 0.3
    H0 = torch.rand(ni, r, generator=g) * 0.3
    Wc, Hc = W0.clone(), H0.clone()
    MF.sgd_update(rows, cols, vals, Wc, Hc, 0.01, 0.05)
    Wg, Hg = W0.to(cuda), H0.to(cuda)
    MF.sgd_update(rows.to(cuda), cols.to(cuda), vals.to(cuda), Wg, Hg, 0.01, 0.05, chunk=n)
    assert torch.allclose(Wg.cpu(), Wc, atol=2e-5) and torch.allclose(Hg.cpu(), Hc, atol=2e-5)


def test_sgd_gpu_converges_like_cpu(cuda):
    nu, ni = 3000, 800
    u, i, v = synthetic_ratings(nu, ni, 120000, seed=2)
    p = torch.randperm(u.numel(), generator=torch.Generator().manual_seed(0))
    k = int(0.9 * u.numel())
    train = (u[p[:k]], i[p[:k]], v[p[:k]])
    test = (u[p[k:]], i[p[k:]], v[p[k:]])
    cfg = SGDConfig(rank=32, lam=0.05, lr=0.01, epochs=10, test_every=10)
    g = run_sgd(Communicator(None, cuda), cfg, nu, ni, train, test)
    c = run_sgd(Communicator(None, torch.device("cpu")), cfg, nu, ni, train, test)
    # ~1.7k concurrent Hogwild streams on only 800 items: staleness costs a little accuracy
    assert abs(g["rmse"][-1][2] - c["rmse"][-1][2]) < 0.04, (g["rmse"], c["rmse"])
    assert g["trained"] == c["trained"] == 10 * k
