"""PageRank pull kernel (``csrc/graph.hip`` pagerank_pull_kernel) against a plain PyTorch
fp64 reference of the same step, for every lane-group size (in-degree 2 .. 100), and the
full ``pagerank`` app on the GPU against the reference's formulation
(contrib/.../simplepagerank/PageRankMapper.java:120-190: PR(src)/outdeg scattered to
the targets, dangling mass spread over all pages, ``0.85 * sum + 0.15 / N``)."""
import pytest
import torch

from harp_amd.models import graph as G
from harp_amd.ops import _lib
from harp_amd.ops import graph as GO
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


def _graph(n, avg, seed):
    g = torch.Generator().manual_seed(seed)
    m = n * avg
    # skewed targets (a few hub pages) + uniform sources; some pages dangle
    dst = (torch.rand(m, generator=g) ** 2 * n).long().clamp_max(n - 1)
    src = torch.randint(0, n - n // 10, (m,), generator=g)
    return src, dst


def _ref_pagerank(src, dst, n, iters, d=0.85):
    src, dst = src.double().long(), dst.long()
    outdeg = torch.bincount(src, minlength=n).double()
    dang = outdeg == 0
    pr = torch.full((n,), 1.0 / n, dtype=torch.float64)
    for _ in range(iters):
        c = torch.zeros(n, dtype=torch.float64)
        c.index_add_(0, dst, pr[src] / outdeg[src])
        c += pr[dang].sum() / n
        pr = d * c + (1 - d) / n
    return pr


@pytest.mark.parametrize("avg", [2, 6, 12, 24, 100])
def test_pull_step_matches_torch(cuda, avg):
    assert _lib.use_native(torch.empty(1, device=cuda)), "native kernels must load on the GPU"
    n = 20000
    src, dst = _graph(n, avg, avg)
    x = torch.rand(n, dtype=torch.float64)
    invdeg = torch.rand(n, dtype=torch.float64)
    dm = torch.tensor([0.125], dtype=torch.float64)
    want = torch.zeros(n, dtype=torch.float64)
    want.index_add_(0, dst, x[src])
    want = 0.85 * want + 0.01 + 0.5 * dm
    csr = GO.build_csr(dst.to(cuda), src.to(cuda), n)
    out, xn = GO.pagerank_pull(csr, x.to(cuda), 0.85, 0.01, 0.5, dm.to(cuda), invdeg.to(cuda), want_xnext=True)
    torch.cuda.synchronize()
    assert torch.allclose(out.cpu(), want, rtol=1e-13, atol=1e-13)
    assert torch.allclose(xn.cpu(), want * invdeg, rtol=1e-13, atol=1e-13)
    out2, none = GO.pagerank_pull(csr, x.to(cuda), 1.0, 0.0, 0.0)
    assert none is None
    ref2 = torch.zeros(n, dtype=torch.float64).index_add_(0, dst, x[src])
    assert torch.allclose(out2.cpu(), ref2, rtol=1e-13, atol=1e-13)


def test_pagerank_app_on_gpu(cuda):
    n = 5000
    src, dst = _graph(n, 8, 7)
    pr = G.pagerank(Communicator(device=cuda), src, dst, torch.arange(n), n, iterations=20)
    want = _ref_pagerank(src, dst, n, 20)
    assert torch.allclose(pr.cpu(), want, rtol=1e-12, atol=1e-15)
    assert abs(float(pr.sum()) - 1.0) < 1e-9
