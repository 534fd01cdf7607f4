"""GPU color-coding kernels (csrc/graph.hip) vs fp64 torch references."""
import pytest
import torch

from harp_amd.models.graph import Template, brute_force_embeddings, color_count
from harp_amd.ops import graph as G
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("C", [1, 3, 10, 35, 64])
def test_csr_spmm_matches_index_add(cuda, C):
    g = torch.Generator().manual_seed(C)
    n, m = 5000, 80000
    rows = (torch.rand(m, generator=g) ** 2 * n).long()  # skewed degrees, some empty rows
    cols = torch.randint(0, 3000, (m,), generator=g)
    M = torch.rand(3000, C, generator=g, dtype=torch.float64)
    ref = torch.zeros(n, C, dtype=torch.float64).index_add_(0, rows, M[cols])
    csr = G.build_csr(rows.to(cuda), cols.to(cuda), n)
    out = G.spmm(csr, M.to(cuda))
    assert torch.allclose(out.cpu(), ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("k,sa,sp", [(5, 1, 1), (5, 2, 3), (7, 3, 3), (7, 1, 6)])
def test_colorset_combine_matches_cpu(cuda, k, sa, sp):
    from harp_amd.models.graph import _colorsets, _split_index

    g = torch.Generator().manual_seed(k * 10 + sa)
    n = 3000
    ca, cp, co = len(_colorsets(k, sa)[0]), len(_colorsets(k, sp)[0]), len(_colorsets(k, sa + sp)[0])
    A = torch.rand(n, ca, generator=g, dtype=torch.float64)
    N = torch.rand(n, cp, generator=g, dtype=torch.float64)
    tc, t1, t2 = _split_index(k, sa, sp)
    ref = G.combine(A, N, tc, t1, t2, co)
    out = G.combine(A.to(cuda), N.to(cuda), tc, t1, t2, co)
    assert torch.allclose(out.cpu(), ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("k", [3, 5, 7])
def test_color_count_gpu_equals_cpu_and_brute_force(cuda, k):
    g = torch.Generator().manual_seed(k)
    n, m = 14, 30
    u = torch.randint(0, n, (m,), generator=g)
    v = torch.randint(0, n, (m,), generator=g)
    keep = u != v
    u, v = u[keep], v[keep]
    e = sorted({(int(a), int(b)) if a < b else (int(b), int(a)) for a, b in zip(u, v)})
    src = torch.tensor([a for a, b in e] + [b for a, b in e])
    dst = torch.tensor([b for a, b in e] + [a for a, b in e])
    T = Template(k, [(i, i + 1) for i in range(k - 1)])
    colors = torch.randint(0, k, (n,), generator=g)
    gpu = color_count(Communicator(None, cuda), T, src, dst, n, colors)
    cpu = color_count(Communicator(None, torch.device("cpu")), T, src, dst, n, colors)
    assert gpu == cpu
    assert round(gpu) == brute_force_embeddings(T, e, n, colors.tolist())
