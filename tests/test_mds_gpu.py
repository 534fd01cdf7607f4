"""GPU WDA-MDS row kernels (csrc/mds.hip) vs the fp64 torch formulas on the CPU."""
import math

import pytest
import torch

from harp_amd.models import mds as MD
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dim", [2, 3, 4])
@pytest.mark.parametrize("T", [0.0, 0.05])
def test_bc_and_stress_match_torch(cuda, dim, T):
    g = torch.Generator().manual_seed(dim)
    n, row0, n_r = 700, 200, 300
    Y = torch.rand(n, dim, generator=g, dtype=torch.float64)
    D = MD.quantize_distances(torch.cdist(Y, Y))[row0:row0 + n_r].contiguous()
    W = (torch.rand(n_r, n, generator=g, dtype=torch.float64) < 0.9).double()
    X = torch.rand(n, dim, generator=g, dtype=torch.float64)
    X[5] = X[row0 + 3]  # a coincident pair (d_ij < 1e-10 branch)
    comm = Communicator()
    cpu = MD._Rows(comm, D, W, row0)
    gpu = MD._Rows(Communicator(None, cuda), D.to(cuda), W.to(cuda), row0)
    assert gpu._native(X.to(cuda))
    bc_ref, bc = cpu.bc(X, T, dim), gpu.bc(X.to(cuda), T, dim).cpu()
    assert torch.allclose(bc, bc_ref, rtol=1e-9, atol=1e-9 * bc_ref.abs().max().item())
    s_ref, s = cpu.stress(X, T, dim), gpu.stress(X.to(cuda), T, dim).cpu()
    assert math.isclose(float(s), float(s_ref), rel_tol=1e-9)


def test_wdamds_gpu_equals_cpu(cuda):
    g = torch.Generator().manual_seed(0)
    Y = torch.rand(60, 3, generator=g, dtype=torch.float64)
    D = MD.quantize_distances(torch.cdist(Y, Y))
    W = torch.ones(60, 60, dtype=torch.float64)
    cfg = MD.MDSConfig(d=3, alpha=0.9, threshold=1e-7)
    ref = MD.wda_mds(Communicator(), D, W, 0, 60, cfg)
    out = MD.wda_mds(Communicator(None, cuda), D, W, 0, 60, cfg)
    assert out["stress"] < 1e-3
    assert abs(out["stress"] - ref["stress"]) < 1e-6
    assert torch.allclose(torch.cdist(out["X"].cpu(), out["X"].cpu()), D, atol=0.05)
