"""RBF kernel matrix: GEMM + the in-place HIP epilogue (csrc/kernelmat.hip) vs the torch
expression exp(-max(|x|^2 + |y|^2 - 2 x.y, 0) / (2 sigma^2))."""
import time

import pytest
import torch

from harp_amd.models import kernels as KF

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-12), (torch.float32, 2e-5)])
@pytest.mark.parametrize("n,m,d", [(1, 1, 3), (300, 77, 16), (1025, 513, 64)])
def test_rbf_matches_torch(cuda, dtype, tol, n, m, d):
    g = torch.Generator(device=cuda).manual_seed(n + m)
    X = torch.randn(n, d, generator=g, device=cuda, dtype=dtype)
    Y = torch.randn(m, d, generator=g, device=cuda, dtype=dtype)
    K = KF.rbf_kernel(X, Y, 2.5)
    ref = torch.exp(-KF.sq_distances(X, Y) / (2 * 2.5 * 2.5))
    assert K.shape == (n, m)
    assert float((K - ref).abs().max()) <= tol


def test_rbf_one_pass_speed(cuda):
    X = torch.randn(20000, 16, device=cuda, dtype=torch.float64)
    ts = {}
    for name, fn in (("fused", lambda: KF.rbf_kernel(X, X, 4.0)),
                     ("torch", lambda: torch.exp(-KF.sq_distances(X, X) / 32.0))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts[name] = (time.perf_counter() - t0) / 3
    print(f"RBF 20k x 20k fp64: fused {ts['fused'] * 1e3:.2f} ms, torch {ts['torch'] * 1e3:.2f} ms")
    assert ts["fused"] < ts["torch"]
