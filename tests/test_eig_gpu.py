"""One-XCD symmetric eigensolver (csrc/eig.hip: cooperative Householder tridiagonalisation +
multisection) vs torch.linalg.eigvalsh (rocSOLVER) in fp64."""
import time

import pytest
import torch

from harp_amd.ops import eig as EIG

pytestmark = pytest.mark.gpu


def _sym(n, seed, cuda):
    g = torch.Generator(device=cuda).manual_seed(seed)
    M = torch.randn(n, n, generator=g, device=cuda, dtype=torch.float64)
    return (M + M.t()) / 2


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 65, 513, 1000, 2048])
def test_random_symmetric(cuda, n):
    C = _sym(n, n, cuda)
    w = EIG.eigvalsh(C)
    ref = torch.linalg.eigvalsh(C)
    scale = max(1.0, float(ref.abs().max()))
    assert float((w - ref).abs().max()) <= 1e-12 * scale * max(1, n) ** 0.5


@pytest.mark.parametrize("variant", ["fused", "twopass"])
@pytest.mark.parametrize("n", [3, 130, 1000])
def test_reduction_variants(cuda, variant, n, monkeypatch):
    """Both reduction forms (fused look-ahead default, two-pass) against rocSOLVER."""
    monkeypatch.setattr(EIG, "VARIANT", variant)
    C = _sym(n, 7 * n, cuda)
    w = EIG.eigvalsh(C)
    ref = torch.linalg.eigvalsh(C)
    assert float((w - ref).abs().max()) <= 1e-12 * max(1.0, float(ref.abs().max())) * max(1, n) ** 0.5


def test_degenerate_structure(cuda):
    """Zero Householder columns (diagonal, already tridiagonal, repeated eigenvalues) take
    the tau = 0 path."""
    for C in (torch.eye(300, dtype=torch.float64, device=cuda) * 3.0,
              torch.diag(torch.arange(200, dtype=torch.float64, device=cuda)),
              torch.diag(torch.ones(149, dtype=torch.float64, device=cuda), 1)
              + torch.diag(torch.ones(149, dtype=torch.float64, device=cuda), -1)
              + 2 * torch.eye(150, dtype=torch.float64, device=cuda)):
        w = EIG.eigvalsh(C)
        ref = torch.linalg.eigvalsh(C)
        assert float((w - ref).abs().max()) <= 1e-12 * max(1.0, float(ref.abs().max())) * 20


def test_correlation_matrix_speed(cuda):
    """The PCA pass's matrix: 1000 x 1000 correlation of uniform data (Marchenko-Pastur
    spectrum around 1): within 1e-12 of rocSOLVER (timings printed; the speed gate lives in
    scripts/bench_speedups.py)."""
    g = torch.Generator(device=cuda).manual_seed(0)
    X = torch.rand(20000, 1000, generator=g, device=cuda, dtype=torch.float64)
    Xc = X - X.mean(0)
    C = Xc.t() @ Xc
    sd = torch.sqrt(torch.diagonal(C))
    C = C / torch.outer(sd, sd)
    ref = torch.linalg.eigvalsh(C)
    w = EIG.eigvalsh(C)
    assert float((w - ref).abs().max()) <= 1e-12
    ts = {}
    for name, fn in (("harp", EIG.eigvalsh), ("torch", torch.linalg.eigvalsh)):
        fn(C)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn(C)
        torch.cuda.synchronize()
        ts[name] = (time.perf_counter() - t0) / 5
    print(f"eigvalsh 1000 x 1000: one-XCD {ts['harp'] * 1e3:.2f} ms, rocSOLVER {ts['torch'] * 1e3:.2f} ms")
