"""One-XCD symmetric eigensolver (csrc/eig.hip: cooperative Householder tridiagonalisation +
multisection) vs torch.linalg.eigvalsh (rocSOLVER) in fp64."""
import os
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
    w = EIG.eigvalsh(C, native=True)
    ref = torch.linalg.eigvalsh(C)
    scale = max(1.0, float(ref.abs().max()))
    assert float((w - ref).abs().max()) <= 1e-12 * scale * max(1, n) ** 0.5


@pytest.mark.parametrize("variant", ["ll", "fused", "twopass"])
@pytest.mark.parametrize("n", [3, 130, 1000])
def test_reduction_variants(cuda, variant, n, monkeypatch):
    """Both reduction forms (fused look-ahead default, two-pass) against rocSOLVER."""
    monkeypatch.setattr(EIG, "VARIANT", variant)
    C = _sym(n, 7 * n, cuda)
    w = EIG.eigvalsh(C)
    ref = torch.linalg.eigvalsh(C)
    assert float((w - ref).abs().max()) <= 1e-12 * max(1.0, float(ref.abs().max())) * max(1, n) ** 0.5


@pytest.mark.parametrize("n", [3, 4, 5, 17, 64, 65, 130, 513, 1000, 1024])
def test_sytrd_ll_eigh(cuda, n):
    """The chip-wide reduction (csrc/eig_ll.hip) runs (no fallback) and eigh through it
    matches rocSOLVER: eigenvalues, |V^T V - I| and the residual |C V - V L| / |C|."""
    C = _sym(n, 3 * n + 1, cuda)
    assert EIG.sytrd_ll(C) is not None
    lam, V = EIG.eigh(C, native=True)
    ref = torch.linalg.eigvalsh(C)
    nc = float(torch.linalg.matrix_norm(C, 2))
    I = torch.eye(n, dtype=torch.float64, device=cuda)
    assert float((lam - ref).abs().max()) <= 1e-12 * nc * n ** 0.5
    assert float((V.t() @ V - I).abs().max()) <= 1e-13 * max(1.0, n / 100)
    assert float((C @ V - V * lam).abs().max()) <= 1e-13 * nc * max(1.0, n / 100)


def test_sytrd_ll_repeated_calls(cuda):
    """Back-to-back calls reuse nothing stale (tags restart from zeroed granules each call)
    and give bit-identical tridiagonals."""
    C = _sym(700, 5, cuda)
    r1 = EIG.sytrd_ll(C)
    r2 = EIG.sytrd_ll(C)
    assert r1 is not None and r2 is not None
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


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


def _tridiag_cases():
    import numpy as np

    rng = np.random.default_rng(0)
    n = 1000
    yield "randn", rng.standard_normal(n), rng.standard_normal(n - 1)
    yield "cluster", 1 + 1e-6 * rng.standard_normal(n), 1e-6 * rng.standard_normal(n - 1)
    yield "wilkinson", np.abs(np.arange(n) - n // 2).astype(float), np.ones(n - 1)
    e = np.ones(n - 1)
    e[::25] = 1e-15
    yield "glued", np.tile(np.abs(np.arange(25) - 12.0), 40), e
    d = np.ones(n)
    d[::2] = 2.0
    yield "decoupled", d, np.zeros(n - 1)
    for m in (1, 2, 3, 17, 64, 65, 4096):
        yield f"n{m}", rng.standard_normal(m), rng.standard_normal(m - 1)
    # every merge on the one-wave path (n <= 64), with rotations (cluster) and zero couplings
    yield "cluster64", 1 + 1e-9 * rng.standard_normal(64), 1e-9 * rng.standard_normal(63)
    e = rng.standard_normal(63)
    e[::4] = 0.0
    yield "split64", np.repeat(rng.standard_normal(16), 4), e


@pytest.mark.parametrize("case", list(_tridiag_cases()), ids=lambda c: c[0])
def test_dc_tridiag_kernels(cuda, case):
    """csrc/tridiag_dc.hip against LAPACK on hard spectra (clusters, Wilkinson, glued,
    decoupled blocks, odd sizes up to the 4096 limit)."""
    _, d, e = case
    n = d.size
    dg = torch.from_numpy(d).to(cuda)
    eg = torch.from_numpy(e).to(cuda)
    w, V = EIG.eigh_tridiag(dg, eg)
    T = torch.diag(dg) + torch.diag(eg, 1) + torch.diag(eg, -1)
    nt = max(float(torch.linalg.matrix_norm(T, 2)), 1e-300)
    I = torch.eye(n, dtype=torch.float64, device=cuda)
    orth = float((V.t() @ V - I).abs().max())
    res = float((T @ V - V * w).abs().max()) / nt
    ev = float((w - torch.linalg.eigvalsh(T)).abs().max()) / nt
    assert orth <= 1e-12 and res <= 1e-12 and ev <= 1e-12, (orth, res, ev)


def test_dc_level_kernels_only(cuda):
    """HARP_DC_WAVE_MERGE=0 (read once per process, so in a child process): every level on
    the level kernels, the path the one-wave merge kernel replaces for merges <= 64 rows."""
    import subprocess
    import sys

    code = (
        "import numpy as np, torch\n"
        "from harp_amd.ops import eig as EIG\n"
        "rng = np.random.default_rng(1)\n"
        "for n in (64, 1000):\n"
        "    for tag in ('randn', 'cluster'):\n"
        "        sc = 1.0 if tag == 'randn' else 1e-9\n"
        "        d = torch.from_numpy(1 + sc * rng.standard_normal(n)).cuda()\n"
        "        e = torch.from_numpy(sc * rng.standard_normal(n - 1)).cuda()\n"
        "        w, V = EIG.eigh_tridiag(d, e)\n"
        "        T = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)\n"
        "        nt = float(torch.linalg.matrix_norm(T, 2))\n"
        "        I = torch.eye(n, dtype=torch.float64, device='cuda')\n"
        "        assert float((V.t() @ V - I).abs().max()) <= 1e-12\n"
        "        assert float((T @ V - V * w).abs().max()) / nt <= 1e-12\n"
        "print('ok')\n")
    env = dict(os.environ, HARP_DC_WAVE_MERGE="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_eigh_correlation_matrix(cuda):
    """The PCA pass's 1000 x 1000 correlation matrix: eigenvalues AND vectors through the
    one-XCD reduction + D&C + WY back-transform: |V^T V - I| <= 1e-12, |C V - V L| <=
    1e-11 |C|, eigenvalues within 1e-12 of rocSOLVER (timings printed)."""
    g = torch.Generator(device=cuda).manual_seed(0)
    X = torch.rand(20000, 1000, generator=g, device=cuda, dtype=torch.float64)
    Xc = X - X.mean(0)
    C = Xc.t() @ Xc
    sd = torch.sqrt(torch.diagonal(C))
    C = C / torch.outer(sd, sd)
    lam, V = EIG.eigh(C)
    ref = torch.linalg.eigvalsh(C)
    I = torch.eye(1000, dtype=torch.float64, device=cuda)
    orth = float((V.t() @ V - I).abs().max())
    res = float((C @ V - V * lam).abs().max()) / float(torch.linalg.matrix_norm(C, 2))
    assert float((lam - ref).abs().max()) <= 1e-12
    assert orth <= 1e-12 and res <= 1e-11, (orth, res)
    ts = {}
    for name, fn in (("harp", EIG.eigh), ("torch", torch.linalg.eigh)):
        fn(C)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn(C)
        torch.cuda.synchronize()
        ts[name] = (time.perf_counter() - t0) / 5
    print(f"eigh 1000 x 1000 (vectors): harp {ts['harp'] * 1e3:.2f} ms, rocSOLVER {ts['torch'] * 1e3:.2f} ms")


def test_eigh_native_above_crossover(cuda):
    """Above NATIVE_MAX_N the library routes to rocSOLVER; native=True still runs the kernels
    (n = 2048: reduction + D&C + back-transform) to the same accuracy."""
    n = 2048
    assert n > EIG.NATIVE_MAX_N
    C = _sym(n, 11, cuda)
    lam, V = EIG.eigh(C, native=True)
    ref = torch.linalg.eigvalsh(C)
    nc = float(torch.linalg.matrix_norm(C, 2))
    I = torch.eye(n, dtype=torch.float64, device=cuda)
    assert float((lam - ref).abs().max()) <= 1e-12 * nc * n ** 0.5
    assert float((V.t() @ V - I).abs().max()) <= 1e-12
    assert float((C @ V - V * lam).abs().max()) <= 1e-11 * nc
    lam2, _ = EIG.eigh(C)  # crossover path
    assert float((lam2 - ref).abs().max()) <= 1e-12 * nc
