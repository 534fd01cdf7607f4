"""ALS normal-equation kernel (``csrc/als.hip``) against the plain PyTorch formulation of
the same per-row systems (outer products + index_add, fp64 on the CPU), explicit and
implicit, fp32 and fp64, f up to the kernel's 64, rows with 0 .. 100 ratings."""
import pytest
import torch

from harp_amd.models import als as A
from harp_amd.ops import als as OA

pytestmark = pytest.mark.gpu


def _problem(n_rows, n_cols, nnz, f, seed):
    g = torch.Generator().manual_seed(seed)
    rows = torch.sort(torch.randint(0, n_rows - 3, (nnz,), generator=g)).values  # last rows empty
    rows[:100] = 0  # one row longer than the kernel's 32-row LDS chunk
    rows = torch.sort(rows).values
    cols = torch.randint(0, n_cols, (nnz,), generator=g)
    vals = torch.rand(nnz, generator=g, dtype=torch.float64) * 5
    vals[::7] = 0.0
    F = torch.randn(n_cols, f, generator=g, dtype=torch.float64) * 0.3
    return rows, cols, vals, F


@pytest.mark.parametrize("implicit", [False, True])
@pytest.mark.parametrize("f,dt,wave", [(8, torch.float64, True), (50, torch.float32, True), (50, torch.float32, False),
                                       (64, torch.float32, True), (64, torch.float64, True)])
def test_solve_rows_native_matches_torch(cuda, implicit, f, dt, wave):
    rows, cols, vals, F = _problem(700, 300, 6000, f, f)
    cfg = A.ALSConfig(factors=f, implicit=implicit, alpha=2.0, lam=0.1, block_bytes=1 << 22, wave_solve=wave)
    want = A.solve_rows(rows, cols, vals, 700, F, cfg)  # CPU: torch path, fp64
    got = A.solve_rows(rows.to(cuda), cols.to(cuda), vals.to(cuda), 700, F.to(cuda, dt), cfg)
    tol = 1e-9 if dt == torch.float64 else 2e-3
    assert torch.allclose(got.cpu().double(), want, rtol=tol, atol=tol)


def test_normal_equations_direct(cuda):
    rows, cols, vals, F = _problem(64, 40, 900, 16, 3)
    crow = torch.zeros(65, dtype=torch.int64)
    crow[1:] = torch.cumsum(torch.bincount(rows, minlength=64), 0)
    G = F.t() @ F
    Am = torch.empty(64, 16, 16, dtype=torch.float64, device=cuda)
    rhs = torch.empty(64, 16, dtype=torch.float64, device=cuda)
    OA.normal_equations(crow.to(cuda), cols.to(cuda), vals.to(cuda), F.to(cuda), G.to(cuda), True, 1.5, 0.2, False,
                        Am, rhs, 0)
    for r in (0, 5, 63):
        sl = slice(int(crow[r]), int(crow[r + 1]))
        Fc, v = F[cols[sl]], vals[sl]
        want = G + Fc.t() @ (1.5 * v[:, None] * Fc) + 0.2 * torch.eye(16, dtype=torch.float64)
        wr = Fc.t() @ ((1 + 1.5 * v) * (v > 0))
        assert torch.allclose(Am[r].cpu(), want, rtol=1e-12, atol=1e-12)
        assert torch.allclose(rhs[r].cpu(), wr, rtol=1e-12, atol=1e-12)


def test_fused_solve_flags_non_spd_rows(cuda):
    rows, cols, vals, F = _problem(64, 40, 4000, 16, 4)  # rows 61..63 have no ratings
    crow = torch.zeros(65, dtype=torch.int64)
    crow[1:] = torch.cumsum(torch.bincount(rows, minlength=64), 0)
    X = torch.empty(64, 16, dtype=torch.float64, device=cuda)
    info = torch.empty(64, dtype=torch.int32, device=cuda)
    # explicit, lam = 0: an empty row's system is the zero matrix
    OA.normal_equations(crow.to(cuda), cols.to(cuda), vals.to(cuda), F.to(cuda), None, False, 0.0, 0.0, True,
                        None, None, 0, X=X, info=info)
    info = info.cpu()
    assert info[61:].tolist() == [1, 1, 1] and int(info[:61].sum()) == 0
    for r in (0, 10):
        sl = slice(int(crow[r]), int(crow[r + 1]))
        Fc, v = F[cols[sl]], vals[sl]
        want = torch.linalg.solve(Fc.t() @ Fc, Fc.t() @ v)
        assert torch.allclose(X[r].cpu(), want, rtol=1e-8, atol=1e-8)
    cfg = A.ALSConfig(factors=16, implicit=False, lam=0.0)
    got = A.solve_rows(rows.to(cuda), cols.to(cuda), vals.to(cuda), 64, F.to(cuda), cfg)
    # the flagged block went through the rocSOLVER path; its SPD rows agree with the fused solve
    assert torch.allclose(got[:61].cpu(), X[:61].cpu(), rtol=1e-8, atol=1e-8)


@pytest.mark.parametrize("f", [1, 7, 32, 64])
def test_wave_chol_solve_matches_torch(cuda, f):
    """One-wave-per-system register Cholesky (als_chol_solve_kernel) vs torch.linalg.solve
    in fp64 on random SPD systems; a non-SPD system is flagged, the others are unaffected."""
    g = torch.Generator().manual_seed(f)
    m = 37
    B = torch.randn(m, f, f + 3, generator=g, dtype=torch.float64)
    Am = B @ B.transpose(1, 2) + 0.5 * torch.eye(f, dtype=torch.float64)
    rhs = torch.randn(m, f, generator=g, dtype=torch.float64)
    Am[5] = -torch.eye(f, dtype=torch.float64)  # not SPD
    want = torch.linalg.solve(Am, rhs[:, :, None])[:, :, 0]
    X = torch.empty(m, f, device=cuda)
    info = torch.full((m,), 7, dtype=torch.int32, device=cuda)
    OA.chol_solve(Am.to(cuda, torch.float32).contiguous(), rhs.to(cuda, torch.float32).contiguous(), X, info)
    info = info.cpu()
    assert info[5] == 1 and int(info.sum()) == 1
    ok = torch.arange(m) != 5
    scale = want[ok].abs().max()
    assert torch.allclose(X.cpu().double()[ok], want[ok], rtol=2e-3, atol=2e-4 * float(scale))
