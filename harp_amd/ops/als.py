"""ALS per-row normal equations (``csrc/als.hip``): A_r = sum_j a_j F_j F_j^T + G +
lam_r I and rhs_r = sum_j b_j F_j for a block of CSR rows, fp32 / fp64, f <= 64."""
from __future__ import annotations

import torch

from . import _lib

MAX_F = 64
THREADS = 256  # workgroup size of the per-row kernel (csrc/als.hip kThreads)

_lib.register({
    name: [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_int, ct, ct,
           _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_void_p, _lib.c_void_p,
           _lib.c_void_p]
    for name, ct in (("harp_als_normal_f32", _lib.c_float), ("harp_als_normal_f64", _lib.c_double))
})
_lib.register({"harp_als_chol_solve_f32": [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_long, _lib.c_void_p,
                                           _lib.c_void_p, _lib.c_int, _lib.c_void_p]})
CHOL_VARIANT = 0  # 0: LDS column broadcast, 1: v_readlane broadcast (profiles/r2_als)


def available(t: torch.Tensor) -> bool:
    return _lib.use_native(t)


def normal_equations(crow: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, F: torch.Tensor, G, implicit: bool,
                     alpha: float, lam: float, scale_lam: bool, A, rhs, row0: int, X=None, info=None) -> None:
    """Fill ``A`` [m, f, f] and ``rhs`` [m, f] for rows row0 .. row0 + m of the CSR
    (``crow`` int64 over all rows, ``cols`` int64 row ids into ``F`` [*, f]); or, with
    ``X`` [m, f] and ``info`` [m] int32 given (A, rhs None), solve each system in the
    kernel (Cholesky in LDS): info[r] = 1 marks a row whose system was not SPD."""
    solve = X is not None
    m, f = (X if solve else rhs).shape
    dt = F.dtype
    assert f <= MAX_F and dt in (torch.float32, torch.float64)
    outs = (X, info) if solve else (A, rhs)
    if solve:
        assert info is not None and info.dtype == torch.int32 and info.shape == (m,) and X.dtype == dt
    else:
        assert A.shape == (m, f, f) and A.dtype == dt and rhs.dtype == dt
    for t in (crow, cols, vals, F) + outs:
        assert t.is_contiguous() and t.device == F.device
    assert crow.dtype == torch.int64 and cols.dtype == torch.int64 and vals.dtype == dt
    assert row0 + m < crow.numel() and int(crow[-1]) <= cols.numel() == vals.numel()
    if G is not None:
        G = G.to(dt).contiguous()
        assert G.shape == (f, f)
    fn = _lib.kernels().harp_als_normal_f32 if dt == torch.float32 else _lib.kernels().harp_als_normal_f64
    st = fn(crow.data_ptr(), cols.data_ptr(), vals.data_ptr(), F.data_ptr(), f,
            G.data_ptr() if G is not None else None, int(bool(implicit)), float(alpha), float(lam),
            int(bool(scale_lam)), None if solve else A.data_ptr(), None if solve else rhs.data_ptr(), int(row0), m,
            X.data_ptr() if solve else None, info.data_ptr() if solve else None, _lib.stream_ptr(F.device))
    _lib.check(st, "als_normal")


def chol_solve(A: torch.Tensor, rhs: torch.Tensor, X: torch.Tensor, info: torch.Tensor,
               variant: int | None = None) -> None:
    """X[r] = A[r]^-1 rhs[r] for a batch of SPD fp32 systems (f <= 64) on the GPU: one wave
    per system, Cholesky in registers (csrc/als.hip als_chol_solve_kernel); info[r] = 1
    marks a non-positive pivot."""
    m, f = rhs.shape
    assert A.shape == (m, f, f) and A.dtype == rhs.dtype == X.dtype == torch.float32 and f <= MAX_F
    assert X.shape == (m, f) and info.shape == (m,) and info.dtype == torch.int32
    for t in (A, rhs, X, info):
        assert t.is_contiguous() and t.device == A.device
    v = CHOL_VARIANT if variant is None else variant
    _lib.check(_lib.kernels().harp_als_chol_solve_f32(A.data_ptr(), rhs.data_ptr(), f, m, X.data_ptr(),
                                                      info.data_ptr(), v, _lib.stream_ptr(A.device)), "als_chol_solve")
