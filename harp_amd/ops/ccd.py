"""MF-CCD device ops (``csrc/ccd.hip``) with the vectorised torch formulation as the CPU
path / numerics oracle (the same per-row, per-dimension update order)."""
from __future__ import annotations

import torch

from . import _lib

_lib.register({
    "harp_ccd_phase": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                       _lib.c_float, _lib.c_int, _lib.c_void_p],
    "harp_ccd_lockstep": [_lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                          _lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_float, _lib.c_void_p,
                          _lib.c_void_p, _lib.c_void_p],
    "harp_ccd_block_max": [_lib.c_int],
    "harp_ccd_block": [_lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                       _lib.c_void_p, _lib.c_int, _lib.c_float, _lib.c_int, _lib.c_void_p],
    "harp_ccd_residual": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_void_p,
                          _lib.c_int, _lib.c_void_p, _lib.c_void_p],
})


def row_ptr_of(rows: torch.Tensor, n_rows: int) -> torch.Tensor:
    """CSR offsets of row-sorted nonzeros."""
    ptr = torch.zeros(n_rows + 1, dtype=torch.int64, device=rows.device)
    ptr[1:] = torch.cumsum(torch.bincount(rows.long(), minlength=n_rows), 0)
    return ptr


LONG_ROW = 256  # rows above this many nonzeros leave the wave-per-row kernel
CHUNK = 4096


def block_max(wide: bool = False) -> int:
    """Longest row of the workgroup-per-row kernel (csrc/ccd.hip ccd_block_kernel: 8192
    nonzeros, ``wide`` 12288); longer rows run the lockstep (chunked, per-dimension) path.
    0 without a GPU library."""
    try:
        return int(_lib.kernels().harp_ccd_block_max(1 if wide else 0))
    except _lib.NativeUnavailable:
        return 0


class RowPlan:
    """Per-phase launch plan: rows of LONG_ROW < n <= block_max() nonzeros (one workgroup
    each; ``mid``), rows up to block_max(wide=True) (``wide``), and the chunks of every
    longer row (lockstep)."""

    def __init__(self, row_ptr: torch.Tensor, block_rows: bool = True):
        lens = (row_ptr[1:] - row_ptr[:-1]).cpu()
        rp = row_ptr.cpu()
        bmax = block_max() if (block_rows and row_ptr.is_cuda) else 0
        wmax = block_max(True) if bmax else 0
        pick = lambda lo, hi: torch.nonzero((lens > lo) & (lens <= hi)).reshape(-1).to(torch.int32).to(row_ptr.device)
        self.mid = pick(LONG_ROW, bmax)
        self.wide = pick(max(LONG_ROW, bmax), wmax)
        longr = torch.nonzero(lens > max(LONG_ROW, wmax)).reshape(-1)
        self.n_long = longr.numel()
        ch = []
        for slot, r in enumerate(longr.tolist()):
            a, b = int(rp[r]), int(rp[r + 1])
            for s in range(a, b, CHUNK):
                ch.append((r, s, min(b, s + CHUNK), slot))
        self.chunks = torch.tensor(ch, dtype=torch.int64).reshape(-1, 4).to(row_ptr.device)
        self.acc = torch.zeros((max(1, self.n_long), 6), dtype=torch.float32, device=row_ptr.device)


def long_rows_of(row_ptr: torch.Tensor) -> "RowPlan":
    return RowPlan(row_ptr)


def phase(rows: torch.Tensor, row_ptr: torch.Tensor, cols: torch.Tensor, res: torch.Tensor, F_own: torch.Tensor,
          F_other: torch.Tensor, lam: float, long_rows: torch.Tensor = None) -> None:
    """Coordinate updates of every row of ``F_own`` (nonzeros sorted by row, residuals
    ``res`` in the same order) against the fixed ``F_other``; updates res in place."""
    n_rows, k = F_own.shape
    if _lib.use_native(res):
        assert res.dtype == torch.float32 and F_own.dtype == torch.float32 and F_other.dtype == torch.float32
        assert F_own.is_contiguous() and F_other.is_contiguous() and cols.dtype == torch.int32
        plan = long_rows if isinstance(long_rows, RowPlan) else RowPlan(row_ptr)
        lib = _lib.kernels()
        stream = _lib.stream_ptr(res.device)
        st = lib.harp_ccd_phase(row_ptr.data_ptr(), cols.data_ptr(), res.data_ptr(), n_rows, F_own.data_ptr(),
                                F_other.data_ptr(), k, float(lam),
                                1 if (plan.n_long or plan.mid.numel() or plan.wide.numel()) else 0, stream)
        _lib.check(st, "ccd_phase")
        for wide, lst in ((0, plan.mid), (1, plan.wide)):
            if lst.numel():
                st = lib.harp_ccd_block(lst.data_ptr(), lst.numel(), row_ptr.data_ptr(), cols.data_ptr(),
                                        res.data_ptr(), F_own.data_ptr(), F_other.data_ptr(), k, float(lam), wide,
                                        stream)
                _lib.check(st, "ccd_block")
        if plan.n_long:
            FxT = F_other.t().contiguous()  # feature-major: one dimension = one L2-resident column
            if getattr(plan, "hbuf", None) is None or plan.hbuf.numel() != res.numel():
                plan.hbuf = torch.empty_like(res)
            plan.acc.zero_()
            for t in range(k + 2):
                st = lib.harp_ccd_lockstep(plan.chunks.data_ptr(), plan.chunks.shape[0], row_ptr.data_ptr(),
                                           cols.data_ptr(), res.data_ptr(), F_own.data_ptr(), FxT.data_ptr(),
                                           FxT.stride(0), k, t, float(lam), plan.acc.data_ptr(), plan.hbuf.data_ptr(),
                                           stream)
                _lib.check(st, "ccd_lockstep")
        return
    cnt = (row_ptr[1:] - row_ptr[:-1]).to(res.dtype)
    rl, cl = rows.long(), cols.long()
    down0 = lam * cnt
    for t in range(k):
        h = F_other[cl, t]
        w = F_own[rl, t]
        up = torch.zeros(n_rows, dtype=res.dtype, device=res.device)
        down = down0.clone()
        up.index_add_(0, rl, (res + w * h) * h)
        down.index_add_(0, rl, h * h)
        z = torch.where(down > 0, up / down.clamp_min(1e-300), F_own[:, t])
        delta = z - F_own[:, t]
        res -= delta[rl] * h
        F_own[:, t] = z


def residual(rows: torch.Tensor, cols: torch.Tensor, val: torch.Tensor, F_rows: torch.Tensor,
             F_cols: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """res_j = val_j - <F_rows[rows_j], F_cols[cols_j]> (ResTask)."""
    if out is None:
        out = torch.empty_like(val)
    if _lib.use_native(val):
        st = _lib.kernels().harp_ccd_residual(rows.data_ptr(), cols.data_ptr(), val.data_ptr(), val.numel(),
                                              F_rows.data_ptr(), F_cols.data_ptr(), F_rows.shape[1], out.data_ptr(),
                                              _lib.stream_ptr(val.device))
        _lib.check(st, "ccd_residual")
        return out
    step = 1 << 20
    for a in range(0, val.numel(), step):
        b = min(val.numel(), a + step)
        out[a:b] = val[a:b] - (F_rows[rows[a:b].long()] * F_cols[cols[a:b].long()]).sum(1)
    return out
