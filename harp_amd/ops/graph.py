"""Color-coding DP ops (``csrc/graph.hip``): CSR neighbour sums and color-set combines in
fp64, with torch fallbacks for the CPU."""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache
from typing import Tuple

import torch

from . import _lib

_lib.register({
    "harp_csr_spmm_f64": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_long,
                          _lib.c_void_p],
    "harp_colorset_combine_f64": [_lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p,
                                  _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_long, _lib.c_void_p],
})


@dataclass
class CSR:
    rowptr: torch.Tensor  # [n + 1] int64
    col: torch.Tensor     # [nnz] int32 (row index into the neighbour table)
    n: int


def build_csr(rows: torch.Tensor, cols: torch.Tensor, n: int) -> CSR:
    """CSR of the (row, col) pairs (rows in [0, n)); neighbour order within a row is the
    input order (stable sort)."""
    order = torch.sort(rows.long(), stable=True).indices
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=rows.device)
    rowptr[1:] = torch.cumsum(torch.bincount(rows.long(), minlength=n)[:n], 0)
    return CSR(rowptr, cols[order].to(torch.int32).contiguous(), n)


def spmm(csr: CSR, M: torch.Tensor) -> torch.Tensor:
    """out[v] = sum of M[col[j]] over v's CSR row (fp64, M [*, C] with C <= 64)."""
    assert M.dtype == torch.float64 and M.is_contiguous()
    C = M.shape[1]
    out = torch.empty((csr.n, C), dtype=torch.float64, device=M.device)
    if _lib.use_native(M) and C <= 64:
        st = _lib.kernels().harp_csr_spmm_f64(csr.rowptr.data_ptr(), csr.col.data_ptr(), M.data_ptr(), C,
                                               out.data_ptr(), csr.n, _lib.stream_ptr(M.device))
        _lib.check(st, "csr_spmm_f64")
        return out
    rows = torch.repeat_interleave(torch.arange(csr.n, device=M.device), csr.rowptr[1:] - csr.rowptr[:-1])
    out.zero_()
    out.index_add_(0, rows, M[csr.col.long()])
    return out


@lru_cache(maxsize=None)
def _split_tables(key: Tuple, device_str: str):
    tc, t1, t2, co = key
    dev = torch.device(device_str)
    tc_t = torch.tensor(tc, dtype=torch.int64)
    toff = torch.zeros(co + 1, dtype=torch.int64)
    toff[1:] = torch.cumsum(torch.bincount(tc_t, minlength=co), 0)
    return (toff.to(torch.int32).to(dev), torch.tensor(t1, dtype=torch.int32, device=dev),
            torch.tensor(t2, dtype=torch.int32, device=dev))


def combine(A: torch.Tensor, N: torch.Tensor, tc: torch.Tensor, t1: torch.Tensor, t2: torch.Tensor,
            co: int) -> torch.Tensor:
    """out[v, c] = sum over splits t with tc[t] == c of A[v, t1[t]] * N[v, t2[t]] (tc sorted)."""
    n = A.shape[0]
    out = torch.empty((n, co), dtype=torch.float64, device=A.device)
    if _lib.use_native(A):
        assert A.is_contiguous() and N.is_contiguous()
        key = (tuple(tc.tolist()), tuple(t1.tolist()), tuple(t2.tolist()), co)
        toff, d1, d2 = _split_tables(key, str(A.device))
        st = _lib.kernels().harp_colorset_combine_f64(A.data_ptr(), A.shape[1], N.data_ptr(), N.shape[1],
                                                       toff.data_ptr(), d1.data_ptr(), d2.data_ptr(), co, t1.numel(),
                                                       out.data_ptr(), n, _lib.stream_ptr(A.device))
        _lib.check(st, "colorset_combine_f64")
        return out
    out.zero_()
    tc, t1, t2 = tc.to(A.device), t1.to(A.device), t2.to(A.device)
    step = max(1, (1 << 24) // max(1, tc.numel()))
    for a in range(0, n, step):
        b = min(n, a + step)
        out[a:b].index_add_(1, tc, A[a:b, t1] * N[a:b, t2])
    return out
