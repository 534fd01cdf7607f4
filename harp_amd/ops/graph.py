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
    "harp_pagerank_pull_f64": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_double, _lib.c_double,
                               _lib.c_double, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                               _lib.c_long, _lib.c_long, _lib.c_void_p],
    "harp_colorset_combine_f64": [_lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p,
                                  _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_long, _lib.c_void_p],
})


@dataclass
class CSR:
    rowptr: torch.Tensor  # [n + 1] int64
    col: torch.Tensor     # [nnz] int32 (row index into the neighbour table)
    n: int


SORT_CHUNK = 1 << 30  # torch sorts at most INT_MAX elements per call


def build_csr(rows: torch.Tensor, cols: torch.Tensor, n: int) -> CSR:
    """CSR of the (row, col) pairs (rows in [0, n)); neighbour order within a row is the
    input order (stable sort). Past 2^30 pairs (a Twitter-size graph has 2.4e9 directed
    edges) the pairs are stable-sorted in input-order chunks and each chunk's row segments
    are placed after the earlier chunks' segments of the same row: the same result."""
    rows = rows.long()
    dev = rows.device
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    E = rows.numel()
    if E <= SORT_CHUNK:
        order = torch.sort(rows, stable=True).indices
        rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n)[:n], 0)
        return CSR(rowptr, cols[order].to(torch.int32).contiguous(), n)
    bounds = list(range(0, E, SORT_CHUNK)) + [E]
    counts = [torch.bincount(rows[a:b], minlength=n)[:n] for a, b in zip(bounds[:-1], bounds[1:])]
    rowptr[1:] = torch.cumsum(torch.stack(counts).sum(0), 0)
    col = torch.empty(E, dtype=torch.int32, device=dev)
    before = torch.zeros(n, dtype=torch.int64, device=dev)  # this row's pairs in earlier chunks
    for (a, b), cnt in zip(zip(bounds[:-1], bounds[1:]), counts):
        r_sorted, order = torch.sort(rows[a:b], stable=True)
        seg = torch.cumsum(cnt, 0) - cnt  # each row's first position in the sorted chunk
        rank = torch.arange(b - a, device=dev) - seg[r_sorted]
        col[rowptr[r_sorted] + before[r_sorted] + rank] = cols[a:b][order].to(torch.int32)
        before += cnt
        del r_sorted, order, rank
    return CSR(rowptr, col, n)


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


def pagerank_pull(csr: CSR, x: torch.Tensor, alpha: float, b0: float, b1: float, dm: torch.Tensor = None,
                  invdeg: torch.Tensor = None, want_xnext: bool = False):
    """One PageRank pull step over a by-target CSR (``csrc/graph.hip`` pagerank_pull_kernel):
    ``out[v] = alpha * sum_{u in in(v)} x[u] + b0 + b1 * dm`` (``dm`` a 1-element device
    tensor, read on the device: no host sync), and with ``want_xnext`` also
    ``xnext[v] = out[v] * invdeg[v]`` for v < len(invdeg). Returns (out, xnext or None)."""
    assert x.dtype == torch.float64 and x.is_contiguous()
    n = csr.n
    out = torch.empty(n, dtype=torch.float64, device=x.device)
    xnext = torch.empty(invdeg.numel(), dtype=torch.float64, device=x.device) if want_xnext else None
    if _lib.use_native(x):
        assert dm is None or (dm.dtype == torch.float64 and dm.device == x.device)
        assert not want_xnext or (invdeg.dtype == torch.float64 and invdeg.is_contiguous() and invdeg.numel() <= n)
        assert csr.col.numel() == 0 or int(csr.rowptr[-1]) == csr.col.numel()
        st = _lib.kernels().harp_pagerank_pull_f64(
            csr.rowptr.data_ptr(), csr.col.data_ptr(), x.data_ptr(), float(alpha), float(b0), float(b1),
            dm.data_ptr() if dm is not None else None, out.data_ptr(),
            invdeg.data_ptr() if want_xnext else None, xnext.data_ptr() if want_xnext else None,
            invdeg.numel() if want_xnext else 0, n, csr.col.numel(), _lib.stream_ptr(x.device))
        _lib.check(st, "pagerank_pull_f64")
        return out, xnext
    rows = torch.repeat_interleave(torch.arange(n, device=x.device), csr.rowptr[1:] - csr.rowptr[:-1])
    out.zero_()
    out.index_add_(0, rows, x[csr.col.long()])
    out.mul_(alpha).add_(b0)
    if dm is not None:
        out.add_(b1 * dm)
    if want_xnext:
        xnext.copy_(out[:invdeg.numel()] * invdeg)
    return out, xnext


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
