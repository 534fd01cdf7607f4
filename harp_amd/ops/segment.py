"""Label bucketing (counting sort) and per-bucket row sums on the GPU.

``bucket_labels(labels, K)`` -> (perm, start): indices grouped by label, bucket offsets.
``bucket_rowsum(X, perm, start, out)``: out[k] = sum of bf16 rows X[perm[start[k]:start[k+1]]].
See csrc/segsum.hip for why this beats float atomics on gfx950.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Tuple

import torch

from . import _lib

_lib.register({
    "harp_bucket_chunk": [_lib.c_long],
    "harp_bucket_workspace_ints": [_lib.c_long, _lib.c_int],
    "harp_bucket_labels": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                           _lib.c_void_p],
    "harp_bucket_rowsum_bf16": [_lib.c_void_p, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                                _lib.c_long, _lib.c_void_p, _lib.c_int, _lib.c_void_p],
})
_WS: Dict[Tuple, torch.Tensor] = {}


def _lib_ret_long(fn):
    fn.restype = ctypes.c_long
    return fn


def bucket_labels(labels: torch.Tensor, K: int) -> Tuple[torch.Tensor, torch.Tensor]:
    n = labels.numel()
    if not _lib.use_native(labels):
        order = torch.argsort(labels.long(), stable=True)
        counts = torch.bincount(labels.long(), minlength=K)
        start = torch.zeros(K + 1, dtype=torch.int64)
        start[1:] = torch.cumsum(counts, 0)
        return order.to(torch.int32), start.to(torch.int32)
    lib = _lib.kernels()
    _lib_ret_long(lib.harp_bucket_workspace_ints)
    need = lib.harp_bucket_workspace_ints(n, K)
    stream = torch.cuda.current_stream(labels.device).cuda_stream
    key = (labels.device, n, K, stream)
    ws = _WS.get(key)
    if ws is None:
        for k in [k for k in _WS if k[3] == stream]:
            del _WS[k]  # one workspace alive per stream (allocated and reused on that stream)
        ws = torch.empty(need, dtype=torch.int32, device=labels.device)
        _WS[key] = ws
    so, po = ctypes.c_long(0), ctypes.c_long(0)
    st = lib.harp_bucket_labels(labels.data_ptr(), n, K, ws.data_ptr(), ctypes.byref(so), ctypes.byref(po),
                                _lib.stream_ptr(labels.device))
    _lib.check(st, "bucket_labels")
    return ws[po.value:po.value + n], ws[so.value:so.value + K + 1]


# 256: the per-slice form before round 4. The kernel takes multiples of 8 in [8, 1024]
SUM_SLICE = min(1024, max(8, int(os.environ.get("HARP_ROWSUM_SLICE", "1024")) // 8 * 8))


def bucket_rowsum(X: torch.Tensor, perm: torch.Tensor, start: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[k] += sum of the bucket's rows (zero ``out`` first for a plain sum)."""
    K = start.numel() - 1
    if not _lib.use_native(X):
        idx = torch.repeat_interleave(torch.arange(K), (start[1:] - start[:-1]).long())
        out[:K, : X.shape[1]].index_add_(0, idx, X[perm.long()].float())
        return out
    assert X.dtype == torch.bfloat16 and X.stride(1) == 1 and out.dtype == torch.float32 and out.is_contiguous()
    # the kernel sums rows of up to SUM_SLICE columns in one pass (one wave per slot past 256
    # columns); wider rows go as slices
    for c0 in range(0, X.shape[1], SUM_SLICE):
        w = min(SUM_SLICE, X.shape[1] - c0)
        st = _lib.kernels().harp_bucket_rowsum_bf16(X[:, c0:].data_ptr(), w, X.stride(0), perm.data_ptr(),
                                                    start.data_ptr(), K, perm.numel(), out[:, c0:].data_ptr(),
                                                    out.stride(0), _lib.stream_ptr(X.device))
        _lib.check(st, "bucket_rowsum")
    return out
