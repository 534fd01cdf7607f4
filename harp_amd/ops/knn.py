"""Exact k-nearest-neighbour search (``csrc/knn.hip``): library GEMM for Q T^T, then one
fused distance + top-k selection pass per (query tile, train tile) that merges into a
running [M, k] state. The CPU path (and the fp32 oracle of the GPU test) is the plain
torch expression: full distance tile + ``torch.topk``.

Reference hot loop: DAAL ``kdtree_knn_classification`` prediction
(ml/daal/.../daal_knn/KnnDaalCollectiveMapper.java, SURVEY §2.9 "kNN distance GEMM +
top-k").
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib

_lib.register({
    "harp_knn_select": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                        _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
})

MAX_NATIVE_K = 32  # lane lists of 64 spill VGPRs; larger k takes the torch path


def _torch_search(train, queries, k, tile):
    tn = (train * train).sum(1)
    ds, ix = [], []
    for a in range(0, queries.shape[0], tile):
        Q = queries[a:a + tile]
        D = ((Q * Q).sum(1)[:, None] + tn[None, :] - 2 * (Q @ train.t())).clamp_min(0)
        d, i = torch.topk(D, k, dim=1, largest=False)
        ds.append(d), ix.append(i)
    return torch.cat(ds), torch.cat(ix)


def knn_search(train: torch.Tensor, queries: torch.Tensor, k: int, q_tile: int = 8192,
               t_tile: int = 1 << 16) -> Tuple[torch.Tensor, torch.Tensor]:
    """(squared distances [M, k] ascending, int64 train indices [M, k]) of the k nearest
    training rows of every query. HIP tensors: fp32 only, k <= 32 (native path is
    mandatory; other dtypes / larger k raise). Ties resolve to the lower train index."""
    n = train.shape[0]
    k = min(k, n)
    if not _lib.use_native(queries):
        return _torch_search(train, queries, k, q_tile)
    if train.dtype != torch.float32 or queries.dtype != torch.float32:
        raise TypeError("native kNN takes fp32 train/query rows")
    if k > MAX_NATIVE_K:
        raise ValueError(f"native kNN supports k <= {MAX_NATIVE_K} (got {k})")
    train = train.contiguous()
    queries = queries.contiguous()
    M = queries.shape[0]
    tn = (train * train).sum(1)
    qn = (queries * queries).sum(1)
    outD = torch.empty((M, k), dtype=torch.float32, device=queries.device)
    outI = torch.empty((M, k), dtype=torch.int32, device=queries.device)
    lib = _lib.kernels()
    stream = _lib.stream_ptr(queries.device)
    for a in range(0, M, q_tile):
        Q = queries[a:a + q_tile]
        m = Q.shape[0]
        for b in range(0, n, t_tile):
            T = train[b:b + t_tile]
            S = Q @ T.t()  # hipBLASLt fp32 GEMM, [m, nt] contiguous
            st = lib.harp_knn_select(S.data_ptr(), S.shape[1], m, T.shape[0], qn[a:].data_ptr(), tn[b:].data_ptr(),
                                     k, b, 1 if b > 0 else 0, outD[a:].data_ptr(), outI[a:].data_ptr(), stream)
            _lib.check(st, "knn_select")
    return outD, outI.long()
