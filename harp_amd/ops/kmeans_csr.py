"""Sparse K-means E-step + accumulate (``csrc/kmeans_csr.hip``), fp64.

One launch per iteration replaces the torch path of ``models/kmeans_csr.py`` (sparse-dense
product, [n, K] distance tensor, one-hot, second SpMM for the sums). Reference:
ml/daal/.../daal_kmeans/allreducecsr/KMeansDaalCollectiveMapper.java (DAAL kmeans
DistributedStep1Local on CSR input).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch

from . import _lib

_lib.register({
    "harp_kmeans_csr_assign": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p,
                               _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                               _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
})


@dataclass
class DeviceCSR:
    rowptr: torch.Tensor  # int64 [n + 1]
    col: torch.Tensor     # int32 [nnz]
    val: torch.Tensor     # fp64 [nnz]
    xn: torch.Tensor      # fp64 [n] squared row norms
    n: int
    d: int


def to_device_csr(X: torch.Tensor) -> DeviceCSR:
    """Kernel operands of a sparse (COO or CSR) matrix on a HIP device (built once)."""
    Xc = X if X.layout == torch.sparse_csr else X.coalesce().to_sparse_csr()
    val = Xc.values().double().contiguous()
    rowptr = Xc.crow_indices().long().contiguous()
    n, d = X.shape
    xn = torch.zeros(n, dtype=torch.float64, device=X.device)
    counts = rowptr[1:] - rowptr[:-1]
    xn.index_add_(0, torch.repeat_interleave(torch.arange(n, device=X.device), counts), val * val)
    return DeviceCSR(rowptr, Xc.col_indices().to(torch.int32).contiguous(), val, xn, n, d)


def assign_accumulate(A: DeviceCSR, C: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """(labels int64 [n], squared distance to the nearest centroid [n], sums [K, d],
    counts [K]) for fp64 centroids C [K, d] on the device of A."""
    K, d = C.shape
    assert d == A.d and C.dtype == torch.float64 and C.device == A.val.device
    lib = _lib.kernels()
    Kp = (K + 63) // 64 * 64
    CT = torch.zeros((d, Kp), dtype=torch.float64, device=C.device)
    CT[:, :K] = C.t()
    cn = (C * C).sum(1).contiguous()
    labels = torch.empty(A.n, dtype=torch.int32, device=C.device)
    mind = torch.empty(A.n, dtype=torch.float64, device=C.device)
    sums = torch.zeros((K, d), dtype=torch.float64, device=C.device)
    counts = torch.zeros(K, dtype=torch.float64, device=C.device)
    st = lib.harp_kmeans_csr_assign(A.rowptr.data_ptr(), A.col.data_ptr(), A.val.data_ptr(), A.n, d, CT.data_ptr(),
                                    K, Kp, cn.data_ptr(), A.xn.data_ptr(), labels.data_ptr(), mind.data_ptr(),
                                    sums.data_ptr(), counts.data_ptr(), _lib.stream_ptr(C.device))
    _lib.check(st, "kmeans_csr_assign")
    return labels.long(), mind, sums, counts
