"""One-vs-rest logistic-regression SGD pass (``csrc/mlr.hip``): one launch per pass over
the local CSR shard, one workgroup per topic chain. Reference: contrib/.../mlr/GDtask.java:30-72."""
from __future__ import annotations

import os

import torch

from . import _lib

_lib.register({
    "harp_mlr_sgd_pass": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_long,
                          _lib.c_void_p, _lib.c_int, _lib.c_long, _lib.c_double, _lib.c_int, _lib.c_int, _lib.c_void_p],
})

# workgroup size: the topic chains are few (T/P workgroups), so wider groups split a
# batch's rows over more waves; but every batch ends in a barrier, so a small batch wants a
# small group. Measured (profiles/r1_mlr/): batch 64 -> 512 threads (15.8 ms vs 20.0 at
# 256, 17.6 at 1024); batch 1 -> 256 beat 512 / 1024 by 1.7x / 3.1x. Rule: one wave per 8
# batch rows, 1..16 waves. HARP_MLR_THREADS overrides.
_THREADS_ENV = os.environ.get("HARP_MLR_THREADS")


def threads_for(batch: int) -> int:
    if _THREADS_ENV:
        return int(_THREADS_ENV)
    return 64 * max(1, min(16, batch // 8))


def sgd_pass(W: torch.Tensor, crow: torch.Tensor, col: torch.Tensor, val: torch.Tensor, n: int, Y: torch.Tensor,
             alpha: float, batch: int) -> None:
    """W [T, D+1] fp64 (bias column 0) updated in place; Y [n, >= T] labels (any float
    view with unit column stride); crow int64, col int32, val fp64 on W's device."""
    assert W.dtype == torch.float64 and W.stride(1) == 1 and crow.dtype == torch.int64
    assert col.dtype == torch.int32 and val.dtype == torch.float64 and crow.numel() == n + 1
    Yf = Y if (Y.dtype == torch.float32 and Y.stride(1) == 1) else Y.to(torch.float32).contiguous()
    assert Yf.shape[0] == n and Yf.shape[1] >= W.shape[0]
    st = _lib.kernels().harp_mlr_sgd_pass(crow.data_ptr(), col.data_ptr(), val.data_ptr(), n, Yf.data_ptr(),
                                          Yf.stride(0), W.data_ptr(), W.shape[0], W.stride(0), float(alpha), batch,
                                          threads_for(batch), _lib.stream_ptr(W.device))
    _lib.check(st, "mlr_sgd_pass")
