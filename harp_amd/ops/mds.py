"""WDA-MDS row-block kernels (``csrc/mds.hip``): B(Z) X and the weighted stress of the
local rows in one fp64 pass over the delta / weight blocks. Reference:
ml/java/.../wdamds/BCCalcTask.java:97-170, StressCalcTask.java:72-96."""
from __future__ import annotations

import torch

from . import _lib

_lib.register({
    "harp_mds_rows": [_lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_int, _lib.c_void_p,
                      _lib.c_int, _lib.c_double, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
})

MAX_DIM = 4


def _run(D: torch.Tensor, W: torch.Tensor, row0: int, X: torch.Tensor, diff: float, stress: bool) -> torch.Tensor:
    n_r, n = D.shape
    dim = X.shape[1]
    assert D.dtype == W.dtype == X.dtype == torch.float64 and D.stride() == W.stride() and D.stride(1) == 1
    assert X.shape[0] == n and 1 <= dim <= MAX_DIM
    Xc = X.contiguous()
    out = torch.empty((n_r,) if stress else (n_r, dim), dtype=torch.float64, device=D.device)
    st = _lib.kernels().harp_mds_rows(D.data_ptr(), W.data_ptr(), D.stride(0), n_r, n, row0, Xc.data_ptr(), dim,
                                      float(diff), 1 if stress else 0, out.data_ptr(), _lib.stream_ptr(D.device))
    _lib.check(st, "mds_rows")
    return out


def bc_rows(D, W, row0, X, diff):
    """(B(Z) X) for the local rows [n_r, dim]."""
    return _run(D, W, row0, X, diff, False)


def stress_rows(D, W, row0, X, diff):
    """Per-row weighted stress sums [n_r]."""
    return _run(D, W, row0, X, diff, True)
