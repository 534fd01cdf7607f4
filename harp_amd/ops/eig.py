"""Symmetric eigenvalues on one XCD (``csrc/eig.hip``): cooperative Householder
tridiagonalisation + multisection, for the PCA pass's d x d fp64 correlation matrix.

Reference: the DAAL PCA correlation step 3 (eigen-decomposition on the master),
ml/daal/src/main/java/edu/iu/daal_pca/cordensedistr/PCADaalCollectiveMapper.java:121-147.
"""
from __future__ import annotations

import os
import warnings

import torch

from . import _lib

_lib.register({
    "harp_eig_ws_ints": [],
    "harp_eig_max_n": [],
    "harp_eig_workgroups": [_lib.c_int, _lib.c_int],
    # A, lda, n, d, e, w, nb_max, ws, wsd, stamps, stream
    "harp_eig_sym": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                     _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    # A, lda, n, d, e, w, nb_max, ws, wsd, stream
    "harp_eig_sym_fused": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                           _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
})

NB_DEFAULT = 32  # workgroups (CUs) of XCD 0
# reduction form: "fused" (one pass over the trailing block and one arrival per column,
# look-ahead Householder vector) or "twopass" (matrix-vector pass + rank-2 update pass)
VARIANT = os.environ.get("HARP_EIG_VARIANT", "fused")


def usable(C: torch.Tensor) -> bool:
    return (C.device.type == "cuda" and C.dtype == torch.float64 and C.dim() == 2 and C.shape[0] == C.shape[1]
            and _lib.use_native(C) and 0 < C.shape[0] <= int(_lib.kernels().harp_eig_max_n()))


def eigvalsh(C: torch.Tensor, stamps: torch.Tensor | None = None) -> torch.Tensor:
    """Ascending eigenvalues of the symmetric matrix ``C`` (fp64 on a GPU: the one-XCD
    kernels; otherwise, or if the cooperative launch could not claim its workgroups,
    torch.linalg.eigvalsh)."""
    if not usable(C):
        return torch.linalg.eigvalsh(C)
    n = C.shape[0]
    dev = C.device
    k = _lib.kernels()
    nb_max = int(os.environ.get("HARP_EIG_NB", NB_DEFAULT))
    nb = int(k.harp_eig_workgroups(n, nb_max))
    if nb < 1:
        return torch.linalg.eigvalsh(C)
    A = C.contiguous().clone()  # symmetric: row-major storage is the column-major matrix
    ws = torch.zeros(int(k.harp_eig_ws_ints()), dtype=torch.int32, device=dev)
    wsd = torch.zeros(3 * n + 4, dtype=torch.float64, device=dev)
    d = torch.empty(n, dtype=torch.float64, device=dev)
    e = torch.empty(n, dtype=torch.float64, device=dev)
    w = torch.empty(n, dtype=torch.float64, device=dev)
    if VARIANT == "fused" and stamps is None:
        st = k.harp_eig_sym_fused(A.data_ptr(), n, n, d.data_ptr(), e.data_ptr(), w.data_ptr(), nb, ws.data_ptr(),
                                  wsd.data_ptr(), _lib.stream_ptr(dev))
    else:
        st = k.harp_eig_sym(A.data_ptr(), n, n, d.data_ptr(), e.data_ptr(), w.data_ptr(), nb_max, ws.data_ptr(),
                            wsd.data_ptr(), _lib.ptr(stamps), _lib.stream_ptr(dev))
    _lib.check(st, "eig_sym")
    claims, _, err = ws[:3].tolist()
    if claims < nb or err:
        warnings.warn(f"one-XCD eigensolver did not run cooperatively (claims {claims}/{nb}, error {err}); "
                      "using torch.linalg.eigvalsh")
        return torch.linalg.eigvalsh(C)
    return w
