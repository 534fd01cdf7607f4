"""EM-GMM device ops (``csrc/gmm.hip``): fused E-step (Cholesky-whitened Mahalanobis +
log-sum-exp responsibilities) and the sufficient-statistics pass, fp64.

Reference: ml/daal/src/main/java/edu/iu/daal_em/BatchDense/EMDaalCollectiveMapper.java:146-156.
GPU tensors only (the PyTorch E-step in ``models.kernels`` is the CPU path and the oracle).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import torch

from . import _lib

_lib.register({
    "harp_gmm_estep_blocks": [_lib.c_long, _lib.c_int],  # returns int
    "harp_gmm_width": [_lib.c_int],
    "harp_gmm_aug_len": [_lib.c_int],
    "harp_gmm_aug_pad": [],
    # X, ldx, n, d, K, Paug, b, R, ldr, ll_part, stream
    "harp_gmm_estep": [_lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_void_p,
                       _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_void_p],
    "harp_gmm_coord_blocks": [_lib.c_int],
    # X, ldx, n, d, R, ldr, K, S, stream
    "harp_gmm_stats_blocks": [_lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_long,
                              _lib.c_int, _lib.c_void_p, _lib.c_void_p],
    # X, ldx, n, d, R, ldr, K, pair_i, pair_j, npairs, S, stream
    "harp_gmm_stats": [_lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_long, _lib.c_int,
                       _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
})

MAX_D = 64
# full-covariance statistics by 4 x 4 coordinate blocks from this width (below it the padded
# blocks waste more than the pair list's extra LDS reads cost: d = 8 1.40 vs 1.03 ms)
BLOCK_STATS_MIN_D = 16
_PAIRS: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}


def usable(X: torch.Tensor) -> bool:
    return X.device.type == "cuda" and X.dtype == torch.float64 and X.dim() == 2 and X.shape[1] <= MAX_D \
        and _lib.use_native(X)


_AUG: Dict[tuple, Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = {}


def _aug_index(D: int, device):
    """Positions of P_ij (j <= i) and of c_i in one component's augmented packed triangle
    (row i = [P_i0 .. P_ii, c_i], starting at i (i + 3) / 2)."""
    key = (D, str(device))
    t = _AUG.get(key)
    if t is None:
        r, c_ = torch.tril_indices(D, D)
        pos = r * (r + 3) // 2 + c_
        cpos = torch.arange(D) * (torch.arange(D) + 3) // 2 + torch.arange(D) + 1
        t = _AUG[key] = (r.to(device), c_.to(device), pos.to(device), cpos.to(device))
    return t


def whiten(w: torch.Tensor, mu: torch.Tensor, cov: torch.Tensor, covariance: str):
    """(Paug [K * A + pad]: per component the rows [P_i0 .. P_ii, c_i] of P = L^-1 and
    c = P mu, padded to the kernel's width D; b [K])."""
    K, d = mu.shape
    lib = _lib.kernels()
    D = int(lib.harp_gmm_width(d))
    A = int(lib.harp_gmm_aug_len(d))
    dev = mu.device
    if covariance == "full":
        L = torch.linalg.cholesky(cov)
        eye = torch.eye(d, dtype=torch.float64, device=dev).expand(K, d, d)
        Pm = torch.linalg.solve_triangular(L, eye, upper=False)
        logdet = 2 * torch.log(torch.diagonal(L, dim1=1, dim2=2)).sum(1)
    else:
        Pm = torch.diag_embed(cov.rsqrt())
        logdet = torch.log(cov).sum(1)
    Pp = torch.zeros((K, D, D), dtype=torch.float64, device=dev)
    Pp[:, :d, :d] = Pm
    cvec = torch.zeros((K, D), dtype=torch.float64, device=dev)
    cvec[:, :d] = torch.einsum("kij,kj->ki", Pm, mu)
    r, c_, pos, cpos = _aug_index(D, dev)
    Paug = torch.zeros(K * A + int(lib.harp_gmm_aug_pad()), dtype=torch.float64, device=dev)
    view = Paug[:K * A].view(K, A)
    view[:, pos] = Pp[:, r, c_]
    view[:, cpos] = cvec
    b = torch.log(w) - 0.5 * (logdet + d * math.log(2 * math.pi))
    return Paug, b.contiguous()


def estep(X: torch.Tensor, w: torch.Tensor, mu: torch.Tensor, cov: torch.Tensor, covariance: str = "full"):
    """Responsibilities R [n, K] (a transposed view of component-major storage) and the
    summed log-likelihood sum_n log sum_k w_k N(x_n | k)."""
    n, d = X.shape
    K = mu.shape[0]
    Paug, b = whiten(w, mu, cov, covariance)
    RT = torch.empty((K, n), dtype=torch.float64, device=X.device)  # component-major (coalesced writes)
    lib = _lib.kernels()
    part = torch.zeros(max(int(lib.harp_gmm_estep_blocks(n, d)), 1), dtype=torch.float64, device=X.device)
    st = lib.harp_gmm_estep(X.data_ptr(), X.stride(0), n, d, K, Paug.data_ptr(), b.data_ptr(),
                            RT.data_ptr(), RT.stride(0), part.data_ptr(), _lib.stream_ptr(X.device))
    _lib.check(st, "gmm_estep")
    return RT.t(), part.sum()


def _pairs(d: int, covariance: str, device) -> Tuple[torch.Tensor, torch.Tensor]:
    key = (d, covariance, str(device))
    p = _PAIRS.get(key)
    if p is None:
        if covariance == "full":  # the upper triangle of x' x'^T, x' = [x, 1]
            ij = [(i, j) for i in range(d + 1) for j in range(i, d + 1)]
        else:  # x_i^2, x_i (paired with the ones column), and the count
            ij = [(i, i) for i in range(d)] + [(i, d) for i in range(d)] + [(d, d)]
        t = torch.tensor(ij, dtype=torch.int32)
        p = _PAIRS[key] = (t[:, 0].contiguous().to(device), t[:, 1].contiguous().to(device))
    return p


def stats(X: torch.Tensor, R: torch.Tensor, covariance: str = "full"):
    """(N_k [K], S1 = sum r x [K, d], S2 = sum r x x^T [K, d, d] (full) or sum r x^2 [K, d]) in one pass."""
    n, d = X.shape
    K = R.shape[1]
    RT = R.t() if (R.stride(0) == 1 and R.t().is_contiguous()) else R.t().contiguous()  # component-major
    lib = _lib.kernels()
    if covariance == "full" and d >= BLOCK_STATS_MIN_D:
        # 4 x 4 coordinate blocks of x' x'^T (upper block triangle), then unpacked
        nbk = int(lib.harp_gmm_coord_blocks(d))
        npb = nbk * (nbk + 1) // 2
        Sb = torch.zeros((K, npb, 16), dtype=torch.float64, device=X.device)
        st = lib.harp_gmm_stats_blocks(X.data_ptr(), X.stride(0), n, d, RT.data_ptr(), RT.stride(0), K,
                                       Sb.data_ptr(), _lib.stream_ptr(X.device))
        _lib.check(st, "gmm_stats_blocks")
        bi, bj = torch.triu_indices(nbk, nbk, device=X.device)
        M = torch.zeros((K, nbk, nbk, 4, 4), dtype=torch.float64, device=X.device)
        blocks = Sb.view(K, npb, 4, 4)
        M[:, bj, bi] = blocks.transpose(2, 3)  # the lower block triangle mirrors the upper
        M[:, bi, bj] = blocks
        M = M.permute(0, 1, 3, 2, 4).reshape(K, 4 * nbk, 4 * nbk)[:, :d + 1, :d + 1]
        return M[:, d, d].contiguous(), M[:, :d, d].contiguous(), M[:, :d, :d].contiguous()
    pi, pj = _pairs(d, covariance, X.device)
    npairs = pi.numel()
    S = torch.zeros((K, npairs), dtype=torch.float64, device=X.device)
    st = _lib.kernels().harp_gmm_stats(X.data_ptr(), X.stride(0), n, d, RT.data_ptr(), RT.stride(0), K,
                                       pi.data_ptr(), pj.data_ptr(), npairs, S.data_ptr(), _lib.stream_ptr(X.device))
    _lib.check(st, "gmm_stats")
    if covariance == "full":
        iu = torch.triu_indices(d + 1, d + 1, device=X.device)
        M = torch.zeros((K, d + 1, d + 1), dtype=torch.float64, device=X.device)
        M[:, iu[0], iu[1]] = S
        M = M + torch.triu(M, 1).transpose(1, 2)
        return M[:, d, d], M[:, :d, d].contiguous(), M[:, :d, :d].contiguous()
    return S[:, 2 * d], S[:, d:2 * d].contiguous(), S[:, :d].contiguous()
