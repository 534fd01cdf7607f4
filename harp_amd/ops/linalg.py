"""Dense linear-algebra device ops for the partial-result family.

``gram(X)`` = X^T X and ``colsum(X)`` — the step-1 partials of covariance / moments /
PCA / normal-equation regressions (DAAL ``DistributedStep1Local``). On the GPU, bf16 and
fp32 inputs go to the hand-written MFMA SYRK kernel in ``csrc/syrk.hip`` (upper-triangle
tiles only, fp32 accumulation, column sums fused); fp64 and sparse inputs use torch
(rocBLAS / rocSPARSE) — plain library GEMMs.
"""
from __future__ import annotations

import os

import torch

from . import _lib


def _is_sparse(X: torch.Tensor) -> bool:
    return X.is_sparse or X.layout in (torch.sparse_csr, torch.sparse_csc)


def colsum(X: torch.Tensor) -> torch.Tensor:
    if _is_sparse(X):
        Xc = X.to_sparse_coo().coalesce()
        out = torch.zeros(X.shape[1], dtype=torch.float64, device=X.device)
        return out.index_add_(0, Xc.indices()[1], Xc.values().double())
    acc = torch.float64 if X.device.type == "cpu" else torch.float32
    return X.to(acc).sum(0)


def gram(X: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """X^T X (fp64 on CPU, fp32 accumulation on the GPU)."""
    if _is_sparse(X):
        Xc = X.to_sparse_csr().to(torch.float64 if X.device.type == "cpu" else torch.float32)
        G = (Xc.t() @ Xc.to_dense()) if X.device.type != "cpu" else (Xc.to_dense().t() @ Xc.to_dense())
        return G if out is None else out.add_(G)
    if X.device.type == "cpu":
        Xd = X.double()
        G = Xd.t() @ Xd
        return G if out is None else out.add_(G)
    if _lib.use_native(X) and X.dtype in (torch.bfloat16, torch.float32) and _has_syrk():
        return syrk(X, out)  # bf16 operands, fp32 accumulation (MFMA)
    Xf = X.float()
    G = Xf.t() @ Xf
    return G if out is None else out.add_(G)


ATB_CHUNK = 1000  # rows per batched slice of a tall A^T B


def atb(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A^T B for tall A [n, m], B [n, k] (n >> m, k). On the GPU the n rows are cut into
    slices of ``ATB_CHUNK`` rows: one batched GEMM of the slices plus a sum. A single
    GEMM with a reduction dimension of millions of rows is pathological in the library
    kernels, especially in fp64: X^T X of 4e6 x 16 fp64 took 0.43 s as one mm and 0.3 ms
    as 4000 batched slices (scripts/probe_fp64_gemm.py, profiles/r2_tsqr)."""
    n = A.shape[0]
    if A.device.type != "cuda" or n < 8 * ATB_CHUNK:
        return A.t() @ B
    c = n // ATB_CHUNK
    m = c * ATB_CHUNK
    At = A[:m].reshape(c, ATB_CHUNK, A.shape[1])
    Bt = B[:m].reshape(c, ATB_CHUNK, B.shape[1])
    out = torch.bmm(At.transpose(1, 2), Bt).sum(0)
    if m < n:
        out += A[m:].t() @ B[m:]
    return out


_lib.register({
    "harp_syrk_t_bf16": [_lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_int,
                         _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p],
    "harp_to_feature_major_bf16": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_long,
                                   _lib.c_int, _lib.c_int, _lib.c_void_p],
})

MT = 128  # SYRK macro tile (features)
KT = 48   # samples per SYRK stage (= the layout's sample block)
LD_ALIGN = 192  # sample padding (a multiple of KT)


class FeatureMajor:
    """Blocked feature-major bf16 copy of a data block for the MFMA SYRK:
    ``XT [ld/KT, d_pad, KT]`` (KT = 48) -- per sample block, every feature's KT samples contiguous
    (a kernel stage's operand panel is one contiguous run; csrc/syrk.hip) -- with a row of
    ones at feature ``d`` (so G[:, d] = column sums and G[d, d] = n), zero padding to
    ``d_pad = round_up(d + 1, 128)`` features and ``ld = round_up(n, 192)`` samples."""

    def __init__(self, XT: torch.Tensor, n: int, d: int):
        self.XT, self.n, self.d = XT, n, d

    @property
    def d_pad(self) -> int:
        return self.XT.shape[1]

    @property
    def ld(self) -> int:
        return self.XT.shape[0] * KT

    @staticmethod
    def dims(n: int, d: int):
        return (d + 1 + MT - 1) // MT * MT, (n + LD_ALIGN - 1) // LD_ALIGN * LD_ALIGN

    def dense(self) -> torch.Tensor:
        """[d_pad, ld] feature-major view materialised (tests / debugging)."""
        return self.XT.permute(1, 0, 2).reshape(self.d_pad, self.ld)

    @classmethod
    def from_rows(cls, X: torch.Tensor) -> "FeatureMajor":
        n, d = X.shape
        d_pad, ld = cls.dims(n, d)
        Xb = X.to(torch.bfloat16).contiguous()
        XT = torch.empty((ld // KT, d_pad, KT), dtype=torch.bfloat16, device=X.device)
        st = _lib.kernels().harp_to_feature_major_bf16(Xb.data_ptr(), n, d, Xb.stride(0), XT.data_ptr(), ld, d_pad, d,
                                                       _lib.stream_ptr(X.device))
        _lib.check(st, "to_feature_major")
        return cls(XT, n, d)

    @classmethod
    def uniform(cls, n: int, d: int, lo: float = 0.0, hi: float = 1.0, seed: int = 0, device="cuda") -> "FeatureMajor":
        """Synthetic U[lo,hi) data generated directly in the blocked layout on the device."""
        from .kmeans import _lib as _kl  # same library

        d_pad, ld = cls.dims(n, d)
        nb = ld // KT
        XT = torch.empty((nb, d_pad, KT), dtype=torch.bfloat16, device=device)
        st = _kl.kernels().harp_uniform_rows_bf16(XT.data_ptr(), nb * d_pad, KT, KT, float(lo), float(hi),
                                                  seed & 0xFFFFFFFFFFFFFFFF, 0, 0, _lib.stream_ptr(XT.device))
        _lib.check(st, "uniform_rows")
        XT[:, d:].zero_()
        full, part = divmod(n, KT)  # whole sample blocks, samples in the partial block
        XT[:full, d] = 1.0
        if part:
            XT[full, d, :part] = 1.0
            XT[full, :, part:].zero_()
        XT[full + (1 if part else 0):].zero_()
        return cls(XT, n, d)


SYRK_VARIANT = 0  # the one shipped kernel (profiles/r2_syrk: alternatives measured slower, removed)


SYRK_SYNC_EVERY = int(os.environ.get("HARP_SYRK_SYNC", "64"))  # stages between split lock-step points (0: off)
_SYNC_WS: dict = {}


def syrk_t(fm: FeatureMajor, G: torch.Tensor | None = None, num_splits: int = 0, variant: int | None = None,
           sync_every: int | None = None) -> torch.Tensor:
    """G (+)= XT XT^T over the upper 128-tiles (fp32); call :func:`symmetrize_upper` after."""
    if G is None:
        G = torch.zeros((fm.d_pad, fm.d_pad), dtype=torch.float32, device=fm.XT.device)
    ws = _SYNC_WS.get(fm.XT.device)
    if ws is None:
        ws = _SYNC_WS[fm.XT.device] = torch.zeros(1024, dtype=torch.int32, device=fm.XT.device)
    every = SYRK_SYNC_EVERY if sync_every is None else sync_every
    st = _lib.kernels().harp_syrk_t_bf16(fm.XT.data_ptr(), fm.ld, fm.ld, fm.d_pad, G.data_ptr(), G.stride(0),
                                         num_splits, SYRK_VARIANT if variant is None else variant,
                                         ws.data_ptr(), int(every), _lib.stream_ptr(fm.XT.device))
    _lib.check(st, "syrk_t")
    return G


def symmetrize_upper(G: torch.Tensor) -> torch.Tensor:
    return torch.triu(G) + torch.triu(G, 1).t()


def gram_stats(fm: FeatureMajor, G: torch.Tensor | None = None):
    """(n, column sums, X^T X) of a FeatureMajor block from ONE SYRK pass."""
    G = symmetrize_upper(syrk_t(fm, G))
    d = fm.d
    return G[d, d], G[:d, d].clone(), G[:d, :d].clone()


def _has_syrk() -> bool:
    try:
        return hasattr(_lib.kernels(), "harp_syrk_t_bf16")
    except _lib.NativeUnavailable:
        return False


def syrk(X: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """X^T X of a row-major GPU block via a feature-major bf16 copy + MFMA SYRK."""
    fm = FeatureMajor.from_rows(X)
    _, _, G = gram_stats(fm)
    return G if out is None else out.add_(G)


# ------------------------------------------------------------------ TSQR panel (csrc/tsqr.hip)
_lib.register({
    "harp_tsqr_width": [_lib.c_int],
    "harp_tsqr_rows_per_block": [],
    "harp_tsqr_level": [_lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_long,
                        _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    "harp_tsqr_apply": [_lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p,
                        _lib.c_void_p, _lib.c_long, _lib.c_void_p],
})

TSQR_MAX_D = 64


def house_tsqr(A: torch.Tensor, want_q: bool = True):
    """Householder TSQR of a tall-skinny fp64 GPU matrix (d <= 64) on the native panel
    kernels: every 256-row block is factored by one workgroup (row per thread, registers),
    the stacked R's are factored level by level until one block remains, and the explicit Q
    is built top-down by applying each block's reflectors to its slice of the level above's
    Q. Returns (Q [n, d] or None, R [d, d]) with R's diagonal made non-negative."""
    n, d = A.shape
    lib = _lib.kernels()
    W = lib.harp_tsqr_width(d)
    if W < 0:
        raise ValueError(f"house_tsqr supports d <= {TSQR_MAX_D} (got {d})")
    TBR = lib.harp_tsqr_rows_per_block()
    dev = A.device
    st = _lib.stream_ptr(dev)
    M = torch.zeros((n, W), dtype=torch.float64, device=dev)
    M[:, :d] = A
    levels = []
    while True:
        rows = M.shape[0]
        nb = (rows + TBR - 1) // TBR
        V = torch.empty_like(M)
        tau = torch.empty((nb, W), dtype=torch.float64, device=dev)
        R = torch.empty((nb, W, W), dtype=torch.float64, device=dev)
        _lib.check(lib.harp_tsqr_level(M.data_ptr(), W, rows, W, V.data_ptr(), W, tau.data_ptr(), R.data_ptr(), st),
                   "tsqr_level")
        levels.append((V, tau, rows))
        if nb == 1:
            Rf = R[0]
            break
        M = R.reshape(nb * W, W)
    sgn = torch.sign(torch.diagonal(Rf)[:d])
    sgn[sgn == 0] = 1
    Rout = (Rf[:d, :d] * sgn[:, None]).contiguous()
    if not want_q:
        return None, Rout
    S = None
    for V, tau, rows in reversed(levels):
        Q = torch.empty((rows, W), dtype=torch.float64, device=dev)
        _lib.check(lib.harp_tsqr_apply(V.data_ptr(), W, rows, W, tau.data_ptr(), _lib.ptr(S), Q.data_ptr(), W, st),
                   "tsqr_apply")
        S = Q
    return (S[:, :d] * sgn[None, :]).contiguous(), Rout
