"""Statistics family: covariance, low-order moments, PCA, normalization, quantiles,
sorting, outlier detection.

Reference (ml/daal): ``daal_cov/{dense,csr}distri`` (covariance step1 ->
gather -> step2, COVDaalCollectiveMapper.java:146-175), ``daal_mom/{dense,csr}distri``
(low_order_moments), ``daal_pca/{cordense,corcsr,svddense}distr`` (correlation /
SVD PCA, PCADaalCollectiveMapper.java:121-147), batch-only ``daal_normalization``
(minmax, zscore), ``daal_quantile``, ``daal_sorting``, ``daal_outlier`` (univariate,
multivariate, BACON).

Each distributed algorithm is: local partial sums on the device (the Gram / cross-product
partial is a GEMM — ``ops.linalg.gram``) -> one packed allreduce
(:func:`~harp_amd.models.common.reduce_partials`) -> finalize on every worker in fp64.
Inputs may be dense tensors or torch sparse (CSR/COO) tensors (the ``csr`` variants).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from ..core.combiner import Operation
from ..ops import linalg as LA
from ..parallel.comm import Communicator
from .common import broadcast_tensor, gather_rows, reduce_partials


def _local(comm: Optional[Communicator]) -> Communicator:
    return comm if comm is not None else Communicator()


# ------------------------------------------------------------------ covariance / moments
# Precision policy of the partial-result family (DAAL computes these in fp64:
# COVDaalCollectiveMapper.java:146-175, PCADaalCollectiveMapper.java:121 Double.class):
#  * "bf16": the MFMA SYRK fast path -- operands rounded to bf16 ONCE (ops.linalg.FeatureMajor),
#    fp32 accumulation; n, the column sums and X^T X all come from that one rounded operand
#    (a row of ones in the Gram), so the finalize never mixes operands. The bf16 rounding
#    (2^-9 relative per element) bounds the result: 3.5e-5 relative (max-norm) covariance
#    error measured on 1e6 x 1000 U[0,1) data (tests/test_linalg_gpu.py bounds it by 3e-4,
#    tests/test_partial_results.py by 3e-3 on the CPU form);
#  * "fp32": fp32 operands, rocBLAS fp32 GEMMs over row slices of ops.linalg.ATB_CHUNK
#    rows on data shifted by a per-rank reference row (no cancellation in the centred
#    sums), slices summed in fp64: <= 1e-6 relative to an fp64 covariance;
#  * "fp64": fp64 operands and GEMMs (the reference's precision).
# dtype=None picks by the input: bf16 / FeatureMajor -> "bf16", fp32 -> "fp32", fp64 or
# CPU -> "fp64" (an fp32 input is never silently rounded to bf16).
DTYPES = ("bf16", "fp32", "fp64")


def _policy(X, dtype: Optional[str]) -> str:
    if dtype is not None:
        if dtype not in DTYPES:
            raise ValueError(f"dtype={dtype!r}: expected one of {DTYPES}")
        return dtype
    if isinstance(X, LA.FeatureMajor) or X.dtype == torch.bfloat16:
        return "bf16"
    if X.device.type == "cpu" or X.dtype == torch.float64 or LA._is_sparse(X):
        return "fp64"
    return "fp32"


def _shifted_sums(X: torch.Tensor, acc: torch.dtype):
    """(n, sum x, X^T X) in fp64 from GEMMs in ``acc`` over row slices of X - c, c = X's
    first row (the centred sums carry no cancellation; the shift is undone in fp64)."""
    n, d = X.shape
    if n == 0:
        z = torch.zeros(d, dtype=torch.float64, device=X.device)
        return 0.0, z, torch.zeros((d, d), dtype=torch.float64, device=X.device)
    c = X[0].to(acc)
    S = torch.zeros((d, d), dtype=torch.float64, device=X.device)
    s = torch.zeros(d, dtype=torch.float64, device=X.device)
    step = LA.ATB_CHUNK * 64
    for a in range(0, n, step):
        Y = X[a:a + step].to(acc) - c
        S += LA.atb(Y, Y).double() if acc != torch.float64 else LA.atb(Y, Y)
        s += Y.double().sum(0) if acc != torch.float64 else Y.sum(0)
    c64 = c.double()
    xtx = S + torch.outer(c64, s) + torch.outer(s, c64) + n * torch.outer(c64, c64)
    return float(n), s + n * c64, xtx


def covariance_partial(X, dtype: Optional[str] = None) -> Dict[str, torch.Tensor]:
    """Step 1: n, sum x, X^T X (cross-product) of the local block, at the ``dtype``
    precision (module notes above). ``X``: a row-major tensor (dense or sparse) or an
    :class:`ops.linalg.FeatureMajor` block."""
    mode = _policy(X, dtype)
    if isinstance(X, LA.FeatureMajor):
        if mode != "bf16":
            raise ValueError("a FeatureMajor block holds bf16 operands: use dtype='bf16'")
        n, s, G = LA.gram_stats(X)
        return {"n": n.reshape(1).double(), "sum": s.double(), "xtx": G.double()}
    if LA._is_sparse(X):
        n = X.shape[0]
        s = LA.colsum(X)
        return {"n": torch.tensor([float(n)], dtype=torch.float64, device=s.device), "sum": s.double(),
                "xtx": LA.gram(X).double()}
    if mode == "bf16":
        if X.device.type == "cuda" and LA._has_syrk() and _native(X):
            return covariance_partial(LA.FeatureMajor.from_rows(X), "bf16")
        Xb = X.to(torch.bfloat16).float()  # the same rounding, fp32 accumulation (CPU)
        n = float(X.shape[0])
        return {"n": torch.tensor([n], dtype=torch.float64, device=X.device), "sum": Xb.sum(0).double(),
                "xtx": (Xb.t() @ Xb).double()}
    n, s, xtx = _shifted_sums(X, torch.float32 if mode == "fp32" else torch.float64)
    return {"n": torch.tensor([n], dtype=torch.float64, device=X.device), "sum": s, "xtx": xtx}


def _native(X) -> bool:
    from ..ops import _lib

    return _lib.use_native(X)


def covariance_finalize(p: Dict[str, torch.Tensor], bias: bool = False) -> Dict[str, torch.Tensor]:
    n = p["n"].double().item()
    mean = p["sum"].double() / n
    cov = (p["xtx"].double() - n * torch.outer(mean, mean)) / (n if bias else max(n - 1, 1))
    return {"mean": mean, "covariance": cov}


def _timed(metrics, kind: str, op: str, nbytes: int, device):
    """``metrics.time_collective`` (HIP events on GPUs) when a Metrics object is given."""
    import contextlib

    if metrics is None:
        return contextlib.nullcontext()
    return metrics.time_collective(kind, "pca", op, nbytes, device)


def covariance(X, comm: Optional[Communicator] = None, bias: bool = False,
               dtype: Optional[str] = None, metrics=None) -> Dict[str, torch.Tensor]:
    """``metrics`` (optional :class:`utils.metrics.Metrics`): the partial-result allreduce is
    recorded as an "allreduce" collective (op "gram") with its bytes and stream time."""
    comm = _local(comm)
    part = covariance_partial(X, dtype)
    nbytes = sum(v.numel() for v in part.values()) * 8 if comm.world_size > 1 else 0
    with _timed(metrics, "allreduce", "gram", nbytes, comm.device):
        red = reduce_partials(comm, part, dtype=torch.float64)
    return covariance_finalize(red, bias)


def correlation(X, comm: Optional[Communicator] = None, dtype: Optional[str] = None,
                metrics=None) -> Dict[str, torch.Tensor]:
    r = covariance(X, comm, dtype=dtype, metrics=metrics)
    sd = r["covariance"].diagonal().clamp_min(0).sqrt()
    r["correlation"] = r["covariance"] / torch.outer(sd, sd).clamp_min(1e-300)
    return r


def low_order_moments(X: torch.Tensor, comm: Optional[Communicator] = None,
                      dtype: Optional[str] = None) -> Dict[str, torch.Tensor]:
    """DAAL low_order_moments: minimum, maximum, sum, sumSquares, sumSquaresCentered, mean,
    secondOrderRawMoment, variance, standardDeviation, variation. ``dtype`` as for
    :func:`covariance`: "bf16" sums the bf16-rounded operands in fp32, "fp32" / "fp64" sum
    shifted row slices and accumulate in fp64 (sumSquaresCentered then has no cancellation)."""
    comm = _local(comm)
    Xd = X.to_dense() if X.is_sparse or X.layout == torch.sparse_csr else X
    mode = _policy(Xd, dtype)
    n = float(Xd.shape[0])
    if mode == "bf16":
        Xf = Xd.to(torch.bfloat16).float()
        s1, s2 = Xf.sum(0).double(), (Xf * Xf).sum(0).double()
        c = torch.zeros_like(s1)
        sc1, sc2 = s1, s2
    else:
        acc = torch.float32 if mode == "fp32" else torch.float64
        c = Xd[0].to(acc).double() if Xd.shape[0] else torch.zeros(Xd.shape[1], dtype=torch.float64, device=Xd.device)
        sc1 = torch.zeros(Xd.shape[1], dtype=torch.float64, device=Xd.device)
        sc2 = torch.zeros_like(sc1)
        step = 1 << 16
        for a in range(0, Xd.shape[0], step):
            Y = Xd[a:a + step].to(acc) - c.to(acc)
            sc1 += Y.sum(0).double()
            sc2 += (Y * Y).sum(0).double()
        s1 = sc1 + n * c
        s2 = sc2 + 2 * c * sc1 + n * c * c
    # shifted sums combine across ranks through the raw sums; the centred sum of squares is
    # formed from per-rank centred pieces (Chan et al.) so no rank's shift cancels
    sums = reduce_partials(comm, {"n": torch.tensor([n], dtype=torch.float64, device=Xd.device), "sum": s1,
                                  "sumsq": s2}, dtype=torch.float64)
    N = sums["n"].item()
    mean = sums["sum"] / N
    local_mean = s1 / max(n, 1.0)
    # this rank's centred SS around its own mean, then the between-rank term
    ss_local = sc2 - (sc1 * sc1) / max(n, 1.0) if mode != "bf16" else s2 - s1 * s1 / max(n, 1.0)
    ss = reduce_partials(comm, {"ss": ss_local + n * (local_mean - mean) ** 2}, dtype=torch.float64)["ss"]
    Xm = Xd.double() if Xd.device.type == "cpu" else Xd.float()
    mm = reduce_partials(comm, {"min": Xm.min(0).values.double(), "negmax": -Xm.max(0).values.double()},
                         Operation.MIN, dtype=torch.float64)
    var = ss / max(N - 1, 1)
    sd = var.clamp_min(0).sqrt()
    return {"minimum": mm["min"], "maximum": -mm["negmax"], "sum": sums["sum"], "sumSquares": sums["sumsq"],
            "sumSquaresCentered": ss, "mean": mean, "secondOrderRawMoment": sums["sumsq"] / N, "variance": var,
            "standardDeviation": sd, "variation": sd / mean}


# ------------------------------------------------------------------ PCA
def pca_step2(corr: torch.Tensor, comm: Optional[Communicator] = None, metrics=None):
    """Step 2 of the correlation method on the master (PCADaalCollectiveMapper.java:136-154):
    eigenvalues AND eigenvectors of the d x d fp64 correlation matrix -- on a GPU the one-XCD
    reduction + divide and conquer of ``ops.eig.eigh`` -- then broadcast. Returns
    (eigenvalues ascending, eigenvectors as columns)."""
    from ..ops import eig as EIG

    comm = _local(comm)
    d = corr.shape[0]
    dev = corr.device
    if comm.rank == 0:
        evals, evecs = EIG.eigh(corr.double().contiguous())
        packed = torch.cat([evals.reshape(1, d), evecs]).contiguous()
    else:
        packed = None
    with _timed(metrics, "broadcast", "eigvecs", (d + 1) * d * 8 if comm.world_size > 1 else 0, comm.device):
        packed = broadcast_tensor(comm, packed, (d + 1, d), torch.float64).to(dev)
    return packed[0], packed[1:]


def pca(X, comm: Optional[Communicator] = None, method: str = "correlation",
        n_components: Optional[int] = None, dtype: Optional[str] = None, metrics=None) -> Dict[str, torch.Tensor]:
    """PCA of the (standardized) data: eigenvalues descending + eigenvectors (rows).

    ``correlation``: eigen-decomposition of the distributed correlation matrix (``X`` may
    be a :class:`ops.linalg.FeatureMajor` block: the one-pass MFMA SYRK path).
    ``svd``: z-score the data with global moments, distributed TSQR, SVD of R
    (the DAAL svdDense method); both yield the correlation-PCA spectrum. ``dtype``: the
    step-1 precision (see :func:`covariance`). ``metrics``: the correlation method's Gram
    allreduce and eigenvector broadcast are recorded as collectives (bench attribution)."""
    comm = _local(comm)
    if method == "correlation":
        r = correlation(X, comm, dtype=dtype, metrics=metrics)
        evals, evecs = pca_step2(r["correlation"], comm, metrics=metrics)
        order = torch.argsort(evals, descending=True)
        evals, evecs = evals[order], evecs[:, order].t()
    elif method == "svd":
        if isinstance(X, LA.FeatureMajor):
            raise ValueError("method='svd' needs the row-major data")
        mom = low_order_moments(X, comm, dtype=dtype)
        Z = (X.double() - mom["mean"].to(X.device)) / mom["standardDeviation"].to(X.device).clamp_min(1e-300)
        qr = tsqr(Z, comm, want_q=False)
        ntot = reduce_partials(comm, {"n": torch.tensor([float(X.shape[0])], device=X.device)})["n"].item()
        _, s, vt = torch.linalg.svd(qr["R"])
        evals, evecs = s * s / max(ntot - 1, 1), vt
    else:
        raise ValueError(method)
    # sign convention: largest-magnitude component of each eigenvector positive
    idx = evecs.abs().argmax(1)
    sign = torch.sign(evecs.gather(1, idx[:, None]))
    evecs = evecs * sign
    if n_components:
        evals, evecs = evals[:n_components], evecs[:n_components]
    return {"eigenvalues": evals, "eigenvectors": evecs}


# ------------------------------------------------------------------ TSQR / SVD (distributed)
def _native_tsqr(X: torch.Tensor) -> bool:
    """GPU blocks with d <= 64 take the native panel kernels (wider panels: rocSOLVER)."""
    from ..ops import _lib
    from ..ops.linalg import TSQR_MAX_D

    return X.device.type == "cuda" and X.shape[1] <= TSQR_MAX_D and _lib.use_native(X)

CHOLQR_MAX_DIAG_RATIO = 1e5  # max(diag R) / min(diag R) beyond which CholeskyQR2 is not trusted
# max |R2 - I| of the second pass beyond which Q1 was too far from orthogonal for the second
# pass to repair (Kahan-like input can pass the diagonal test with cond(X) ~ 1e14)
CHOLQR_MAX_R2_DEV = 1e-3


def cholesky_qr2(X: torch.Tensor, comm: Optional[Communicator] = None) -> Optional[Dict[str, torch.Tensor]]:
    """Distributed CholeskyQR2 in fp64: G = sum_ranks X^T X (one d x d allreduce), R1 =
    chol(G), Q1 = X R1^-1; the same again on Q1 restores orthogonality to ~1e-15, R =
    R2 R1. Every flop is a GEMM / TRSM on the fp64 matrix cores and the data is read a
    handful of times, against D sequential Householder steps of the panel kernels.

    Stable while cond(X) is well below 1e8; returns None (the caller falls back to
    Householder TSQR) when the Cholesky fails, when the R1 diagonal spread -- a lower bound
    of cond(X) -- exceeds ``CHOLQR_MAX_DIAG_RATIO``, or when the second factor R2 is not
    within ``CHOLQR_MAX_R2_DEV`` of the identity (R2^T R2 = Q1^T Q1: Q1 was not near
    orthogonal, which a small diagonal spread does not rule out). Every decision is taken
    from allreduced values, so every worker takes the same branch."""
    comm = _local(comm)
    Xd = X.double().contiguous()
    Q, R = Xd, None
    for _ in range(2):
        G = reduce_partials(comm, {"g": LA.atb(Q, Q)})["g"].to(Xd.device)
        L, info = torch.linalg.cholesky_ex(G)
        if int(info) != 0:
            return None
        Rk = L.t().contiguous()
        dg = torch.diagonal(Rk)
        if R is None and float(dg.max()) > CHOLQR_MAX_DIAG_RATIO * float(dg.min().clamp_min(1e-300)):
            return None
        if R is not None:
            eye = torch.eye(Rk.shape[0], dtype=Rk.dtype, device=Rk.device)
            if float((Rk - eye).abs().max()) > CHOLQR_MAX_R2_DEV:
                return None
        # Q R^-1 as one GEMM with the d x d triangular inverse (a right-side TRSM over the
        # tall matrix measured ~200x slower in rocBLAS and runs out of workspace)
        eye = torch.eye(Rk.shape[0], dtype=Rk.dtype, device=Rk.device)
        Q = Q @ torch.linalg.solve_triangular(Rk, eye, upper=True)
        R = Rk if R is None else Rk @ R
    return {"Q": Q, "R": R}


def tsqr(X: torch.Tensor, comm: Optional[Communicator] = None, want_q: bool = True,
         method: str = "auto") -> Dict[str, torch.Tensor]:
    """Distributed tall-skinny QR (daal_qr 3-step: local QR -> QR of stacked R's -> local
    Q update). The stacked R's are all-gathered so every worker runs step 2 itself.

    ``method``: "auto" (GPU: :func:`cholesky_qr2`, falling back to Householder for
    ill-conditioned input; CPU: Householder), "cholqr2", or "householder". The result
    (R with a non-negative diagonal, orthonormal Q) is the same either way."""
    comm = _local(comm)
    d = X.shape[1]
    if method == "cholqr2" or (method == "auto" and X.device.type == "cuda"):  # same branch on every rank
        out = cholesky_qr2(X, comm)
        if out is not None:
            if not want_q:
                out.pop("Q")
            return out
        if method == "cholqr2":
            raise ValueError("CholeskyQR2 failed (matrix too ill-conditioned)")
    if _native_tsqr(X):
        # step 1 on the hand-written fp64 Householder panel kernels (csrc/tsqr.hip)
        from ..ops.linalg import house_tsqr

        Xd = X.double().contiguous()
        Q1, R1 = house_tsqr(Xd, want_q)
        Rs = gather_rows(comm, R1)  # [P*d, d]
        Q2, R = house_tsqr(Rs.contiguous(), want_q)
        out = {"R": R}
        if want_q:
            out["Q"] = Q1 @ Q2[comm.rank * d:(comm.rank + 1) * d]
        return out
    Xd = X.double() if X.device.type == "cpu" or X.dtype == torch.float64 else X.float()
    Q1, R1 = torch.linalg.qr(Xd, mode="reduced")
    Rs = gather_rows(comm, R1)  # [P*d, d]
    Q2, R = torch.linalg.qr(Rs.double(), mode="reduced")
    # make R's diagonal non-negative (unique QR)
    sgn = torch.sign(torch.diagonal(R))
    sgn[sgn == 0] = 1
    R = R * sgn[:, None]
    Q2 = Q2 * sgn[None, :]
    out = {"R": R}
    if want_q:
        blk = Q2[comm.rank * d:(comm.rank + 1) * d].to(Xd.device, Xd.dtype)
        out["Q"] = Q1 @ blk
    return out


def svd(X: torch.Tensor, comm: Optional[Communicator] = None, want_u: bool = True) -> Dict[str, torch.Tensor]:
    """Distributed SVD via TSQR (daal_svd 3-step): X = Q R, R = U_r S V^T, U = Q U_r."""
    r = tsqr(X, comm, want_q=want_u)
    Ur, s, vt = torch.linalg.svd(r["R"])
    out = {"singularValues": s, "rightSingularMatrix": vt}
    if want_u:
        out["leftSingularMatrix"] = r["Q"] @ Ur.to(r["Q"].device, r["Q"].dtype)
    return out


def cholesky(A: torch.Tensor) -> torch.Tensor:
    """Lower-triangular Cholesky factor (daal_cholesky, batch)."""
    return torch.linalg.cholesky(A.double())


def pivoted_qr(X: torch.Tensor) -> Dict[str, torch.Tensor]:
    """QR with column pivoting (daal_pivoted_qr, batch): X[:, perm] = Q R."""
    import scipy.linalg

    Q, R, piv = scipy.linalg.qr(X.double().cpu().numpy(), mode="economic", pivoting=True)
    return {"Q": torch.from_numpy(Q), "R": torch.from_numpy(R), "permutation": torch.from_numpy(piv)}


# ------------------------------------------------------------------ normalization
def normalize_minmax(X: torch.Tensor, lower: float = 0.0, upper: float = 1.0,
                     comm: Optional[Communicator] = None) -> torch.Tensor:
    m = reduce_partials(_local(comm), {"min": X.min(0).values, "negmax": -X.max(0).values}, Operation.MIN)
    mn, mx = m["min"].to(X.device, X.dtype), (-m["negmax"]).to(X.device, X.dtype)
    rng = (mx - mn)
    rng = torch.where(rng == 0, torch.ones_like(rng), rng)
    return lower + (X - mn) / rng * (upper - lower)


def normalize_zscore(X: torch.Tensor, comm: Optional[Communicator] = None) -> torch.Tensor:
    mom = low_order_moments(X, comm)
    sd = mom["standardDeviation"].to(X.device, X.dtype)
    return (X - mom["mean"].to(X.device, X.dtype)) / torch.where(sd == 0, torch.ones_like(sd), sd)


# ------------------------------------------------------------------ quantiles / sorting
def quantiles(X: torch.Tensor, q=(0.1, 0.5, 0.9), comm: Optional[Communicator] = None) -> torch.Tensor:
    """Per-feature quantiles [len(q), d] (daal_quantile). Distributed: exact, over the
    all-gathered columns."""
    Xa = gather_rows(_local(comm), X) if comm is not None else X
    return torch.quantile(Xa.double(), torch.tensor(q, dtype=torch.float64, device=Xa.device), dim=0)


def sort_features(X: torch.Tensor) -> torch.Tensor:
    """Each feature column sorted ascending (daal_sorting)."""
    return torch.sort(X, dim=0).values


# ------------------------------------------------------------------ outlier detection
def outliers_univariate(X: torch.Tensor, threshold: float = 3.0, comm: Optional[Communicator] = None,
                        init: str = "moments", location: Optional[torch.Tensor] = None,
                        scatter: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-feature weights (1 = inlier): |x - location| / scatter <= threshold.
    ``init``: "moments" (global mean / standard deviation), "default" (DAAL
    univariate_outlier_detection's default initialisation: location 0, scatter 1 -- the
    reference app, daal_outlier/unidensebatch, runs it), or "given" (``location`` /
    ``scatter`` per feature)."""
    if init == "moments":
        mom = low_order_moments(X, comm)
        loc, sc = mom["mean"].to(X.device), mom["standardDeviation"].to(X.device)
    elif init == "default":
        loc = torch.zeros(X.shape[1], dtype=torch.float64, device=X.device)
        sc = torch.ones_like(loc)
    elif init == "given":
        loc, sc = location.double().to(X.device), scatter.double().to(X.device)
    else:
        raise ValueError(init)
    z = (X.double() - loc) / sc.clamp_min(1e-300)
    return (z.abs() <= threshold).to(X.dtype)


def mahalanobis_sq(X: torch.Tensor, mean: torch.Tensor, cov: torch.Tensor) -> torch.Tensor:
    L = torch.linalg.cholesky(cov.double() + 1e-12 * torch.eye(cov.shape[0], dtype=torch.float64, device=cov.device))
    Z = torch.linalg.solve_triangular(L, (X.double() - mean.double()).t(), upper=False)
    return (Z * Z).sum(0)


def outliers_multivariate(X: torch.Tensor, threshold: Optional[float] = None,
                          comm: Optional[Communicator] = None) -> torch.Tensor:
    """Row weights (1 = inlier) by Mahalanobis distance to the global mean/covariance;
    default threshold = chi2_{0.999}(d) on the squared distance."""
    r = covariance(X, comm)
    d2 = mahalanobis_sq(X, r["mean"].to(X.device), r["covariance"].to(X.device))
    if threshold is None:
        from scipy.stats import chi2

        threshold = float(chi2.ppf(0.999, X.shape[1]))
    return (d2 <= threshold).to(X.dtype)


def outliers_bacon(X: torch.Tensor, alpha: float = 0.05, init: str = "median", max_iter: int = 100) -> torch.Tensor:
    """BACON outlier detection (Billor, Hadi & Velleman 2000; daal bacon_outlier_detection):
    grow a clean basic subset by Mahalanobis distance until it stabilises; returns row
    weights (1 = inlier)."""
    from scipy.stats import chi2

    Xd = X.double()
    n, p = Xd.shape
    if init == "median":
        d0 = (Xd - Xd.median(0).values).norm(dim=1)
    else:
        d0 = mahalanobis_sq(Xd, Xd.mean(0), torch.cov(Xd.t()))
    m = min(n, max(4 * p, p + 1))
    basic = torch.zeros(n, dtype=torch.bool, device=X.device)
    basic[torch.argsort(d0)[:m]] = True
    cnp = lambda r: max(0.0, 1 + (p + 1) / (n - p) + 2 / (n - 1 - 3 * p) if n - 1 - 3 * p > 0 else 1.0)  # noqa: E731
    for _ in range(max_iter):
        sub = Xd[basic]
        mu = sub.mean(0)
        cov = torch.cov(sub.t()).reshape(p, p)
        dist = mahalanobis_sq(Xd, mu, cov).clamp_min(0).sqrt()
        r = int(basic.sum())
        h = (n + p + 1) // 2
        c = max(0.0, (h - r) / (h + r)) + 1 + (p + 1) / max(n - p, 1) + 1 / max(n - h - p, 1)
        thr = c * math.sqrt(chi2.ppf(1 - alpha / n, p))
        new = dist < thr
        if torch.equal(new, basic):
            break
        basic = new
    return basic.to(X.dtype)
