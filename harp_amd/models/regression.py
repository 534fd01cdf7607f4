"""Linear / ridge regression and their quality metrics.

Reference: ml/daal/.../daal_linreg/normaleq (XtX, Xty partials -> gather -> solve),
daal_linreg/qrdense (per-worker QR -> merged R, Q^T y -> solve), daal_ridgereg (normal
equations + ridge penalty), daal_quality_metrics/LinRegMetrics (single-beta and group-of-
betas metrics) — all step1 local / step2 master (SURVEY §2.8.2, §2.9 rows
"linear/ridge regression").

MI355X design: the normal-equation partial is one Gram of the augmented design
``[X | 1 | y]`` (intercept column + responses), so a single SYRK-shaped pass yields
XtX, X^T 1, X^T y and y^T y; one packed allreduce merges workers; the (d+1)x(d+1) solve
runs in fp64 on every worker.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..ops import linalg as LA
from ..parallel.comm import Communicator
from .common import reduce_partials
from .stats import _local, tsqr


def _augment(X: torch.Tensor, y: torch.Tensor, intercept: bool) -> torch.Tensor:
    y2 = y.reshape(X.shape[0], -1).to(X.dtype)
    cols = [X]
    if intercept:
        cols.append(torch.ones((X.shape[0], 1), dtype=X.dtype, device=X.device))
    return torch.cat(cols + [y2], 1)


def train_linear(X: torch.Tensor, y: torch.Tensor, comm: Optional[Communicator] = None, ridge: float = 0.0,
                 intercept: bool = True, method: str = "normal") -> Dict[str, torch.Tensor]:
    """Returns ``beta`` [n_responses, d(+1)] with the intercept FIRST (DAAL layout)."""
    comm = _local(comm)
    p = X.shape[1] + (1 if intercept else 0)
    if method == "normal":
        A = _augment(X, y, intercept)
        G = reduce_partials(comm, {"g": LA.gram(A)})["g"].double()
        XtX, Xty = G[:p, :p], G[:p, p:]
        if ridge:
            reg = torch.eye(p, dtype=torch.float64, device=G.device) * ridge
            if intercept:
                reg[p - 1, p - 1] = 0.0  # the intercept is not penalised
            XtX = XtX + reg
        beta = torch.linalg.solve(XtX, Xty)
    elif method == "qr":
        A = _augment(X, y, intercept).double()
        R = tsqr(A, comm, want_q=False)["R"]
        Rx, Rxy = R[:p, :p], R[:p, p:]
        beta = torch.linalg.solve_triangular(Rx, Rxy, upper=True)
    else:
        raise ValueError(method)
    beta = beta.t()  # [responses, p]
    if intercept:
        beta = torch.cat([beta[:, -1:], beta[:, :-1]], 1)
    return {"beta": beta}


def predict_linear(X: torch.Tensor, beta: torch.Tensor) -> torch.Tensor:
    b = beta.to(X.device, torch.float64)
    if b.shape[1] == X.shape[1] + 1:
        return X.double() @ b[:, 1:].t() + b[:, 0]
    return X.double() @ b.t()


def linreg_quality(X: torch.Tensor, y: torch.Tensor, beta: torch.Tensor, comm: Optional[Communicator] = None,
                   alpha: float = 0.05) -> Dict[str, torch.Tensor]:
    """DAAL LinRegMetrics (single beta): expected means / variances, regression / residual /
    total sums of squares, R^2, F-statistic, residual variance, beta variances + z-scores
    and 1-alpha confidence intervals, inverse of X^T X."""
    from scipy.stats import norm

    comm = _local(comm)
    y2 = y.reshape(X.shape[0], -1).double()
    yhat = predict_linear(X, beta)
    n_loc = float(X.shape[0])
    parts = reduce_partials(comm, {"n": torch.tensor([n_loc], device=y2.device), "sy": y2.sum(0),
                                   "syy": (y2 * y2).sum(0), "res": ((y2 - yhat) ** 2).sum(0),
                                   "xtx": LA.gram(torch.cat([torch.ones((X.shape[0], 1), device=X.device, dtype=X.dtype), X], 1))})
    n = parts["n"].item()
    mean = parts["sy"] / n
    tss = parts["syy"] - n * mean * mean
    rss = parts["res"]
    regss = tss - rss
    p = beta.shape[1]
    var_res = rss / max(n - p, 1)
    inv = torch.linalg.inv(parts["xtx"].double())
    vb = torch.diagonal(inv)[None, :] * var_res[:, None]
    z = beta.double().cpu() / vb.sqrt().cpu()
    q = float(norm.ppf(1 - alpha / 2))
    ci = torch.stack([beta.double().cpu() - q * vb.sqrt().cpu(), beta.double().cpu() + q * vb.sqrt().cpu()], -1)
    return {"expectedMeans": mean, "expectedVariance": tss / max(n - 1, 1), "regSS": regss, "resSS": rss,
            "tSS": tss, "determinationCoeff": regss / tss, "fStatistics": (regss / max(p - 1, 1)) / var_res,
            "rms": (rss / n).sqrt(), "variance": var_res, "betaVariance": vb, "zScore": z, "confidenceIntervals": ci,
            "inverseOfXtX": inv}


def classification_quality(y_true: torch.Tensor, y_pred: torch.Tensor, num_classes: int) -> Dict[str, torch.Tensor]:
    """Multi-class quality metrics (DAAL SVMMultiMetrics): confusion matrix, average
    accuracy, error rate, micro/macro precision, recall, F-score, specificity."""
    yt, yp = y_true.long().cpu(), y_pred.long().cpu()
    cm = torch.zeros((num_classes, num_classes), dtype=torch.float64)
    cm.index_put_((yt, yp), torch.ones(yt.numel(), dtype=torch.float64), accumulate=True)
    tp = cm.diagonal()
    fp = cm.sum(0) - tp
    fn = cm.sum(1) - tp
    tn = cm.sum() - tp - fp - fn
    prec = tp / (tp + fp).clamp_min(1e-300)
    rec = tp / (tp + fn).clamp_min(1e-300)
    f = 2 * prec * rec / (prec + rec).clamp_min(1e-300)
    acc = (tp + tn) / cm.sum()
    return {"confusionMatrix": cm, "averageAccuracy": acc.mean(), "errorRate": 1 - tp.sum() / cm.sum(),
            "microPrecision": tp.sum() / (tp + fp).sum(), "microRecall": tp.sum() / (tp + fn).sum(),
            "macroPrecision": prec.mean(), "macroRecall": rec.mean(), "macroFscore": f.mean(),
            "macroSpecificity": (tn / (tn + fp).clamp_min(1e-300)).mean()}
