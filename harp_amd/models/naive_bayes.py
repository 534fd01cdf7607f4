"""Multinomial Naive Bayes (dense and CSR), distributed.

Reference: ml/daal/.../daal_naive/{dense,csr}distri (multinomial_naive_bayes step1 on
every worker -> gather -> step2 master; NaiveDaalCollectiveMapper.java). Partial result =
per-class feature sums + per-class counts. Here the per-class sums are one
(one-hot)^T X GEMM on the device; one allreduce merges the partials; every worker holds
the model. Prediction is X log(theta)^T (+ log prior): a GEMM + argmax.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..ops import linalg as LA

from ..parallel.comm import Communicator
from .common import reduce_partials
from .stats import _local


def _dense(X):
    return X.to_dense() if (X.is_sparse or X.layout == torch.sparse_csr) else X


def train(X: torch.Tensor, y: torch.Tensor, num_classes: int, comm: Optional[Communicator] = None,
          alpha: float = 1.0, prior: str = "fit") -> Dict[str, torch.Tensor]:
    comm = _local(comm)
    yl = y.reshape(-1).long().to(X.device)
    acc = torch.float64 if X.device.type == "cpu" else torch.float32
    if X.is_sparse or X.layout == torch.sparse_csr:
        Xc = X.to_sparse_coo().coalesce()
        rows, cols = Xc.indices()
        sums = torch.zeros((num_classes, X.shape[1]), dtype=acc, device=X.device)
        sums.index_put_((yl[rows], cols), Xc.values().to(acc), accumulate=True)
    else:
        onehot = torch.nn.functional.one_hot(yl, num_classes).to(acc)
        sums = LA.atb(onehot, X.to(acc))
    counts = torch.bincount(yl, minlength=num_classes).to(acc)
    p = reduce_partials(comm, {"sums": sums, "counts": counts})
    fs = p["sums"] + alpha
    log_theta = (fs / fs.sum(1, keepdim=True)).log()
    if prior == "uniform":
        log_prior = torch.full((num_classes,), -torch.log(torch.tensor(float(num_classes))).item(),
                               dtype=torch.float64, device=log_theta.device)
    else:
        log_prior = (p["counts"] / p["counts"].sum()).clamp_min(1e-300).log()
    return {"logTheta": log_theta, "logPrior": log_prior, "featureSums": p["sums"], "classCounts": p["counts"]}


def predict(X: torch.Tensor, model: Dict[str, torch.Tensor]) -> torch.Tensor:
    lt = model["logTheta"].to(X.device)
    Xd = _dense(X).to(lt.dtype)
    return (Xd @ lt.t() + model["logPrior"].to(X.device)).argmax(1)
