"""Multi-label one-vs-rest logistic regression with model rotation (contrib MLR).

Reference: contrib/src/main/java/edu/iu/mlr/MLRMapper.java:58-140 — per-topic weight
vectors are partitions; they are regrouped to owners, then rotated ``ITER * P`` times so
that every topic model visits every worker's data shard (GDtask.java:30-72: sequential
per-instance gradient step ``W += alpha (label - sigmoid(W.x)) x`` with the bias in
W[0]); finally the table is allgathered; evaluation repeats the rotation computing
per-topic TP/FP/FN (EVtask) and the master reports precision / recall / F1.

MI355X design: the topic models are ONE device slab per worker ([T/P, D+1], topics
padded to a multiple of P) rotated with :class:`DeviceRotator` (async p2p on a private
RCCL channel). The per-instance loop becomes mini-batches: ``S = X_b W^T`` (sparse x
dense), ``G = (Y_b - sigmoid(S))^T X_b`` (scatter-add over the batch's nonzeros) —
``batch_size=1`` reproduces the reference's update order exactly. Evaluation is one
GEMM over the allgathered model + one allreduce of the [T, 3] confusion counts.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ..parallel.comm import Communicator
from ..runtime.dymoro import DeviceRotator, RotationSchedule
from .common import gather_rows, reduce_partials


@dataclass
class MLRConfig:
    alpha: float = 1.0
    iterations: int = 1
    batch_size: int = 64
    threshold: float = 0.5


class CSRRows:
    """Row-sliceable sparse matrix (crow/col/val) living on one device."""

    def __init__(self, crow: torch.Tensor, col: torch.Tensor, val: torch.Tensor, ncols: int):
        self.crow, self.col, self.val, self.ncols = crow.long(), col.long(), val, ncols

    @classmethod
    def from_dense(cls, X: torch.Tensor) -> "CSRRows":
        c = X.to_sparse_csr()
        return cls(c.crow_indices(), c.col_indices(), c.values(), X.shape[1])

    @classmethod
    def from_torch(cls, X) -> "CSRRows":
        if X.layout != torch.sparse_csr:
            X = X.to_sparse_csr() if X.is_sparse else X.to_sparse_csr()
        return cls(X.crow_indices(), X.col_indices(), X.values(), X.shape[1])

    @property
    def nrows(self) -> int:
        return self.crow.numel() - 1

    def rows(self, a: int, b: int):
        """(row ids relative to a, col ids, values) of rows [a, b)."""
        s, e = int(self.crow[a]), int(self.crow[b])
        cnt = self.crow[a + 1:b + 1] - self.crow[a:b]
        r = torch.repeat_interleave(torch.arange(b - a, device=self.col.device), cnt)
        return r, self.col[s:e], self.val[s:e]

    def matmul_t(self, W: torch.Tensor, a: int, b: int) -> torch.Tensor:
        """X[a:b] @ W^T for W [T, ncols] -> [b-a, T]."""
        r, c, v = self.rows(a, b)
        out = torch.zeros((b - a, W.shape[0]), dtype=W.dtype, device=W.device)
        out.index_add_(0, r, W[:, c].t() * v.to(W.dtype)[:, None])
        return out

    def to(self, device) -> "CSRRows":
        return CSRRows(self.crow.to(device), self.col.to(device), self.val.to(device), self.ncols)


    def kernel_operands(self):
        """(crow int64, col int32, val fp64) for ``csrc/mlr.hip``, built once per device."""
        ops = getattr(self, "_kops", None)
        if ops is None:
            ops = (self.crow.contiguous(), self.col.to(torch.int32).contiguous(),
                   self.val.to(torch.float64).contiguous())
            self._kops = ops
        return ops


def _sgd_pass(W: torch.Tensor, X: CSRRows, Y: torch.Tensor, alpha: float, batch: int) -> None:
    """One pass of the GDtask update over the local rows; W [T, D+1], bias in column 0.

    HIP tensors: the whole pass is one launch of ``csrc/mlr.hip`` (one workgroup per
    topic chain); CPU: the mini-batch torch expression below (its numerics oracle)."""
    from ..ops import _lib

    if W.device.type == "cuda" and W.dtype == torch.float64 and batch <= 1024:
        from ..ops import mlr as mlr_ops

        mlr_ops.sgd_pass(W, *X.kernel_operands(), X.nrows, Y, alpha, batch)
        return
    if W.device.type == "cuda":
        _lib.kernels()
    _sgd_pass_torch(W, X, Y, alpha, batch)


def _sgd_pass_torch(W: torch.Tensor, X: CSRRows, Y: torch.Tensor, alpha: float, batch: int) -> None:
    n = X.nrows
    for a in range(0, n, batch):
        b = min(n, a + batch)
        r, c, v = X.rows(a, b)
        S = torch.zeros((b - a, W.shape[0]), dtype=W.dtype, device=W.device)
        S.index_add_(0, r, W[:, c + 1].t() * v.to(W.dtype)[:, None])
        S += W[:, 0]
        R = alpha * (Y[a:b].to(W.dtype) - torch.sigmoid(S))  # [b, T]
        W[:, 0] += R.sum(0)
        W.index_add_(1, c + 1, (R[r] * v.to(W.dtype)[:, None]).t())


def train(comm: Communicator, X: CSRRows, Y: torch.Tensor, cfg: MLRConfig, num_topics: int,
          dim: int) -> Dict[str, object]:
    """X: local CSR rows [n_local, dim]; Y: local 0/1 label matrix [n_local, num_topics].
    Returns the full model W [num_topics, dim+1] on every worker plus timings."""
    P, me, dev = comm.world_size, comm.rank, comm.device
    tps = math.ceil(num_topics / P)
    Tp = tps * P
    Yp = torch.zeros((Y.shape[0], Tp), dtype=torch.float32, device=dev)
    Yp[:, :num_topics] = Y.to(dev)
    X = X.to(dev)
    # regroup: worker r owns topics [r*tps, (r+1)*tps) (contiguous blocks; Partitioner
    # semantics up to a relabeling of topic ids)
    slab = torch.zeros((tps, dim + 1), dtype=torch.float64, device=dev)
    rot = DeviceRotator(comm, [slab], name="mlr-w")
    sched = RotationSchedule(P, None)
    t0 = time.perf_counter()
    for it in range(cfg.iterations):
        for s in range(P):
            blk = sched.block_at(me, it, s)
            W = rot.get(0)
            _sgd_pass(W, X, Yp[:, blk * tps:(blk + 1) * tps], cfg.alpha, cfg.batch_size)
            rot.start(0, sched.rotation_map(it, s))
    rot.wait_all()
    # after ITER*P ring steps every slab is back at its owner
    W_all = gather_rows(comm, rot.slabs[0])
    blocks = [sched.block_at(r, cfg.iterations, 0) for r in range(P)]
    order = torch.empty(Tp, dtype=torch.long)
    for r, blk in enumerate(blocks):
        order[blk * tps:(blk + 1) * tps] = torch.arange(r * tps, (r + 1) * tps)
    W_full = W_all[order.to(W_all.device)][:num_topics]
    return {"W": W_full, "train_s": time.perf_counter() - t0}


def evaluate(comm: Communicator, X: CSRRows, Y: torch.Tensor, W: torch.Tensor, threshold: float = 0.5) -> Dict:
    """Per-topic TP/FP/FN summed over all workers; micro/macro F1 (EVtask + outputEval)."""
    X = X.to(W.device)
    S = X.matmul_t(W[:, 1:], 0, X.nrows) + W[:, 0]
    pred = torch.sigmoid(S) > threshold
    lab = Y.to(W.device) > 0.5
    tp = (pred & lab).sum(0).double()
    fp = (pred & ~lab).sum(0).double()
    fn = (~pred & lab).sum(0).double()
    c = reduce_partials(comm, {"tp": tp, "fp": fp, "fn": fn})
    tp, fp, fn = c["tp"], c["fp"], c["fn"]
    prec = tp / (tp + fp).clamp_min(1)
    rec = tp / (tp + fn).clamp_min(1)
    f1 = 2 * prec * rec / (prec + rec).clamp_min(1e-12)
    T = tp.sum()
    micro_p = T / (T + fp.sum()).clamp_min(1)
    micro_r = T / (T + fn.sum()).clamp_min(1)
    micro_f1 = float(2 * micro_p * micro_r / (micro_p + micro_r).clamp_min(1e-12))
    return {"tp": tp, "fp": fp, "fn": fn, "precision": prec, "recall": rec, "f1": f1,
            "macro_f1": float(f1.mean()), "micro_f1": micro_f1}


def synthetic_multilabel(n: int, dim: int, topics: int, density: float = 0.02, seed: int = 0):
    """rcv1-shaped synthetic data: sparse tf-idf-like rows, topics defined by hidden
    linear scorers (a row carries topic t when its score is in the top quantile)."""
    g = torch.Generator().manual_seed(seed)
    mask = torch.rand(n, dim, generator=g) < density
    X = torch.rand(n, dim, generator=g) * mask
    X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-9)
    V = torch.randn(topics, dim, generator=g)
    S = X @ V.t()
    Y = (S > S.quantile(0.85, dim=0)).float()
    return X, Y
