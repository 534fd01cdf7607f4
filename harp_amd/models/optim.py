"""Optimization solvers and sum-of-functions objectives (DAAL ``optimization_solver``).

Reference: ml/daal/.../daal_optimization_solver/{sgd, sgd-mini, sgd-momentum, adagrad,
lbfgs, mse, opt variants}: a solver minimises F(x) = sum_i f_i(x) given by an objective
(MSE of a linear model; logistic / cross-entropy loss), with ``nIterations``,
``accuracyThreshold``, ``batchSize``, a learning-rate sequence, and ``batchIndices`` for
stochastic draws; results are ``minimum`` and ``nIterations``.

MI355X design: objectives evaluate value/gradient of the whole (or sampled) local block
with GEMMs; in a distributed run each worker holds a row shard and the gradient of the
sampled batch is summed across workers with ONE allreduce per step (synchronous
data-parallel), so every worker follows the same trajectory.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

import torch

from ..ops import linalg as LA

from ..parallel.comm import Communicator
from .common import reduce_partials


# ---------------------------------------------------------------- objectives
class Objective:
    """Sum over the rows of (X, y) of a per-row loss of the argument ``x``.
    ``value_grad(x, idx)`` evaluates the (global when ``comm`` is set) sum over the
    rows ``idx`` (local indices; None = all rows), divided by the global row count of
    the batch (DAAL normalises by the batch size)."""

    def __init__(self, X: torch.Tensor, y: torch.Tensor, comm: Optional[Communicator] = None, l2: float = 0.0,
                 intercept: bool = True):
        self.X, self.y, self.comm, self.l2, self.intercept = X, y, comm, l2, intercept
        self.n_local = X.shape[0]

    @property
    def dim(self) -> int:
        return self._dim()

    def _dim(self) -> int:
        return self.X.shape[1] + (1 if self.intercept else 0)

    def _lin(self, x, Xb):
        # x layout: [b0, b1..bp] (intercept first, as DAAL's linear model argument)
        if self.intercept:
            return Xb @ x[1:] + x[0]
        return Xb @ x

    def _local(self, x, idx):
        raise NotImplementedError

    def value_grad(self, x: torch.Tensor, idx: Optional[torch.Tensor] = None):
        v, g, n = self._local(x, idx)
        if self.comm is not None and self.comm.world_size > 1:
            r = reduce_partials(self.comm, {"v": v.reshape(1), "g": g, "n": torch.tensor([float(n)], dtype=g.dtype,
                                                                                         device=g.device)})
            v, g, n = r["v"][0].to(x.dtype), r["g"].to(x.dtype), float(r["n"][0])
        n = max(n, 1.0)
        v, g = v / n, g / n
        if self.l2:
            w = x[1:] if self.intercept else x
            v = v + self.l2 * (w * w).sum()
            gl = 2 * self.l2 * w
            g = g + (torch.cat([gl.new_zeros(1), gl]) if self.intercept else gl)
        return v, g

    def value(self, x, idx=None):
        return self.value_grad(x, idx)[0]


class MSE(Objective):
    """f_i = (x0 + x_{1..p} . X_i - y_i)^2 / 2 (daal mse)."""

    def _local(self, x, idx):
        Xb, yb = (self.X, self.y) if idx is None else (self.X[idx], self.y[idx])
        r = self._lin(x, Xb.to(x.dtype)) - yb.to(x.dtype).reshape(-1)
        gw = Xb.to(x.dtype).t() @ r
        g = torch.cat([r.sum().reshape(1), gw]) if self.intercept else gw
        return 0.5 * (r * r).sum(), g, Xb.shape[0]


class LogisticLoss(Objective):
    """Binary cross-entropy of sigmoid(x0 + x.X_i) against y_i in {0, 1} (daal logistic_loss)."""

    def _local(self, x, idx):
        Xb, yb = (self.X, self.y) if idx is None else (self.X[idx], self.y[idx])
        Xb, yb = Xb.to(x.dtype), yb.to(x.dtype).reshape(-1)
        z = self._lin(x, Xb)
        v = torch.nn.functional.binary_cross_entropy_with_logits(z, yb, reduction="sum")
        r = torch.sigmoid(z) - yb
        gw = Xb.t() @ r
        g = torch.cat([r.sum().reshape(1), gw]) if self.intercept else gw
        return v, g, Xb.shape[0]


class CrossEntropyLoss(Objective):
    """Multinomial cross-entropy; the argument is the flattened [K, p+1] coefficient
    matrix (intercept column first), y holds class ids (daal cross_entropy_loss)."""

    def __init__(self, X, y, num_classes: int, comm=None, l2: float = 0.0, intercept: bool = True):
        super().__init__(X, y, comm, l2, intercept)
        self.K = num_classes

    def _dim(self):
        return self.K * (self.X.shape[1] + (1 if self.intercept else 0))

    def _local(self, x, idx):
        Xb, yb = (self.X, self.y) if idx is None else (self.X[idx], self.y[idx])
        Xb = Xb.to(x.dtype)
        B = x.reshape(self.K, -1)
        Z = Xb @ B[:, 1:].t() + B[:, 0] if self.intercept else Xb @ B.t()
        yl = yb.long().reshape(-1)
        v = torch.nn.functional.cross_entropy(Z, yl, reduction="sum")
        R = torch.softmax(Z, 1)
        R[torch.arange(Xb.shape[0], device=Xb.device), yl] -= 1
        G = LA.atb(R, Xb)
        if self.intercept:
            G = torch.cat([R.sum(0)[:, None], G], 1)
        return v, G.reshape(-1), Xb.shape[0]

    def value_grad(self, x, idx=None):
        if not self.l2:
            return super().value_grad(x, idx)
        l2, self.l2 = self.l2, 0.0
        try:
            v, g = super().value_grad(x, idx)
        finally:
            self.l2 = l2
        B = x.reshape(self.K, -1)
        W = B[:, 1:] if self.intercept else B
        gW = torch.zeros_like(B)
        if self.intercept:
            gW[:, 1:] = 2 * l2 * W
        else:
            gW = 2 * l2 * W
        return v + l2 * (W * W).sum(), g + gW.reshape(-1)


# ---------------------------------------------------------------- solvers
@dataclass
class SolverResult:
    minimum: torch.Tensor
    n_iterations: int
    value: float


def _lr(seq, k):
    if callable(seq):
        return float(seq(k))
    if isinstance(seq, (list, tuple)):
        return float(seq[min(k, len(seq) - 1)])
    return float(seq)


class _Sampler:
    """Shared batch-index stream: the same seed on every worker, drawing local indices
    (each worker samples its own shard — the global batch is P * batch_size rows)."""

    def __init__(self, n: int, batch: int, seed: int, device, batch_indices=None):
        self.n, self.batch, self.dev, self.fixed = n, batch, device, batch_indices
        self.g = torch.Generator().manual_seed(seed)

    def __call__(self, k):
        if self.fixed is not None:
            return torch.as_tensor(self.fixed[k % len(self.fixed)], device=self.dev).long().reshape(-1)
        if self.batch >= self.n:
            return None
        return torch.randint(0, self.n, (self.batch,), generator=self.g).to(self.dev)


def sgd(obj: Objective, x0: Optional[torch.Tensor] = None, n_iterations: int = 1000, learning_rate=0.01,
        batch_size: int = 1, accuracy_threshold: float = 0.0, momentum: float = 0.0, seed: int = 0,
        batch_indices: Optional[Sequence] = None, conservative_sequence=None, inner_iterations: int = 1,
        dtype=torch.float64) -> SolverResult:
    """SGD family: ``batch_size=1`` -> daal sgd defaultDense; ``batch_size>1`` ->
    miniBatch (optionally with ``conservative_sequence`` proximal term and
    ``inner_iterations``); ``momentum>0`` -> momentum method. Stops when the relative
    step ||x_{k+1}-x_k|| / max(1, ||x_k||) falls below ``accuracy_threshold``."""
    dev = obj.X.device
    x = (torch.zeros(obj.dim, dtype=dtype, device=dev) if x0 is None else x0.to(dev, dtype).clone())
    v = torch.zeros_like(x)
    sample = _Sampler(obj.n_local, batch_size, seed, dev, batch_indices)
    k = 0
    for k in range(n_iterations):
        idx = sample(k)
        lr = _lr(learning_rate, k)
        x_prev = x.clone()
        anchor = x.clone()
        gamma = _lr(conservative_sequence, k) if conservative_sequence is not None else 0.0
        for _ in range(max(1, inner_iterations)):
            _, g = obj.value_grad(x, idx)
            if gamma:
                g = g + gamma * (x - anchor)
            if momentum:
                v = momentum * v + lr * g
                x = x - v
            else:
                x = x - lr * g
        if accuracy_threshold and float((x - x_prev).norm()) / max(1.0, float(x_prev.norm())) < accuracy_threshold:
            break
    return SolverResult(x, k + 1, float(obj.value(x)))


def adagrad(obj: Objective, x0=None, n_iterations: int = 1000, learning_rate=0.1, batch_size: int = 1,
            degenerate_cases_threshold: float = 1e-8, accuracy_threshold: float = 0.0, seed: int = 0,
            batch_indices=None, dtype=torch.float64) -> SolverResult:
    """AdaGrad: G += g^2; x -= lr g / sqrt(G + eps) (daal adagrad)."""
    dev = obj.X.device
    x = torch.zeros(obj.dim, dtype=dtype, device=dev) if x0 is None else x0.to(dev, dtype).clone()
    G = torch.zeros_like(x)
    sample = _Sampler(obj.n_local, batch_size, seed, dev, batch_indices)
    k = 0
    for k in range(n_iterations):
        _, g = obj.value_grad(x, sample(k))
        if accuracy_threshold and float(g.norm()) < accuracy_threshold:
            break
        G += g * g
        x = x - _lr(learning_rate, k) * g / torch.sqrt(G + degenerate_cases_threshold)
    return SolverResult(x, k + 1, float(obj.value(x)))


def lbfgs(obj: Objective, x0=None, n_iterations: int = 100, m: int = 10, accuracy_threshold: float = 1e-8,
          batch_size: Optional[int] = None, step_length: Optional[float] = None, seed: int = 0,
          dtype=torch.float64) -> SolverResult:
    """L-BFGS two-loop recursion. Full-batch with Armijo backtracking by default;
    ``batch_size`` + fixed ``step_length`` gives the stochastic variant DAAL ships."""
    dev = obj.X.device
    x = torch.zeros(obj.dim, dtype=dtype, device=dev) if x0 is None else x0.to(dev, dtype).clone()
    sample = _Sampler(obj.n_local, batch_size or obj.n_local, seed, dev)
    S, Y = [], []
    idx = sample(0)
    f, g = obj.value_grad(x, idx)
    k = 0
    for k in range(n_iterations):
        if float(g.norm()) < accuracy_threshold:
            break
        q = g.clone()
        al = []
        for s, y in reversed(list(zip(S, Y))):
            a = (s @ q) / (y @ s)
            al.append(a)
            q = q - a * y
        if S:
            q = q * ((S[-1] @ Y[-1]) / (Y[-1] @ Y[-1]))
        for (s, y), a in zip(zip(S, Y), reversed(al)):
            b = (y @ q) / (y @ s)
            q = q + s * (a - b)
        d = -q
        if step_length is not None:
            t = step_length
            xn = x + t * d
            fn, gn = obj.value_grad(xn, idx)
        else:
            t, gd = 1.0, float(g @ d)
            if gd >= 0:
                d, gd = -g, -float(g @ g)
            while True:
                xn = x + t * d
                fn, gn = obj.value_grad(xn, idx)
                if float(fn) <= float(f) + 1e-4 * t * gd or t < 1e-12:
                    break
                t *= 0.5
        if batch_size:
            idx = sample(k + 1)
            fn, gn = obj.value_grad(xn, idx)
        s, y = xn - x, gn - g
        if float(s @ y) > 1e-12:
            S.append(s), Y.append(y)
            if len(S) > m:
                S.pop(0), Y.pop(0)
        x, f, g = xn, fn, gn
    return SolverResult(x, k + 1, float(obj.value(x)))


SOLVERS: dict = {"sgd": sgd, "adagrad": adagrad, "lbfgs": lbfgs}
