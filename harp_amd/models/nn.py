"""Multi-layer perceptron training: periodic model averaging and synchronous SGD.

Reference: contrib/src/main/java/edu/iu/NN/NNMapper.java:138-185 + HarpNeuralNetwork.java
(jblas MLP with sigmoid units; every mapper trains mini-batches locally for
``syncIterNum`` steps, then the weight table is allreduced and divided by P — local-SGD
/ model averaging) and ml/daal/.../daal_nn/NNDaalCollectiveMapper.java (DAAL
``neural_networks`` fully-connected + softmax-cross-entropy topology with an SGD
solver: distributed step 1 computes the local gradient, the master sums them, updates
and broadcasts the model — synchronous data-parallel SGD).

MI355X design: all weights and biases live in ONE flat fp32 device buffer with per-layer
views, so a model average or a gradient sum is ONE allreduce of one contiguous buffer
(a single-partition PackedTable) instead of a table of per-layer partitions; forward
and backward are explicit GEMMs (hipBLASLt) with the activation derivative fused into
the backward GEMM's input (no autograd graph on the hot path).
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..core.combiner import ArrCombiner, Operation
from ..core.table import PackedTable
from ..parallel import collectives as CL
from ..parallel.comm import Communicator

_ACT = {
    "sigmoid": (torch.sigmoid, lambda a: a * (1 - a)),
    "tanh": (torch.tanh, lambda a: 1 - a * a),
    "relu": (torch.relu, lambda a: (a > 0).to(a.dtype)),
}


class MLP:
    """Fully-connected network ``sizes[0] -> ... -> sizes[-1]`` with a softmax /
    cross-entropy output (or sigmoid / squared error with ``output='sigmoid'``, as the
    contrib jblas net)."""

    def __init__(self, sizes: Sequence[int], activation: str = "sigmoid", output: str = "softmax",
                 device="cpu", dtype=torch.float32, seed: int = 0):
        self.sizes, self.act, self.output = list(sizes), activation, output
        shapes = []
        for a, b in zip(sizes[:-1], sizes[1:]):
            shapes += [(b, a), (b,)]
        self.numel = sum(math.prod(s) for s in shapes)
        self.flat = torch.zeros(self.numel, dtype=dtype, device=device)
        self.params: List[torch.Tensor] = []
        o = 0
        for s in shapes:
            n = math.prod(s)
            self.params.append(self.flat[o:o + n].view(s))
            o += n
        g = torch.Generator().manual_seed(seed)
        for W in self.params[0::2]:
            lim = math.sqrt(6.0 / (W.shape[0] + W.shape[1]))
            W.copy_((torch.rand(W.shape, generator=g) * 2 - 1) * lim)

    def forward(self, X: torch.Tensor) -> List[torch.Tensor]:
        f, _ = _ACT[self.act]
        acts = [X.to(self.flat.dtype)]
        L = len(self.params) // 2
        for l in range(L):
            W, b = self.params[2 * l], self.params[2 * l + 1]
            z = torch.addmm(b, acts[-1], W.t())
            if l < L - 1:
                acts.append(f(z))
            else:
                acts.append(torch.softmax(z, 1) if self.output == "softmax" else torch.sigmoid(z))
        return acts

    def predict_proba(self, X):
        return self.forward(X)[-1]

    def predict(self, X):
        return self.predict_proba(X).argmax(1)

    def _native(self, X) -> bool:
        from ..ops import nn as NO

        return self.output == "softmax" and NO.available(self.flat) and X.device == self.flat.device

    def _gradient_native(self, X: torch.Tensor, labels: torch.Tensor, s: float) -> torch.Tensor:
        """GPU path: GEMMs on hipBLASLt, every epilogue one fused pass (csrc/nn.hip):
        bias + activation, softmax-xent forward + backward + output bias gradient, and the
        activation derivative + hidden bias gradient."""
        from ..ops import nn as NO

        L = len(self.params) // 2
        acts = [X.to(self.flat.dtype).contiguous()]
        for l in range(L - 1):
            z = torch.mm(acts[-1], self.params[2 * l].t())
            acts.append(NO.bias_act_(z, self.params[2 * l + 1], self.act))
        logits = torch.addmm(self.params[-1], acts[-1], self.params[-2].t())
        grad = torch.zeros_like(self.flat)  # bias slots accumulate
        gp, o = [], 0
        for p in self.params:
            gp.append(grad[o:o + p.numel()].view(p.shape))
            o += p.numel()
        delta = torch.empty_like(logits)
        self.last_loss = NO.softmax_xent(logits, labels, s, delta, gp[-1])
        for l in reversed(range(L)):
            torch.mm(delta.t(), acts[l], out=gp[2 * l])  # delta already carries the scale
            if l:
                delta = delta @ self.params[2 * l]
                NO.dact_bgrad_(delta, acts[l], self.act, gp[2 * l - 1])
        return grad

    def gradient(self, X: torch.Tensor, Y: torch.Tensor, scale: Optional[float] = None) -> torch.Tensor:
        """Flat gradient of the summed loss over the batch (times ``scale``, default 1/b);
        Y is one-hot [b, C] (or int class labels [b])."""
        b = X.shape[0]
        s = (1.0 / b) if scale is None else scale
        if self._native(X):
            labels = (Y.argmax(1) if Y.dim() == 2 else Y).to(torch.int32).contiguous()
            return self._gradient_native(X, labels, s)
        if Y.dim() == 1:
            Y = torch.nn.functional.one_hot(Y.long(), self.sizes[-1])
        _, df = _ACT[self.act]
        acts = self.forward(X)
        grad = torch.empty_like(self.flat)
        gp = []
        o = 0
        for p in self.params:
            gp.append(grad[o:o + p.numel()].view(p.shape))
            o += p.numel()
        out = acts[-1]
        delta = out - Y.to(out.dtype)
        if self.output != "softmax":  # squared error through the sigmoid
            delta = delta * out * (1 - out)
        L = len(self.params) // 2
        for l in reversed(range(L)):
            torch.mm(delta.t(), acts[l], out=gp[2 * l])
            gp[2 * l].mul_(s)
            torch.sum(delta, 0, out=gp[2 * l + 1])
            gp[2 * l + 1].mul_(s)
            if l:
                delta = (delta @ self.params[2 * l]) * df(acts[l])
        return grad

    def loss(self, X, Y) -> float:
        p = self.predict_proba(X).clamp(1e-12, 1)
        if self.output == "softmax":
            return float(-(Y.to(p.dtype) * p.log()).sum(1).mean())
        return float(0.5 * ((p - Y.to(p.dtype)) ** 2).sum(1).mean())


def _flat_table(buf: torch.Tensor) -> PackedTable:
    t = PackedTable([0], buf.view(1, -1), combiner=ArrCombiner(Operation.SUM))
    t.static_layout = True
    return t


def _allreduce_mean(comm: Communicator, buf: torch.Tensor) -> None:
    if comm.world_size == 1:
        return
    dev_buf = buf if buf.device == comm.device else buf.to(comm.device)
    if not CL.allreduce(comm, _flat_table(dev_buf)):
        raise IOError("NN allreduce failed")
    dev_buf.div_(comm.world_size)
    if dev_buf is not buf:
        buf.copy_(dev_buf)


def _batches(n: int, batch: int, g: torch.Generator):
    perm = torch.randperm(n, generator=g)
    for a in range(0, n, batch):
        yield perm[a:a + batch]


def train_model_averaging(comm: Communicator, net: MLP, X, Y, epochs: int = 5, batch: int = 64, lr: float = 0.5,
                          sync_iters: int = 10, seed: int = 0) -> Dict[str, object]:
    """contrib NN: ``sync_iters`` local mini-batch steps, then average the weights."""
    _allreduce_mean(comm, net.flat)  # identical start (the reference broadcasts the init)
    g = torch.Generator().manual_seed(seed + comm.rank)
    step, syncs = 0, 0
    t0 = time.perf_counter()
    for _ in range(epochs):
        for idx in _batches(X.shape[0], batch, g):
            idx = idx.to(X.device)
            net.flat.sub_(lr * net.gradient(X[idx], Y[idx]))
            step += 1
            if step % sync_iters == 0:
                _allreduce_mean(comm, net.flat)
                syncs += 1
    _allreduce_mean(comm, net.flat)
    return {"steps": step, "syncs": syncs + 1, "train_s": time.perf_counter() - t0}


def train_sync_sgd(comm: Communicator, net: MLP, X, Y, epochs: int = 5, batch: int = 64, lr: float = 0.5,
                   seed: int = 0, momentum: float = 0.0) -> Dict[str, object]:
    """DAAL NN distributed: every step each worker's batch gradient is summed (one
    allreduce of the flat gradient) and every worker applies the same update. The
    global batch is P * batch."""
    _allreduce_mean(comm, net.flat)
    g = torch.Generator().manual_seed(seed + comm.rank)
    # all workers take the same number of steps per epoch
    n_local = torch.tensor([X.shape[0]], dtype=torch.float64)
    from .common import reduce_partials

    n_min = int(reduce_partials(comm, {"n": n_local}, op=Operation.MIN)["n"][0])
    steps_per_epoch = max(1, n_min // batch)
    vel = torch.zeros_like(net.flat) if momentum else None
    step = 0
    t0 = time.perf_counter()
    for _ in range(epochs):
        it = _batches(X.shape[0], batch, g)
        for _ in range(steps_per_epoch):
            idx = next(it).to(X.device)
            gr = net.gradient(X[idx], Y[idx])
            _allreduce_mean(comm, gr)
            if momentum:
                vel.mul_(momentum).add_(gr, alpha=lr)
                net.flat.sub_(vel)
            else:
                net.flat.sub_(lr * gr)
            step += 1
    return {"steps": step, "train_s": time.perf_counter() - t0}
