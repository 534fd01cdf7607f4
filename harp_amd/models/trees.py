"""Decision trees, decision forests and boosting.

Reference: ml/daal batch algorithms ``daal_dtree`` (classification / regression, plus
"traverse" variants that walk the trained model), ``daal_dforest`` (classification /
regression forests), ``daal_stump``, ``daal_adaboost``, ``daal_brownboost``,
``daal_logitboost``; contrib random forests (contrib/.../randomforest, rf, com/rf/fast:
per-mapper trees on local data, predictions combined by vote through allreduce / reduce).

MI355X design: trees grow level-wise with histogram split search: features are quantile-
binned once, then per level ONE scatter-add builds (node, feature, bin) histograms of the
class counts (or gradient sums), a cumulative sum over bins scores every candidate split
of every node at once, and samples are re-routed with a gather — no per-node host loops
over samples, so the same code runs on CPU (gloo tests) and on the GPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from ..core.writable import DataInput, DataOutput, Writable
from ..parallel.comm import Communicator


def _bins(X: torch.Tensor, n_bins: int) -> torch.Tensor:
    """Per-feature quantile thresholds [d, n_bins-1]."""
    q = torch.linspace(0, 1, n_bins + 1, dtype=torch.float64, device=X.device)[1:-1]
    Xs = X.double()
    if Xs.shape[0] > 200000:
        idx = torch.randint(0, Xs.shape[0], (200000,), device=X.device)
        Xs = Xs[idx]
    return torch.quantile(Xs, q, dim=0).t().contiguous()


class DecisionTree(Writable):
    """CART tree. ``task``: "classification" (gini / entropy) or "regression" (mse)."""

    def __init__(self, task: str = "classification", max_depth: int = 8, min_samples_leaf: int = 1,
                 max_features=None, n_bins: int = 64, criterion: str = "gini", seed: int = 0):
        self.task, self.max_depth, self.min_leaf = task, max_depth, min_samples_leaf
        self.max_features, self.n_bins, self.criterion, self.seed = max_features, n_bins, criterion, seed
        self.feature = torch.empty(0, dtype=torch.int64)
        self.threshold = torch.empty(0, dtype=torch.float64)
        self.left = torch.empty(0, dtype=torch.int64)
        self.value = torch.empty(0, 0, dtype=torch.float64)

    # ---------------------------------------------------------------- training
    def fit(self, X: torch.Tensor, y: torch.Tensor, sample_weight: Optional[torch.Tensor] = None,
            num_classes: Optional[int] = None, thresholds: Optional[torch.Tensor] = None) -> "DecisionTree":
        dev = X.device
        n, d = X.shape
        w = torch.ones(n, dtype=torch.float64, device=dev) if sample_weight is None else sample_weight.double().to(dev)
        cls = self.task == "classification"
        if cls:
            C = int(num_classes or int(y.max()) + 1)
            stats = torch.nn.functional.one_hot(y.long().to(dev), C).double() * w[:, None]
        else:
            yd = y.double().to(dev).reshape(n)
            stats = torch.stack([w, w * yd, w * yd * yd], 1)
            C = 3
        th = thresholds if thresholds is not None else _bins(X, self.n_bins)
        B = th.shape[1] + 1
        Xb = torch.searchsorted(th, X.double().t().contiguous(), right=True).t()  # [n, d] bin ids
        gen = torch.Generator(device="cpu").manual_seed(self.seed)
        feats, thrs, lefts, vals = [], [], [], []
        node_of = torch.zeros(n, dtype=torch.int64, device=dev)
        frontier = [0]
        feats.append(-1), thrs.append(0.0), lefts.append(-1)
        vals.append(stats.sum(0))
        depth = 0
        while frontier and depth < self.max_depth:
            m = len(frontier)
            fmap = torch.full((len(feats),), -1, dtype=torch.int64, device=dev)
            fmap[torch.tensor(frontier, device=dev)] = torch.arange(m, device=dev)
            loc = fmap[node_of]
            act = loc >= 0
            if not bool(act.any()):
                break
            li, lx, ls = loc[act], Xb[act], stats[act]
            # histogram [m, d, B, C]
            H = torch.zeros((m * d * B, C), dtype=torch.float64, device=dev)
            idx = (li[:, None] * d + torch.arange(d, device=dev)[None, :]) * B + lx
            H.index_add_(0, idx.reshape(-1), ls[:, None, :].expand(-1, d, -1).reshape(-1, C))
            H = H.view(m, d, B, C)
            Lc = H.cumsum(2)[:, :, :-1, :]  # left = bins <= b
            tot = H.sum(2, keepdim=True)
            Rc = tot - Lc
            gain = self._gain(Lc, Rc, tot)
            # feature subsampling
            if self.max_features:
                k = self.max_features if isinstance(self.max_features, int) else max(1, int(math.sqrt(d)))
                mask = torch.full((m, d), float("-inf"), dtype=torch.float64, device=dev)
                for j in range(m):
                    sel = torch.randperm(d, generator=gen)[:k].to(dev)
                    mask[j, sel] = 0.0
                gain = gain + mask[:, :, None]
            nL = self._count(Lc)
            nR = self._count(Rc)
            gain = torch.where((nL >= self.min_leaf) & (nR >= self.min_leaf), gain, torch.full_like(gain, float("-inf")))
            flat = gain.reshape(m, -1)
            best, arg = flat.max(1)
            bf, bb = arg // (B - 1), arg % (B - 1)
            new_frontier = []
            split_nodes = []
            for j, node in enumerate(frontier):
                if best[j].item() > 1e-12:
                    f, b = int(bf[j]), int(bb[j])
                    feats[node], thrs[node] = f, float(th[f, b])
                    lefts[node] = len(feats)
                    for side in (Lc, Rc):
                        feats.append(-1), thrs.append(0.0), lefts.append(-1)
                        vals.append(side[j, f, b])
                    new_frontier += [lefts[node], lefts[node] + 1]
                    split_nodes.append((node, f, b))
            if not split_nodes:
                break
            # route samples of split nodes
            feat_t = torch.tensor(feats, device=dev)
            bin_t = torch.full((len(feats),), 0, dtype=torch.int64, device=dev)
            for node, f, b in split_nodes:
                bin_t[node] = b
            left_t = torch.tensor(lefts, device=dev)
            is_split = left_t[node_of] >= 0
            fsel = feat_t[node_of].clamp_min(0)
            go_right = Xb.gather(1, fsel[:, None])[:, 0] > bin_t[node_of]
            node_of = torch.where(is_split, left_t[node_of] + go_right.long(), node_of)
            frontier = new_frontier
            depth += 1
        self.feature = torch.tensor(feats, dtype=torch.int64)
        self.threshold = torch.tensor(thrs, dtype=torch.float64)
        self.left = torch.tensor(lefts, dtype=torch.int64)
        V = torch.stack(vals).cpu()
        if cls:
            self.value = V / V.sum(1, keepdim=True).clamp_min(1e-300)
        else:
            self.value = (V[:, 1] / V[:, 0].clamp_min(1e-300))[:, None]
        return self

    def _count(self, S):
        return S.sum(-1) if self.task == "classification" else S[..., 0]

    def _impurity(self, S):
        if self.task == "classification":
            n = S.sum(-1, keepdim=True).clamp_min(1e-300)
            p = S / n
            if self.criterion == "entropy":
                return -(p * torch.log2(p.clamp_min(1e-300))).sum(-1) * n[..., 0]
            return (1 - (p * p).sum(-1)) * n[..., 0]
        w, s, ss = S[..., 0], S[..., 1], S[..., 2]
        return ss - s * s / w.clamp_min(1e-300)

    def _gain(self, L, R, T):
        return self._impurity(T) - self._impurity(L) - self._impurity(R)

    # ---------------------------------------------------------------- inference
    def apply(self, X: torch.Tensor) -> torch.Tensor:
        """Leaf index of every sample (the DAAL "traverse" variants walk the same arrays)."""
        dev = X.device
        f, t, l = self.feature.to(dev), self.threshold.to(dev), self.left.to(dev)
        node = torch.zeros(X.shape[0], dtype=torch.int64, device=dev)
        Xd = X.double()
        for _ in range(self.max_depth + 1):
            lf = l[node]
            inner = lf >= 0
            if not bool(inner.any()):
                break
            xv = Xd.gather(1, f[node].clamp_min(0)[:, None])[:, 0]
            node = torch.where(inner, lf + (xv >= t[node]).long(), node)  # training: left <=> x < thr
        return node

    def predict_proba(self, X: torch.Tensor) -> torch.Tensor:
        return self.value.to(X.device)[self.apply(X)]

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        v = self.predict_proba(X)
        return v.argmax(1) if self.task == "classification" else v[:, 0]

    # ---------------------------------------------------------------- wire format
    def write(self, out: DataOutput) -> None:
        out.write_utf(self.task)
        out.write_int(self.max_depth)
        out.write_int(self.feature.numel())
        out.write_int(self.value.shape[1])
        for i in range(self.feature.numel()):
            out.write_int(int(self.feature[i]))
            out.write_double(float(self.threshold[i]))
            out.write_int(int(self.left[i]))
            for v in self.value[i].tolist():
                out.write_double(v)

    def read(self, inp: DataInput) -> None:
        self.task = inp.read_utf()
        self.max_depth = inp.read_int()
        n, c = inp.read_int(), inp.read_int()
        f, t, l, v = [], [], [], []
        for _ in range(n):
            f.append(inp.read_int())
            t.append(inp.read_double())
            l.append(inp.read_int())
            v.append([inp.read_double() for _ in range(c)])
        self.feature = torch.tensor(f, dtype=torch.int64)
        self.threshold = torch.tensor(t, dtype=torch.float64)
        self.left = torch.tensor(l, dtype=torch.int64)
        self.value = torch.tensor(v, dtype=torch.float64).reshape(n, c)


class DecisionForest:
    """Random forest: bootstrap rows + sqrt(d) features per split. ``fit_distributed``
    trains ``n_trees / P`` trees per worker on its local rows and all-gathers the trees
    (the contrib RF combines per-mapper trees the same way)."""

    def __init__(self, task="classification", n_trees=50, max_depth=10, max_features="sqrt", n_bins=64, seed=0,
                 min_samples_leaf=1):
        self.task, self.n_trees, self.max_depth = task, n_trees, max_depth
        self.max_features, self.n_bins, self.seed, self.min_leaf = max_features, n_bins, seed, min_samples_leaf
        self.trees: List[DecisionTree] = []
        self.num_classes = None

    def fit(self, X, y, num_classes=None, n_trees=None, seed_offset=0):
        n = X.shape[0]
        self.num_classes = num_classes or (int(y.max()) + 1 if self.task == "classification" else None)
        th = _bins(X, self.n_bins)
        g = torch.Generator().manual_seed(self.seed + seed_offset)
        for t in range(n_trees or self.n_trees):
            idx = torch.randint(0, n, (n,), generator=g).to(X.device)
            w = torch.bincount(idx, minlength=n).double()
            tree = DecisionTree(self.task, self.max_depth, self.min_leaf, self.max_features, self.n_bins,
                                seed=self.seed * 1000 + seed_offset + t)
            self.trees.append(tree.fit(X, y, sample_weight=w, num_classes=self.num_classes, thresholds=th))
        return self

    def fit_distributed(self, X, y, comm: Communicator, num_classes=None):
        from ..parallel.partition_util import allgather_objects

        P, r = comm.world_size, comm.rank
        mine = self.n_trees // P + (1 if r < self.n_trees % P else 0)
        self.fit(X, y, num_classes, n_trees=mine, seed_offset=7919 * r)
        self.trees = allgather_objects(comm, self.trees)
        return self

    def predict_proba(self, X):
        return torch.stack([t.predict_proba(X) for t in self.trees]).mean(0)

    def predict(self, X):
        p = self.predict_proba(X)
        return p.argmax(1) if self.task == "classification" else p[:, 0]


# ---------------------------------------------------------------- boosting
def stump(X, y, sample_weight=None, num_classes=None, task="classification"):
    """Decision stump (daal_stump): a depth-1 tree."""
    return DecisionTree(task, max_depth=1, n_bins=256).fit(X, y, sample_weight, num_classes)


class AdaBoost:
    """Multi-class AdaBoost (SAMME) with stumps (daal_adaboost)."""

    def __init__(self, n_rounds=50, learner_depth=1):
        self.n_rounds, self.depth = n_rounds, learner_depth
        self.learners, self.alphas = [], []

    def fit(self, X, y, num_classes=None):
        K = num_classes or int(y.max()) + 1
        n = X.shape[0]
        w = torch.full((n,), 1.0 / n, dtype=torch.float64, device=X.device)
        yl = y.long().to(X.device)
        self.K = K
        for _ in range(self.n_rounds):
            h = DecisionTree("classification", self.depth, n_bins=256).fit(X, yl, w * n, K)
            miss = (h.predict(X) != yl).double()
            err = float((w * miss).sum() / w.sum())
            if err >= 1 - 1.0 / K:
                break
            a = math.log((1 - err) / max(err, 1e-12)) + math.log(K - 1)
            self.learners.append(h)
            self.alphas.append(a)
            w = w * torch.exp(a * miss)
            w = w / w.sum()
            if err < 1e-12:
                break
        return self

    def decision(self, X):
        S = torch.zeros((X.shape[0], self.K), dtype=torch.float64, device=X.device)
        for h, a in zip(self.learners, self.alphas):
            S[torch.arange(X.shape[0], device=X.device), h.predict(X)] += a
        return S

    def predict(self, X):
        return self.decision(X).argmax(1)


class BrownBoost:
    """Binary BrownBoost (Freund 2001; daal_brownboost): boosting in continuous time with
    a total time budget ``c``. Each round picks the weak learner on weights
    exp(-(r_i + s)^2 / c), then solves for the step (alpha, t): t(alpha) keeps the total
    potential sum_i (1 - erf((r_i + s) / sqrt(c))) constant, alpha zeroes the weighted
    correlation of the learner after the step (both by bisection: robust also when the
    weak learner is nearly perfect). Stops when the remaining time s reaches 0."""

    def __init__(self, c: float = 2.0, max_rounds: int = 100, nu: float = 1e-3, newton_iters: int = 60):
        self.c, self.max_rounds, self.nu, self.iters = c, max_rounds, nu, newton_iters
        self.learners, self.alphas = [], []

    def _pot(self, z):
        return (1 - torch.erf(z / math.sqrt(self.c))).sum()

    def fit(self, X, y):
        yl = y.long().to(X.device)
        ys = (2 * yl - 1).double()  # {-1, +1}
        r = torch.zeros(X.shape[0], dtype=torch.float64, device=X.device)
        s = self.c
        for _ in range(self.max_rounds):
            if s <= 1e-9:
                break
            w = torch.exp(-(r + s) ** 2 / self.c)
            h = DecisionTree("classification", 1, n_bins=256).fit(X, yl, w / w.sum() * X.shape[0], 2)
            u = (2 * h.predict(X) - 1).double() * ys
            if float((w * u).sum()) <= 0:
                break
            target = self._pot(r + s)

            def t_of(a):
                lo, hi = 0.0, s
                if float(self._pot(r + s - hi + a * u)) <= float(target):
                    return hi
                for _ in range(self.iters):
                    mid = 0.5 * (lo + hi)
                    if float(self._pot(r + s - mid + a * u)) < float(target):
                        lo = mid
                    else:
                        hi = mid
                return 0.5 * (lo + hi)

            def corr(a):
                t = t_of(a)
                z = r + s - t + a * u
                return float((torch.exp(-z * z / self.c) * u).sum()), t

            a_lo, a_hi = 0.0, 1.0
            g_hi, t_hi = corr(a_hi)
            while g_hi > 0 and t_hi < s and a_hi < 1e3:
                a_lo, a_hi = a_hi, a_hi * 2
                g_hi, t_hi = corr(a_hi)
            if g_hi > 0:  # time runs out before the correlation vanishes
                a, t = a_hi, t_hi
            else:
                for _ in range(self.iters):
                    mid = 0.5 * (a_lo + a_hi)
                    g, _t = corr(mid)
                    if g > 0:
                        a_lo = mid
                    else:
                        a_hi = mid
                    if a_hi - a_lo < self.nu * 1e-3:
                        break
                a = 0.5 * (a_lo + a_hi)
                t = t_of(a)
            r = r + a * u
            s -= max(t, self.nu)
            self.learners.append(h)
            self.alphas.append(a)
        return self

    def decision(self, X):
        out = torch.zeros(X.shape[0], dtype=torch.float64, device=X.device)
        for h, a in zip(self.learners, self.alphas):
            out += a * (2 * h.predict(X) - 1).double()
        return out

    def predict(self, X):
        return (self.decision(X) > 0).long()


class LogitBoost:
    """Multi-class LogitBoost (Friedman, Hastie & Tibshirani 2000; daal_logitboost) with
    regression stumps fit to the Newton working responses."""

    def __init__(self, n_rounds=50, depth=1, zmax=4.0):
        self.n_rounds, self.depth, self.zmax = n_rounds, depth, zmax
        self.rounds: List[List[DecisionTree]] = []

    def fit(self, X, y, num_classes=None):
        K = num_classes or int(y.max()) + 1
        self.K = K
        n = X.shape[0]
        Y = torch.nn.functional.one_hot(y.long().to(X.device), K).double()
        F = torch.zeros((n, K), dtype=torch.float64, device=X.device)
        th = _bins(X, 256)
        for _ in range(self.n_rounds):
            Pm = torch.softmax(F, 1)
            fs = []
            for k in range(K):
                p = Pm[:, k]
                w = (p * (1 - p)).clamp_min(1e-12)
                z = ((Y[:, k] - p) / w).clamp(-self.zmax, self.zmax)
                fs.append(DecisionTree("regression", self.depth, n_bins=256).fit(X, z, w, thresholds=th))
            G = torch.stack([f.predict(X) for f in fs], 1)
            G = (K - 1) / K * (G - G.mean(1, keepdim=True))
            F = F + G
            self.rounds.append(fs)
        return self

    def decision(self, X):
        F = torch.zeros((X.shape[0], self.K), dtype=torch.float64, device=X.device)
        for fs in self.rounds:
            G = torch.stack([f.predict(X) for f in fs], 1)
            F += (self.K - 1) / self.K * (G - G.mean(1, keepdim=True))
        return F

    def predict(self, X):
        return self.decision(X).argmax(1)
