"""Kernel functions, kNN and EM for Gaussian mixtures.

Reference: ml/daal/.../daal_kernel_func/{LinDenseBatch, LinCSRBatch, RbfDenseBatch,
RbfCSRBatch} (linear ``k X Y^T + b``; RBF ``exp(-||x-y||^2 / (2 sigma^2))``),
daal_knn (kd-tree kNN classifier, batch), daal_em (EM-GMM, batch, full covariance with
``covariance_storage``, ``nIterations`` and ``accuracyThreshold``).

MI355X design: all three are GEMM-shaped. Pairwise work goes through one matmul of the
row blocks (hipBLASLt) with the norm terms fused into its epilogue (``addmm`` of the
-2 X Y^T product onto the broadcast norms), so the N x M distance matrix is produced in
one pass; kNN tiles the query set and keeps a running top-k per tile (no N x M
materialisation for large M); distributed kNN selects the local top-k on each
training shard and merges the P candidates with one all-gather. EM on the GPU runs the
fused HIP E-step (``ops.gmm``: whitened Mahalanobis for all components in registers +
LDS, log-sum-exp responsibilities in the same kernel) and one GEMM-shaped statistics pass
(N_k, sum r x, sum r x x^T from the augmented point); on the CPU the E-step is one
batched triangular solve per component. Either way the sufficient statistics are ONE
allreduce per iteration.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch

from ..ops import _lib

from ..ops import linalg as LA

from ..parallel.comm import Communicator
from .common import reduce_partials


def _dense(X):
    return X.to_dense() if (X.is_sparse or X.layout in (torch.sparse_csr, torch.sparse_csc)) else X


def _mm_t(X, Y):
    """X @ Y^T for dense or sparse X / Y."""
    if X.is_sparse or X.layout == torch.sparse_csr:
        return torch.sparse.mm(X, _dense(Y).t().contiguous())
    if Y.is_sparse or Y.layout == torch.sparse_csr:
        return torch.sparse.mm(Y, X.t().contiguous()).t()
    return X @ Y.t()


def _sqnorm(X):
    if X.is_sparse or X.layout == torch.sparse_csr:
        Xc = X.to_sparse_coo().coalesce()
        out = torch.zeros(X.shape[0], dtype=Xc.values().dtype, device=X.device)
        out.index_add_(0, Xc.indices()[0], Xc.values() ** 2)
        return out
    return (X * X).sum(1)


def linear_kernel(X, Y, k: float = 1.0, b: float = 0.0) -> torch.Tensor:
    """K[i, j] = k <x_i, y_j> + b (dense or CSR inputs)."""
    return k * _mm_t(X, Y) + b


def sq_distances(X, Y) -> torch.Tensor:
    """||x_i - y_j||^2 via ||x||^2 + ||y||^2 - 2 X Y^T (one GEMM, clamped at 0)."""
    G = _mm_t(X, Y)
    return (_sqnorm(X)[:, None] + _sqnorm(Y)[None, :] - 2 * G).clamp_min(0)


_lib.register({
    # G, ldg, n, m, nx, ny, inv2s2, dtype (0 fp32 / 1 fp64), stream
    "harp_rbf_from_gram": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_void_p,
                           _lib.c_double, _lib.c_int, _lib.c_void_p],
})


def rbf_kernel(X, Y, sigma: float = 1.0) -> torch.Tensor:
    """K[i, j] = exp(-||x_i - y_j||^2 / (2 sigma^2)). Dense fp32 / fp64 GPU inputs: one GEMM
    (hipBLASLt) and the in-place HIP epilogue ``csrc/kernelmat.hip`` (one pass instead of
    five elementwise torch passes over the n x m block)."""
    dense = not (X.is_sparse or Y.is_sparse or X.layout == torch.sparse_csr or Y.layout == torch.sparse_csr)
    if (dense and X.device.type == "cuda" and X.dtype == Y.dtype and X.dtype in (torch.float32, torch.float64)
            and _lib.use_native(X)):
        G = (X @ Y.t()).contiguous()
        nx, ny = _sqnorm(X).contiguous(), _sqnorm(Y).contiguous()
        st = _lib.kernels().harp_rbf_from_gram(G.data_ptr(), G.stride(0), G.shape[0], G.shape[1], nx.data_ptr(),
                                               ny.data_ptr(), 1.0 / (2 * sigma * sigma),
                                               1 if X.dtype == torch.float64 else 0, _lib.stream_ptr(X.device))
        _lib.check(st, "rbf_from_gram")
        return G
    return torch.exp(-sq_distances(X, Y) / (2 * sigma * sigma))


# ---------------------------------------------------------------- kNN
def knn_search(train: torch.Tensor, queries: torch.Tensor, k: int, tile: int = 8192) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact k nearest training rows of each query: (sq distances [M, k], indices [M, k]).

    Dense fp32 rows on a HIP device go through the fused GEMM + top-k selection kernel
    (``ops/knn.py``, ``csrc/knn.hip``); sparse / other-dtype / CPU inputs use the torch
    expression below."""
    from ..ops import knn as knn_ops

    dense = not (train.is_sparse or queries.is_sparse or train.layout == torch.sparse_csr
                 or queries.layout == torch.sparse_csr)
    if (dense and queries.device.type == "cuda" and train.dtype == torch.float32
            and queries.dtype == torch.float32 and min(k, train.shape[0]) <= knn_ops.MAX_NATIVE_K):
        return knn_ops.knn_search(train, queries, k)
    n = train.shape[0]
    k = min(k, n)
    tn = _sqnorm(train)
    ds, ix = [], []
    for a in range(0, queries.shape[0], tile):
        Q = queries[a:a + tile]
        D = (_sqnorm(Q)[:, None] + tn[None, :] - 2 * _mm_t(Q, train)).clamp_min(0)
        d, i = torch.topk(D, k, dim=1, largest=False)
        ds.append(d), ix.append(i)
    return torch.cat(ds), torch.cat(ix)


class KNNClassifier:
    """kNN classifier (daal kdtree_knn_classification semantics: majority vote of the
    k nearest training points, ties to the smallest label). ``comm`` distributes the
    training set: each worker's shard answers the queries locally, candidates are
    merged with one allgather."""

    def __init__(self, k: int = 5, comm: Optional[Communicator] = None):
        self.k, self.comm = k, comm

    def fit(self, X, y, num_classes: Optional[int] = None):
        self.X, self.y = X, y.long().reshape(-1)
        self.C = num_classes or int(self.y.max()) + 1
        if self.comm is not None and self.comm.world_size > 1:
            self.C = int(reduce_partials(self.comm, {"c": torch.tensor([float(self.C)])}, op=_max())["c"][0])
        return self

    def kneighbors(self, Q):
        d, i = knn_search(self.X, Q, self.k)
        lab = self.y.to(i.device)[i]
        if self.comm is None or self.comm.world_size == 1:
            return d, lab
        from .common import gather_rows

        k = self.k
        pad = k - d.shape[1]
        if pad > 0:
            d = torch.cat([d, torch.full((d.shape[0], pad), float("inf"), dtype=d.dtype, device=d.device)], 1)
            lab = torch.cat([lab, torch.full((lab.shape[0], pad), -1, dtype=lab.dtype, device=lab.device)], 1)
        both = torch.cat([d.double(), lab.double()], 1).to(self.comm.device)
        allc = gather_rows(self.comm, both).reshape(self.comm.world_size, Q.shape[0], 2 * k)
        D = allc[:, :, :k].permute(1, 0, 2).reshape(Q.shape[0], -1)
        L = allc[:, :, k:].permute(1, 0, 2).reshape(Q.shape[0], -1)
        dd, j = torch.topk(D, k, dim=1, largest=False)
        return dd, L.gather(1, j).long()

    def predict(self, Q):
        _, lab = self.kneighbors(Q)
        votes = torch.zeros((lab.shape[0], self.C + 1), dtype=torch.float64, device=lab.device)
        votes.scatter_add_(1, lab.clamp_min(-1) + 1, torch.ones_like(lab, dtype=torch.float64))
        return votes[:, 1:].argmax(1)


def _max():
    from ..core.combiner import Operation

    return Operation.MAX


# ---------------------------------------------------------------- EM-GMM
def em_gmm(X: torch.Tensor, K: int, comm: Optional[Communicator] = None, n_iterations: int = 100,
           accuracy_threshold: float = 1e-6, reg: float = 1e-6, covariance: str = "full",
           init: Optional[Dict[str, torch.Tensor]] = None, seed: int = 0, estep: str = "auto") -> Dict[str, torch.Tensor]:
    """EM for a K-component Gaussian mixture (full or diagonal covariance).
    Distributed: each worker holds a row shard; sufficient statistics are allreduced.
    Stops when the log-likelihood improves by less than ``accuracy_threshold``.
    ``estep``: "auto" (HIP kernels for fp64 GPU data, d <= 64) or "torch"."""
    from ..parallel.partition_util import broadcast_objects

    Xd = _dense(X).double()
    n, d = Xd.shape
    dev = Xd.device
    if init is None:
        g = torch.Generator().manual_seed(seed)
        cand = Xd[torch.randperm(n, generator=g)[:K].to(dev)]
        if comm is not None and comm.world_size > 1:
            cand = broadcast_objects(comm, [cand.cpu()] if comm.rank == 0 else None)[0].to(dev)
        mom = reduce_partials(comm or _one(), {"n": torch.tensor([float(n)]), "s": Xd.sum(0).cpu(),
                                               "ss": (Xd * Xd).sum(0).cpu()})
        var = (mom["ss"] / mom["n"] - (mom["s"] / mom["n"]) ** 2).to(dev)
        w = torch.full((K,), 1.0 / K, dtype=torch.float64, device=dev)
        mu = cand.clone()
        cov = torch.diag_embed(var.expand(K, d).clone()) if covariance == "full" else var.expand(K, d).clone()
    else:
        w, mu, cov = init["weights"].double().to(dev), init["means"].double().to(dev), init["covariances"].double().to(dev)
    prev = -math.inf
    ll = prev
    it = 0
    from ..ops import gmm as GM

    native = GM.usable(Xd) and estep != "torch"
    for it in range(n_iterations):
        if native:
            R, llsum = GM.estep(Xd, w, mu, cov, covariance)
            Nk, S1, S2 = GM.stats(Xd, R, covariance)
        else:
            logp = _log_gauss(Xd, mu, cov, covariance) + torch.log(w)[None, :]
            lse = torch.logsumexp(logp, 1)
            R = torch.exp(logp - lse[:, None])  # [n, K]
            llsum = lse.sum()
            Nk = R.sum(0)
            S1 = LA.atb(R, Xd)
            if covariance == "full":
                S2 = torch.einsum("nk,ni,nj->kij", R, Xd, Xd)
            else:
                S2 = LA.atb(R, Xd * Xd)
        st = reduce_partials(comm or _one(), {"Nk": Nk.cpu(), "S1": S1.cpu(), "S2": S2.cpu(),
                                              "ll": llsum.reshape(1).cpu(),
                                              "n": torch.tensor([float(n)])})
        Nk, S1, S2 = st["Nk"].to(dev), st["S1"].to(dev), st["S2"].to(dev)
        ll = float(st["ll"][0]) / float(st["n"][0])
        Nk_c = Nk.clamp_min(1e-12)
        mu = S1 / Nk_c[:, None]
        if covariance == "full":
            cov = S2 / Nk_c[:, None, None] - mu[:, :, None] * mu[:, None, :]
            cov = cov + reg * torch.eye(d, dtype=torch.float64, device=dev)
        else:
            cov = S2 / Nk_c[:, None] - mu * mu + reg
        w = Nk / Nk.sum()
        if abs(ll - prev) < accuracy_threshold:
            break
        prev = ll
    return {"weights": w, "means": mu, "covariances": cov, "loglik": torch.tensor(ll), "n_iterations": it + 1}


def _log_gauss(X, mu, cov, covariance):
    n, d = X.shape
    if covariance == "full":
        Lc = torch.linalg.cholesky(cov)  # [K, d, d]
        diff = (X[None, :, :] - mu[:, None, :]).transpose(1, 2)  # [K, d, n]
        z = torch.linalg.solve_triangular(Lc, diff, upper=False)  # [K, d, n]
        maha = (z * z).sum(1).t()  # [n, K]
        logdet = 2 * torch.log(torch.diagonal(Lc, dim1=1, dim2=2)).sum(1)
    else:
        maha = (((X[:, None, :] - mu[None]) ** 2) / cov[None]).sum(2)
        logdet = torch.log(cov).sum(1)
    return -0.5 * (maha + logdet[None, :] + d * math.log(2 * math.pi))


def gmm_predict(X, model) -> torch.Tensor:
    cov = model["covariances"]
    kind = "full" if cov.dim() == 3 else "diag"
    return (_log_gauss(_dense(X).double(), model["means"], cov, kind) + torch.log(model["weights"])[None]).argmax(1)


def _one():
    return Communicator()
