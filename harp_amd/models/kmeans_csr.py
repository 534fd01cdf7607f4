"""K-means on sparse (CSR) data + K-means initialisation methods.

Reference: ml/daal/.../daal_kmeans/allreducecsr (DAAL ``kmeans.init`` then
``kmeans`` DistributedStep1Local on a CSRNumericTable; partial sums gathered to the
master (harpdaal_gather), master finalises and MST-broadcasts the centroids) and DAAL's
init methods (defaultDense = first K rows, randomDense, plusPlusDense).

MI355X design: the distance matrix of a CSR block is one sparse x dense product
(hipSPARSE SpMM) plus the norm epilogue; the partial sums are one sparse^T x one-hot
product; sums + counts + objective travel in ONE allreduce (every worker finalises, so
no broadcast step). k-means++ runs distributed: each round every worker draws a
candidate proportional to its local D^2 mass, the candidates and masses are
all-gathered, and every worker picks the same winner.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..ops import linalg as LA

from ..parallel.comm import Communicator
from .common import gather_rows, reduce_partials


def _is_sparse(X) -> bool:
    return X.is_sparse or X.layout == torch.sparse_csr


def _sqn(X):
    if _is_sparse(X):
        c = X.to_sparse_coo().coalesce()
        out = torch.zeros(X.shape[0], dtype=torch.float64, device=X.device)
        out.index_add_(0, c.indices()[0], c.values().double() ** 2)
        return out
    return (X.double() ** 2).sum(1)


def _xct(X, C):
    if _is_sparse(X):
        return torch.sparse.mm(X.double() if X.dtype != torch.float64 else X, C.t().contiguous())
    return X.double() @ C.t()


def _rows(X, idx):
    if _is_sparse(X):
        return torch.stack([X[int(i)].to_dense() for i in idx]).double() if len(idx) else \
            torch.zeros((0, X.shape[1]), dtype=torch.float64)
    return X[idx].double()


def sq_dist(X, C):
    return (_sqn(X)[:, None] + (C * C).sum(1)[None, :] - 2 * _xct(X, C)).clamp_min(0)


def kmeans_init(X, K: int, comm: Optional[Communicator] = None, method: str = "first", seed: int = 0) -> torch.Tensor:
    """Initial centroids [K, d] fp64, identical on every worker."""
    comm = comm or Communicator()
    n = X.shape[0]
    if method == "first":  # defaultDense: first K rows of the (rank-ordered) global data
        return gather_rows(comm, _rows(X, list(range(min(K, n)))).to(comm.device))[:K].cpu()
    g = torch.Generator().manual_seed(seed + 7 * comm.rank)
    if method == "random":
        pick = torch.randperm(n, generator=g)[:K].tolist()
        cand = gather_rows(comm, _rows(X, pick).to(comm.device)).cpu()
        gs = torch.Generator().manual_seed(seed)
        return cand[torch.randperm(cand.shape[0], generator=gs)[:K]]
    if method != "plusplus":
        raise ValueError(method)
    gs = torch.Generator().manual_seed(seed)  # shared stream: same choices everywhere
    first = int(torch.randint(0, n, (1,), generator=g))
    c0 = gather_rows(comm, _rows(X, [first]).to(comm.device)).cpu()
    C = c0[int(torch.randint(0, c0.shape[0], (1,), generator=gs))][None]
    best = sq_dist(X, C.to(X.device))[:, 0].cpu()
    while C.shape[0] < K:
        mass = best.sum()
        i = int(torch.multinomial(best / mass, 1, generator=g)) if float(mass) > 0 else \
            int(torch.randint(0, n, (1,), generator=g))
        row = _rows(X, [i])
        info = torch.cat([row, mass.reshape(1, 1)], 1)
        allc = gather_rows(comm, info.to(comm.device)).cpu()
        w = allc[:, -1]
        j = int(torch.multinomial(w / w.sum(), 1, generator=gs)) if float(w.sum()) > 0 else 0
        newc = allc[j, :-1][None]
        C = torch.cat([C, newc])
        best = torch.minimum(best, sq_dist(X, newc.to(X.device))[:, 0].cpu())
    return C


def kmeans_sparse(X, C0: torch.Tensor, iterations: int = 10, comm: Optional[Communicator] = None) -> Dict:
    comm = comm or Communicator()
    C = C0.to(device=X.device, dtype=torch.float64, copy=True)
    K, d = C.shape
    obj = []
    if _is_sparse(X) and X.device.type == "cuda":
        # fused HIP E-step + accumulate (csrc/kmeans_csr.hip): no [n, K] tensors
        from ..ops import kmeans_csr as KC

        A = KC.to_device_csr(X)
        for _ in range(iterations):
            lab, m, S, cnt = KC.assign_accumulate(A, C)
            r = reduce_partials(comm, {"S": S, "n": cnt, "o": m.sum().reshape(1)})
            cnt = r["n"].to(C.device)
            nz = cnt > 0
            C[nz] = r["S"].to(C.device)[nz] / cnt[nz, None]
            obj.append(float(r["o"][0]))
        return {"centroids": C, "objective": obj, "labels": lab}
    for _ in range(iterations):
        D = sq_dist(X, C)
        m, lab = D.min(1)
        onehot = torch.zeros((X.shape[0], K), dtype=torch.float64, device=X.device)
        onehot[torch.arange(X.shape[0], device=X.device), lab] = 1.0
        if _is_sparse(X):
            S = torch.sparse.mm(X.double().t() if X.layout != torch.sparse_csr else
                                X.to_sparse_coo().double().t(), onehot).t()
        else:
            S = LA.atb(onehot, X.double())
        r = reduce_partials(comm, {"S": S, "n": onehot.sum(0), "o": m.sum().reshape(1)})
        cnt = r["n"].to(C.device)
        nz = cnt > 0
        C[nz] = r["S"].to(C.device)[nz] / cnt[nz, None]
        obj.append(float(r["o"][0]))
    return {"centroids": C, "objective": obj, "labels": lab}
