"""Sparse K-means (daal_kmeans/allreducecsr) + init methods: CSR equals dense Lloyd,
2-worker run equals single, k-means++ picks distinct data rows on every worker."""
import torch

from harp_amd.models import kmeans_csr as KC
from harp_amd.parallel.comm import Communicator
from harp_amd.runtime.launcher import launch


def _data(n=200, d=20, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, d, generator=g, dtype=torch.float64)
    X = X * (torch.rand(n, d, generator=g) < 0.3)
    return X


def _lloyd(X, C, iters):
    C = C.clone()
    for _ in range(iters):
        lab = torch.cdist(X, C).argmin(1)
        for k in range(C.shape[0]):
            m = lab == k
            if m.any():
                C[k] = X[m].mean(0)
    return C


def test_csr_matches_dense_lloyd():
    X = _data()
    C0 = KC.kmeans_init(X, 5, method="first")
    assert torch.equal(C0, X[:5])
    out = KC.kmeans_sparse(X.to_sparse_csr(), C0, 8)
    assert torch.allclose(out["centroids"], _lloyd(X, C0, 8), atol=1e-10)
    assert all(b <= a + 1e-9 for a, b in zip(out["objective"], out["objective"][1:]))


def _job(comm, X, method):
    n, P, r = X.shape[0], comm.world_size, comm.rank
    Xs = X[r * n // P:(r + 1) * n // P]
    C0 = KC.kmeans_init(Xs.to_sparse_csr(), 6, comm, method=method, seed=2)
    out = KC.kmeans_sparse(Xs.to_sparse_csr(), C0, 6, comm)
    return C0, out["centroids"]


def test_csr_distributed():
    X = _data()
    res = launch(_job, 2, args=(X, "first"), timeout=300)
    ref = _lloyd(X, X[:6], 6)
    for C0, C in res:
        assert torch.allclose(C, ref, atol=1e-10)
    for method in ("random", "plusplus"):
        res = launch(_job, 2, args=(X, method), timeout=300)
        assert torch.equal(res[0][0], res[1][0])
        C0 = res[0][0]
        assert len({tuple(r.tolist()) for r in C0}) == 6
        assert all(((X - c).abs().sum(1) < 1e-12).any() for c in C0)  # centroids are data rows
