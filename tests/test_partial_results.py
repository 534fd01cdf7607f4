"""DAAL-family distributed partial results on 2 gloo workers vs single-process numpy /
scipy / sklearn on the full data (covariance, moments, PCA x2, TSQR/SVD, normalization,
outliers, linear/ridge regression (normal eq + QR), quality metrics, Naive Bayes)."""
import numpy as np
import pytest
import torch

from harp_amd.models import naive_bayes as NB
from harp_amd.models import regression as RG
from harp_amd.models import stats as ST
from harp_amd.runtime.launcher import launch


def _data(seed=0, n=400, d=6):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(d, d, generator=g, dtype=torch.float64)
    X = torch.randn(n, d, generator=g, dtype=torch.float64) @ A + torch.arange(d, dtype=torch.float64)
    beta = torch.randn(d, generator=g, dtype=torch.float64)
    y = X @ beta + 0.5 + 0.01 * torch.randn(n, generator=g, dtype=torch.float64)
    cls = (X[:, 0] > X[:, 0].median()).long() + (X[:, 1] > X[:, 1].median()).long()
    counts = torch.poisson(torch.rand(n, 12, generator=g) * 3 + cls[:, None].double() * torch.linspace(0, 2, 12))
    return X, y, cls, counts


def _job(comm, X, y, cls, counts):
    P, r = comm.world_size, comm.rank
    n = X.shape[0]
    sl = slice(r * n // P, (r + 1) * n // P)
    Xs, ys, cs, ks = X[sl], y[sl], cls[sl], counts[sl]
    out = {}
    out["cov"] = ST.covariance(Xs, comm)
    out["cov_csr"] = ST.covariance(Xs.to_sparse_csr(), comm)
    out["mom"] = ST.low_order_moments(Xs, comm)
    out["pca_cor"] = ST.pca(Xs, comm, "correlation")
    out["pca_svd"] = ST.pca(Xs, comm, "svd")
    q = ST.tsqr(Xs, comm)
    out["qr_R"], out["qr_Q"] = q["R"], q["Q"]
    out["svd"] = ST.svd(Xs, comm)
    out["minmax"] = ST.normalize_minmax(Xs, comm=comm)
    out["zscore"] = ST.normalize_zscore(Xs, comm=comm)
    out["uni"] = ST.outliers_univariate(Xs, comm=comm)
    out["multi"] = ST.outliers_multivariate(Xs, comm=comm)
    out["lin_ne"] = RG.train_linear(Xs, ys, comm)["beta"]
    out["lin_qr"] = RG.train_linear(Xs, ys, comm, method="qr")["beta"]
    out["ridge"] = RG.train_linear(Xs, ys, comm, ridge=3.0)["beta"]
    out["lrq"] = RG.linreg_quality(Xs, ys, out["lin_ne"], comm)
    out["nb"] = NB.train(ks, cs, 3, comm)
    out["nb_csr"] = NB.train(ks.to_sparse_csr(), cs, 3, comm)
    return out


@pytest.fixture(scope="module")
def results():
    X, y, cls, counts = _data()
    res = launch(_job, 2, args=(X, y, cls, counts), timeout=300)
    return (X, y, cls, counts), res


def test_covariance_moments(results):
    (X, y, cls, counts), res = results
    Xn = X.numpy()
    for k in ("cov", "cov_csr"):
        assert np.allclose(res[0][k]["covariance"].numpy(), np.cov(Xn.T), atol=1e-8)
        assert np.allclose(res[1][k]["mean"].numpy(), Xn.mean(0))
    m = res[0]["mom"]
    assert np.allclose(m["minimum"].numpy(), Xn.min(0)) and np.allclose(m["maximum"].numpy(), Xn.max(0))
    assert np.allclose(m["variance"].numpy(), Xn.var(0, ddof=1)) and np.allclose(m["sumSquares"].numpy(), (Xn ** 2).sum(0))
    assert np.allclose(m["standardDeviation"].numpy(), Xn.std(0, ddof=1))


def test_pca_both_methods(results):
    (X, *_), res = results
    C = np.corrcoef(X.numpy().T)
    w = np.sort(np.linalg.eigvalsh(C))[::-1]
    for k in ("pca_cor", "pca_svd"):
        assert np.allclose(res[0][k]["eigenvalues"].numpy(), w, atol=1e-8)
    a, b = res[0]["pca_cor"]["eigenvectors"].numpy(), res[0]["pca_svd"]["eigenvectors"].numpy()
    assert np.allclose(np.abs(a), np.abs(b), atol=1e-6)


def test_tsqr_svd(results):
    (X, *_), res = results
    Xn = X.numpy()
    R = res[0]["qr_R"].numpy()
    assert np.allclose(R.T @ R, Xn.T @ Xn, atol=1e-7) and np.allclose(np.tril(R, -1), 0)
    Q = np.concatenate([res[0]["qr_Q"].numpy(), res[1]["qr_Q"].numpy()])
    assert np.allclose(Q @ R, Xn, atol=1e-8) and np.allclose(Q.T @ Q, np.eye(Xn.shape[1]), atol=1e-8)
    s = np.linalg.svd(Xn, compute_uv=False)
    assert np.allclose(res[0]["svd"]["singularValues"].numpy(), s)
    U = np.concatenate([res[0]["svd"]["leftSingularMatrix"].numpy(), res[1]["svd"]["leftSingularMatrix"].numpy()])
    assert np.allclose(U * s @ res[0]["svd"]["rightSingularMatrix"].numpy(), Xn, atol=1e-8)


def test_normalization_outliers(results):
    (X, *_), res = results
    Xn = X.numpy()
    mm = np.concatenate([res[0]["minmax"].numpy(), res[1]["minmax"].numpy()])
    assert np.allclose(mm, (Xn - Xn.min(0)) / (Xn.max(0) - Xn.min(0)))
    z = np.concatenate([res[0]["zscore"].numpy(), res[1]["zscore"].numpy()])
    assert np.allclose(z, (Xn - Xn.mean(0)) / Xn.std(0, ddof=1))
    uni = np.concatenate([res[0]["uni"].numpy(), res[1]["uni"].numpy()])
    assert uni.shape == Xn.shape and uni.mean() > 0.98
    multi = np.concatenate([res[0]["multi"].numpy(), res[1]["multi"].numpy()])
    assert multi.mean() > 0.98


def test_regressions(results):
    (X, y, *_), res = results
    from sklearn.linear_model import LinearRegression, Ridge

    lr = LinearRegression().fit(X.numpy(), y.numpy())
    ref = np.concatenate([[lr.intercept_], lr.coef_])
    for k in ("lin_ne", "lin_qr"):
        assert np.allclose(res[0][k].numpy()[0], ref, atol=1e-7), k
    rd = Ridge(alpha=3.0).fit(X.numpy(), y.numpy())
    assert np.allclose(res[1]["ridge"].numpy()[0], np.concatenate([[rd.intercept_], rd.coef_]), atol=1e-6)
    q = res[0]["lrq"]
    assert float(q["determinationCoeff"][0]) > 0.999 and float(q["rms"][0]) < 0.02


def test_naive_bayes(results):
    (X, y, cls, counts), res = results
    from sklearn.naive_bayes import MultinomialNB

    nb = MultinomialNB(alpha=1.0).fit(counts.numpy(), cls.numpy())
    for k in ("nb", "nb_csr"):
        m = res[0][k]
        assert np.allclose(m["logTheta"].numpy(), nb.feature_log_prob_, atol=1e-10)
        assert np.allclose(m["logPrior"].numpy(), nb.class_log_prior_)
        assert (NB.predict(counts, m).numpy() == nb.predict(counts.numpy())).all()


def test_quality_metrics_and_batch_ops():
    yt = torch.tensor([0, 1, 2, 2, 1, 0, 2])
    yp = torch.tensor([0, 2, 2, 2, 1, 0, 1])
    q = RG.classification_quality(yt, yp, 3)
    assert q["confusionMatrix"].sum() == 7 and abs(float(q["errorRate"]) - 2 / 7) < 1e-12
    X = torch.randn(50, 4, dtype=torch.float64)
    L = ST.cholesky(X.t() @ X)
    assert torch.allclose(L @ L.t(), X.t() @ X)
    pq = ST.pivoted_qr(X)
    assert torch.allclose(pq["Q"] @ pq["R"], X[:, pq["permutation"]])
    assert torch.equal(ST.sort_features(X), torch.sort(X, 0).values)
    qs = ST.quantiles(X, (0.25, 0.75))
    assert torch.allclose(qs, torch.quantile(X, torch.tensor([0.25, 0.75], dtype=torch.float64), dim=0))
    Xo = torch.cat([torch.randn(200, 3, dtype=torch.float64), torch.full((5, 3), 25.0, dtype=torch.float64)])
    w = ST.outliers_bacon(Xo)
    assert w[-5:].sum() == 0 and w[:200].mean() > 0.9


def _cholqr_job(comm, X):
    from harp_amd.models import stats as ST

    P, r = comm.world_size, comm.rank
    n = X.shape[0]
    Xs = X[r * n // P:(r + 1) * n // P]
    out = ST.tsqr(Xs, comm, method="cholqr2")
    return out["Q"], out["R"]


@pytest.mark.parametrize("P", [1, 3])
def test_cholesky_qr2_distributed_matches_householder(P):
    from harp_amd.runtime.launcher import launch

    g = torch.Generator().manual_seed(11)
    X = torch.randn(900, 12, generator=g, dtype=torch.float64) @ torch.diag(torch.logspace(0, 3, 12, dtype=torch.float64))
    res = launch(_cholqr_job, P, args=(X,), timeout=120)
    Q = torch.cat([q for q, _ in res])
    R = res[0][1]
    _, Rt = torch.linalg.qr(X)
    Rt = Rt * torch.sign(torch.diagonal(Rt))[:, None]
    assert torch.allclose(R, Rt, rtol=1e-10, atol=1e-9)
    assert torch.allclose(Q.t() @ Q, torch.eye(12, dtype=torch.float64), atol=1e-13)
    assert torch.allclose(Q @ R, X, atol=1e-10)


def test_cholesky_qr2_refuses_ill_conditioned_and_auto_falls_back():
    from harp_amd.models import stats as ST

    g = torch.Generator().manual_seed(12)
    X = torch.randn(500, 6, generator=g, dtype=torch.float64) @ torch.diag(torch.tensor([1, 1, 1, 1, 1, 1e-9],
                                                                                        dtype=torch.float64))
    assert ST.cholesky_qr2(X) is None
    out = ST.tsqr(X, method="auto")  # CPU auto = Householder anyway; result must stay exact
    assert torch.allclose(out["Q"] @ out["R"], X, atol=1e-12)


def test_cholesky_qr2_refuses_kahan_with_small_diagonal_spread():
    """A Kahan matrix (cond ~1e14, R diagonal spread ~100) passes the diagonal test; the
    second-pass factor R2 being far from I must send tsqr to Householder."""
    import math

    from harp_amd.models import stats as ST

    n, c = 100, 0.3
    s = math.sqrt(1 - c * c)
    K = torch.diag(torch.tensor([s ** i for i in range(n)], dtype=torch.float64)) @ (
        torch.eye(n, dtype=torch.float64) - c * torch.triu(torch.ones(n, n, dtype=torch.float64), 1))
    g = torch.Generator().manual_seed(0)
    Q0, _ = torch.linalg.qr(torch.randn(3000, n, generator=g, dtype=torch.float64))
    X = Q0 @ K
    dg = torch.diagonal(K)
    assert float(dg.max() / dg.min()) < ST.CHOLQR_MAX_DIAG_RATIO  # the old test alone accepts it
    assert ST.cholesky_qr2(X) is None
    with pytest.raises(ValueError):
        ST.tsqr(X, method="cholqr2")
    out = ST.tsqr(X, method="householder")
    eye = torch.eye(n, dtype=torch.float64)
    assert (out["Q"].t() @ out["Q"] - eye).abs().max() < 1e-12


def _np_cov(X):
    import numpy as np

    return np.cov(X.astype(np.float64), rowvar=False)


def test_precision_policy_covariance_cpu():
    """dtype='fp32' / 'fp64' / 'bf16' on an fp32 block (CPU): fp32 within 1e-6 (normwise,
    relative) of the fp64 covariance, fp64 within 1e-12, bf16 within its documented 3e-3;
    an fp32 input defaults to the fp32 mode, never to bf16."""
    import numpy as np

    from harp_amd.models import stats as ST

    g = torch.Generator().manual_seed(4)
    X = torch.rand(200_000, 40, generator=g, dtype=torch.float32) + 10.0  # a large mean: cancellation
    ref = _np_cov(X.numpy())
    nrm = np.abs(ref).max()
    errs = {}
    for mode in ("fp32", "fp64", "bf16", None):
        cov = ST.covariance(X, dtype=mode)["covariance"].numpy()
        errs[mode] = np.abs(cov - ref).max() / nrm
    assert errs["fp64"] <= 1e-12 and errs["fp32"] <= 1e-6, errs
    assert ST._policy(X.cuda() if torch.cuda.is_available() else X, None) in ("fp32", "fp64")
    # bf16 of data offset by +10 keeps 3 significant digits of the U[0,1) part: not bounded;
    # on U[0,1) data the module's documented bound holds
    Xu = X - 10.0  # U[0,1): the bf16 bound the module notes state
    e16 = np.abs(ST.covariance(Xu, dtype="bf16")["covariance"].numpy() - _np_cov(Xu.numpy())).max() / nrm
    assert e16 <= 3e-3, e16


def test_precision_policy_moments_cpu():
    import numpy as np

    from harp_amd.models import stats as ST

    g = torch.Generator().manual_seed(5)
    X = torch.rand(100_000, 16, generator=g, dtype=torch.float32) * 3 + 100.0
    Xn = X.numpy().astype(np.float64)
    for mode, tol in (("fp32", 1e-6), ("fp64", 1e-12)):
        m = ST.low_order_moments(X, dtype=mode)
        assert np.abs(m["variance"].numpy() - Xn.var(0, ddof=1)).max() <= tol * Xn.var(0).max(), mode
        assert np.abs(m["mean"].numpy() - Xn.mean(0)).max() <= tol * 100


def _prec_worker(comm):
    from harp_amd.models import stats as ST

    g = torch.Generator().manual_seed(100 + comm.rank)
    X = torch.rand(30_000 + 1000 * comm.rank, 12, generator=g, dtype=torch.float32) + 5.0
    return {"cov": ST.covariance(X, comm, dtype="fp32")["covariance"],
            "var": ST.low_order_moments(X, comm, dtype="fp32")["variance"], "X": X}


def test_precision_policy_distributed_gloo():
    import numpy as np

    from harp_amd.runtime.launcher import launch

    outs = launch(_prec_worker, 2, timeout=300)
    Xall = torch.cat([o["X"] for o in outs]).numpy().astype(np.float64)
    ref = np.cov(Xall, rowvar=False)
    for o in outs:
        assert np.abs(o["cov"].numpy() - ref).max() <= 1e-6 * np.abs(ref).max()
        assert np.abs(o["var"].numpy() - Xall.var(0, ddof=1)).max() <= 1e-6 * Xall.var(0).max()
