"""Optimization solvers (DAAL optimization_solver), rotation MLR (contrib), kernel
functions, kNN and EM-GMM: single process against closed forms / sklearn, and the
distributed variants on 2 gloo workers against the single-process answer."""
import math

import pytest
import torch

from harp_amd.models import kernels as KF
from harp_amd.models import mlr as M
from harp_amd.models import optim as O
from harp_amd.parallel.comm import Communicator
from harp_amd.runtime.launcher import launch


def _lin_data(n=400, d=5, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g, dtype=torch.float64)
    beta = torch.randn(d, generator=g, dtype=torch.float64)
    y = X @ beta + 0.7 + 0.01 * torch.randn(n, generator=g, dtype=torch.float64)
    return X, y, beta


def _ols(X, y):
    A = torch.cat([torch.ones(X.shape[0], 1, dtype=X.dtype), X], 1)
    return torch.linalg.lstsq(A, y[:, None]).solution[:, 0]


def test_mse_gradient_matches_autograd():
    X, y, _ = _lin_data(50)
    obj = O.MSE(X, y, l2=0.1)
    x = torch.randn(6, dtype=torch.float64, requires_grad=True)
    r = X @ x[1:] + x[0] - y
    f = 0.5 * (r * r).sum() / 50 + 0.1 * (x[1:] ** 2).sum()
    f.backward()
    v, g = obj.value_grad(x.detach())
    assert torch.allclose(v, f.detach()) and torch.allclose(g, x.grad)


def test_logistic_and_xent_gradients():
    X, y, _ = _lin_data(60)
    yb = (y > y.median()).double()
    x = torch.randn(6, dtype=torch.float64, requires_grad=True)
    f = torch.nn.functional.binary_cross_entropy_with_logits(X @ x[1:] + x[0], yb)
    f.backward()
    v, g = O.LogisticLoss(X, yb).value_grad(x.detach())
    assert torch.allclose(v, f.detach()) and torch.allclose(g, x.grad)
    yc = torch.bucketize(y, y.quantile(torch.tensor([0.33, 0.66], dtype=torch.float64)))
    B = torch.randn(3, 6, dtype=torch.float64, requires_grad=True)
    f = torch.nn.functional.cross_entropy(X @ B[:, 1:].t() + B[:, 0], yc) + 0.05 * (B[:, 1:] ** 2).sum()
    f.backward()
    v, g = O.CrossEntropyLoss(X, yc, 3, l2=0.05).value_grad(B.detach().reshape(-1))
    assert torch.allclose(v, f.detach()) and torch.allclose(g, B.grad.reshape(-1))


@pytest.mark.parametrize("solver,kw", [
    ("sgd", dict(batch_size=400, learning_rate=0.3, n_iterations=400)),
    ("sgd", dict(batch_size=32, learning_rate=0.05, n_iterations=3000, momentum=0.9)),
    ("sgd", dict(batch_size=1, learning_rate=lambda k: 0.1 / (1 + k / 500), n_iterations=6000)),
    ("sgd", dict(batch_size=64, learning_rate=0.1, n_iterations=2000, conservative_sequence=0.01,
                 inner_iterations=2)),
    ("adagrad", dict(batch_size=50, learning_rate=0.5, n_iterations=3000)),
    ("lbfgs", dict(n_iterations=50)),
    ("lbfgs", dict(n_iterations=300, batch_size=200, step_length=0.5)),
])
def test_solvers_reach_least_squares(solver, kw):
    X, y, _ = _lin_data()
    ref = _ols(X, y)
    res = O.SOLVERS[solver](O.MSE(X, y), **kw)
    assert (res.minimum - ref).abs().max().item() < 0.05, (res.minimum, ref)


def test_sgd_accuracy_threshold_stops_early():
    X, y, _ = _lin_data()
    res = O.sgd(O.MSE(X, y), batch_size=400, learning_rate=0.3, n_iterations=10000, accuracy_threshold=1e-10)
    assert res.n_iterations < 10000


def _dist_solver_job(comm, X, y):
    n, P, r = X.shape[0], comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    a = O.lbfgs(O.MSE(X[sl], y[sl], comm=comm), n_iterations=50).minimum
    b = O.sgd(O.MSE(X[sl], y[sl], comm=comm), batch_size=10 ** 9, learning_rate=0.3, n_iterations=300).minimum
    return a, b


def test_distributed_solvers_match_global():
    X, y, _ = _lin_data()
    ref = _ols(X, y)
    res = launch(_dist_solver_job, 2, args=(X, y), timeout=300)
    for a, b in res:
        assert (a - ref).abs().max() < 1e-5
        assert (b - ref).abs().max() < 1e-3
    assert torch.equal(res[0][0], res[1][0])


# ---------------------------------------------------------------- MLR
def _seq_mlr(X, Y, alpha, iters, P):
    """The reference's sequential per-instance update order for 1 worker holding all
    rows: per iteration, P passes over the data (ITER * P rotations)."""
    T, D = Y.shape[1], X.shape[1]
    W = torch.zeros(T, D + 1, dtype=torch.float64)
    Xd = X.double()
    for _ in range(iters * P):
        for i in range(X.shape[0]):
            p = torch.sigmoid(W[:, 1:] @ Xd[i] + W[:, 0])
            r = alpha * (Y[i].double() - p)
            W[:, 0] += r
            W[:, 1:] += r[:, None] * Xd[i][None, :]
    return W


def test_mlr_single_worker_matches_sequential_update():
    X, Y = M.synthetic_multilabel(60, 30, 4, density=0.2)
    comm = Communicator()
    out = M.train(comm, M.CSRRows.from_dense(X), Y, M.MLRConfig(alpha=0.5, iterations=2, batch_size=1), 4, 30)
    ref = _seq_mlr(X, Y, 0.5, 2, 1)
    assert torch.allclose(out["W"], ref, atol=1e-9)


def _mlr_job(comm, X, Y):
    n, P, r = X.shape[0], comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    Xs = M.CSRRows.from_dense(X[sl])
    out = M.train(comm, Xs, Y[sl], M.MLRConfig(alpha=0.5, iterations=3, batch_size=8), 5, X.shape[1])
    ev = M.evaluate(comm, Xs, Y[sl], out["W"])
    return out["W"], ev["micro_f1"], ev["tp"]


def test_mlr_rotation_distributed():
    X, Y = M.synthetic_multilabel(600, 80, 5, density=0.1)
    res = launch(_mlr_job, 2, args=(X, Y), timeout=300)
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] and res[0][1] > 0.5
    # vs a single worker running the same number of passes: close, not bitwise (order)
    comm = Communicator()
    single = M.train(comm, M.CSRRows.from_dense(X), Y, M.MLRConfig(alpha=0.5, iterations=3, batch_size=8), 5, 80)
    f1_single = M.evaluate(comm, M.CSRRows.from_dense(X), Y, single["W"])["micro_f1"]
    assert abs(f1_single - res[0][1]) < 0.15


# ---------------------------------------------------------------- kernels / kNN / GMM
def test_kernel_functions_dense_and_csr():
    g = torch.Generator().manual_seed(0)
    X = torch.randn(30, 7, generator=g, dtype=torch.float64)
    Y = torch.randn(20, 7, generator=g, dtype=torch.float64)
    Xs = (X * (X > 0.3)).to_sparse_csr()
    lin = KF.linear_kernel(X, Y, k=2.0, b=1.0)
    assert torch.allclose(lin, 2 * X @ Y.t() + 1)
    assert torch.allclose(KF.linear_kernel(Xs, Y), Xs.to_dense() @ Y.t())
    ref = torch.exp(-torch.cdist(X, Y) ** 2 / (2 * 1.5 ** 2))
    assert torch.allclose(KF.rbf_kernel(X, Y, 1.5), ref, atol=1e-12)
    ref2 = torch.exp(-torch.cdist(Xs.to_dense(), Y) ** 2 / 2)
    assert torch.allclose(KF.rbf_kernel(Xs, Y), ref2, atol=1e-12)


def test_knn_matches_sklearn():
    from sklearn.datasets import make_classification
    from sklearn.neighbors import KNeighborsClassifier

    X, y = make_classification(800, 10, n_informative=5, n_classes=3, random_state=2)
    X, y = torch.tensor(X), torch.tensor(y)
    ours = KF.KNNClassifier(5).fit(X[:600], y[:600]).predict(X[600:])
    ref = KNeighborsClassifier(5).fit(X[:600].numpy(), y[:600].numpy()).predict(X[600:].numpy())
    assert (ours.numpy() == ref).mean() > 0.97


def _knn_job(comm, X, y, Q):
    n, P, r = X.shape[0], comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    c = KF.KNNClassifier(7, comm).fit(X[sl], y[sl], num_classes=3)
    return c.kneighbors(Q)[0], c.predict(Q)


def test_knn_distributed_equals_single():
    from sklearn.datasets import make_classification

    X, y = make_classification(500, 6, n_informative=4, n_classes=3, random_state=3)
    X, y = torch.tensor(X), torch.tensor(y)
    Q = X[:50] + 0.01
    single = KF.KNNClassifier(7).fit(X, y)
    d1 = single.kneighbors(Q)[0]
    res = launch(_knn_job, 2, args=(X, y, Q), timeout=300)
    assert torch.allclose(res[0][0], d1.double(), atol=1e-9)
    assert torch.equal(res[0][1], single.predict(Q))


def _gmm_data():
    g = torch.Generator().manual_seed(5)
    A = torch.randn(300, 2, generator=g, dtype=torch.float64) * 0.3 + torch.tensor([2.0, 0.0], dtype=torch.float64)
    B = torch.randn(300, 2, generator=g, dtype=torch.float64) @ torch.tensor([[0.5, 0.2], [0.0, 0.3]],
                                                                            dtype=torch.float64) - 1
    return torch.cat([A, B])[torch.randperm(600, generator=g)]


def test_em_gmm_matches_sklearn():
    from sklearn.mixture import GaussianMixture

    X = _gmm_data()
    m = KF.em_gmm(X, 2, n_iterations=300, accuracy_threshold=1e-10, reg=1e-6)
    sk = GaussianMixture(2, covariance_type="full", reg_covar=1e-6, tol=1e-10, max_iter=300, random_state=0).fit(
        X.numpy())
    assert abs(float(m["loglik"]) - sk.score(X.numpy())) < 1e-3
    ours = sorted(m["means"].tolist())
    ref = sorted(sk.means_.tolist())
    assert torch.allclose(torch.tensor(ours), torch.tensor(ref), atol=1e-3)
    md = KF.em_gmm(X, 2, covariance="diag", n_iterations=200)
    assert md["covariances"].shape == (2, 2)
    assert (KF.gmm_predict(X, m) == KF.gmm_predict(X, m)).all()


def _gmm_job(comm, X, init):
    n, P, r = X.shape[0], comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    return KF.em_gmm(X[sl], 2, comm, n_iterations=30, accuracy_threshold=0, init=init)


def test_em_gmm_distributed_equals_single():
    X = _gmm_data()
    init = {"weights": torch.tensor([0.5, 0.5], dtype=torch.float64), "means": X[:2].clone(),
            "covariances": torch.eye(2, dtype=torch.float64).expand(2, 2, 2).clone()}
    single = KF.em_gmm(X, 2, n_iterations=30, accuracy_threshold=0, init=init)
    res = launch(_gmm_job, 2, args=(X, init), timeout=300)
    for r in res:
        assert torch.allclose(r["means"], single["means"], atol=1e-9)
        assert torch.allclose(r["covariances"], single["covariances"], atol=1e-9)
