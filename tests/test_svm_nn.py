"""SVM (SMO vs sklearn's libsvm, OvO multiclass, cascade SVM over the HarpString
allreduce path on 2 gloo workers) and MLP training (gradient vs autograd, model
averaging and synchronous SGD on 2 gloo workers)."""
import pytest
import torch

from harp_amd.core.table import Table
from harp_amd.models import nn as NN
from harp_amd.models import svm as S
from harp_amd.parallel import collectives as CL
from harp_amd.runtime.launcher import launch

sk_ds = pytest.importorskip("sklearn.datasets")


def _blobs(n=300, seed=0, classes=2, d=4):
    X, y = sk_ds.make_blobs(n, d, centers=classes, cluster_std=2.5, random_state=seed)
    return torch.tensor(X), torch.tensor(y)


@pytest.mark.parametrize("kernel", ["linear", "rbf"])
def test_binary_svm_matches_libsvm(kernel):
    from sklearn.svm import SVC

    X, y = _blobs()
    m = S.BinarySVM(C=1.0, kernel=kernel, sigma=2.0, accuracy_threshold=1e-6).fit(X, y)
    ref = SVC(C=1.0, kernel=kernel, gamma=1 / (2 * 2.0 ** 2), tol=1e-6).fit(X.numpy(), y.numpy())
    ours = m.decision(X)
    theirs = torch.tensor(ref.decision_function(X.numpy()))
    # sklearn's decision is for class 1 vs 0; ours maps {0,1} -> {-1,+1}
    assert torch.allclose(ours, theirs, atol=2e-3), (ours - theirs).abs().max()
    assert abs(m.coef.abs().sum().item() - float(abs(ref.dual_coef_).sum())) < 1e-3


def test_multiclass_svm():
    from sklearn.svm import SVC

    X, y = _blobs(400, 1, classes=4)
    m = S.MultiClassSVM(4, C=0.5, kernel="rbf", sigma=3.0).fit(X[:300], y[:300])
    ours = m.predict(X[300:])
    ref = SVC(C=0.5, kernel="rbf", gamma=1 / 18.0).fit(X[:300].numpy(), y[:300].numpy()).predict(X[300:].numpy())
    assert (ours.numpy() == ref).mean() > 0.97
    Xs = X.to_sparse_csr()
    mc = S.MultiClassSVM(4, C=0.5).fit(Xs, y)
    assert (mc.predict(X) == y).double().mean() > 0.8


def test_harp_string_plus_combiner():
    t = Table(0, S.HarpStringPlus())
    t.add(0, S.HarpString("a b"))
    t.add(0, S.HarpString("c"))
    assert t[0].s == "a b\nc"


def _cascade_job(comm, X, y):
    n, P, r = X.shape[0], comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    out = S.cascade_svm(comm, X[sl], y[sl], iterations=3, C=1.0)
    return sorted(out["support_vectors"]), out["sizes"], out["model"].decision(X)


def test_cascade_svm_two_workers():
    X, y = _blobs(200, 3)
    res = launch(_cascade_job, 2, args=(X, y), timeout=300)
    assert res[0][0] == res[1][0]
    full = S.BinarySVM(C=1.0).fit(X, y)
    # the cascade's final model agrees with the single-machine SVM on the training set
    agree = ((res[0][2] > 0) == (full.decision(X) > 0)).double().mean().item()
    assert agree > 0.97


def test_mlp_gradient_matches_autograd():
    g = torch.Generator().manual_seed(0)
    X = torch.randn(16, 5, generator=g, dtype=torch.float64)
    y = torch.randint(0, 3, (16,), generator=g)
    Y = torch.nn.functional.one_hot(y, 3)
    for act, out in (("sigmoid", "softmax"), ("relu", "softmax"), ("tanh", "sigmoid")):
        net = NN.MLP([5, 7, 6, 3], act, out, dtype=torch.float64)
        grad = net.gradient(X, Y)
        ps = [p.clone().requires_grad_(True) for p in net.params]
        h = X
        for l in range(3):
            z = h @ ps[2 * l].t() + ps[2 * l + 1]
            if l < 2:
                h = {"sigmoid": torch.sigmoid, "relu": torch.relu, "tanh": torch.tanh}[act](z)
            else:
                h = z
        if out == "softmax":
            loss = torch.nn.functional.cross_entropy(h, y)
        else:
            p = torch.sigmoid(h)
            loss = 0.5 * ((p - Y) ** 2).sum(1).mean()
        loss.backward()
        ref = torch.cat([p.grad.reshape(-1) for p in ps])
        assert torch.allclose(grad, ref, atol=1e-10), act


def _nn_job(comm, X, Y, mode):
    n, P, r = X.shape[0], comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    net = NN.MLP([X.shape[1], 16, Y.shape[1]], "sigmoid", seed=comm.rank)
    if mode == "avg":
        NN.train_model_averaging(comm, net, X[sl], Y[sl], epochs=30, batch=32, lr=0.5, sync_iters=5)
    else:
        NN.train_sync_sgd(comm, net, X[sl], Y[sl], epochs=30, batch=32, lr=0.5, momentum=0.5)
    return net.flat.clone(), (net.predict(X) == Y.argmax(1)).double().mean().item()


@pytest.mark.parametrize("mode", ["avg", "sync"])
def test_mlp_distributed(mode):
    X, y = _blobs(600, 4, classes=3)
    X = (X - X.mean(0)) / X.std(0)
    Y = torch.nn.functional.one_hot(y, 3).float()
    res = launch(_nn_job, 2, args=(X.float(), Y, mode), timeout=300)
    assert torch.allclose(res[0][0], res[1][0])  # replicas identical
    assert res[0][1] > 0.85
