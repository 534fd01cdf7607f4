"""Decision tree / forest / boosting (DAAL dtree, dforest, stump, adaboost, brownboost,
logitboost; contrib RF) against sklearn on synthetic data, plus the distributed forest
on 2 gloo workers (trees all-gathered as Writables)."""
import pytest
import torch

from harp_amd.core.writable import DataInput, DataOutput
from harp_amd.models import trees as T
from harp_amd.runtime.launcher import launch

sk_ds = pytest.importorskip("sklearn.datasets")


@pytest.fixture(scope="module")
def cls_data():
    X, y = sk_ds.make_classification(3000, 16, n_informative=8, n_classes=3, random_state=0)
    X, y = torch.tensor(X), torch.tensor(y)
    return X[:2000], y[:2000], X[2000:], y[2000:]


def _acc(m, X, y):
    return (m.predict(X) == y).double().mean().item()


def test_tree_matches_sklearn_accuracy(cls_data):
    from sklearn.tree import DecisionTreeClassifier

    Xtr, ytr, Xte, yte = cls_data
    ours = _acc(T.DecisionTree(max_depth=6, n_bins=128).fit(Xtr, ytr), Xte, yte)
    ref = DecisionTreeClassifier(max_depth=6, random_state=0).fit(Xtr, ytr).score(Xte, yte)
    assert ours > ref - 0.04
    ent = _acc(T.DecisionTree(max_depth=6, criterion="entropy").fit(Xtr, ytr), Xte, yte)
    assert ent > ref - 0.05


def test_tree_exact_separable():
    # axis-aligned labels are learned exactly
    g = torch.Generator().manual_seed(1)
    X = torch.rand(500, 3, generator=g, dtype=torch.float64)
    y = ((X[:, 0] > 0.5) ^ (X[:, 2] > 0.3)).long()
    t = T.DecisionTree(max_depth=3, n_bins=256).fit(X, y)
    assert _acc(t, X, y) > 0.98
    leaves = t.apply(X)
    assert (t.left[leaves] < 0).all()


def test_regression_tree_and_forest():
    from sklearn.tree import DecisionTreeRegressor

    X, y = sk_ds.make_regression(2000, 8, noise=1.0, random_state=0)
    X, y = torch.tensor(X), torch.tensor(y)
    t = T.DecisionTree("regression", max_depth=7, n_bins=128).fit(X[:1500], y[:1500])
    mse = ((t.predict(X[1500:]) - y[1500:]) ** 2).mean().item()
    ref = DecisionTreeRegressor(max_depth=7, random_state=0).fit(X[:1500], y[:1500]).predict(X[1500:].numpy())
    ref_mse = ((torch.tensor(ref) - y[1500:]) ** 2).mean().item()
    assert mse < 1.2 * ref_mse
    f = T.DecisionForest("regression", n_trees=15, max_depth=9, max_features=None).fit(X[:1500], y[:1500])
    assert ((f.predict(X[1500:]) - y[1500:]) ** 2).mean().item() < mse


def test_forest_beats_tree(cls_data):
    Xtr, ytr, Xte, yte = cls_data
    f = T.DecisionForest(n_trees=25, max_depth=10).fit(Xtr, ytr)
    t = T.DecisionTree(max_depth=10).fit(Xtr, ytr)
    assert _acc(f, Xte, yte) > _acc(t, Xte, yte)
    p = f.predict_proba(Xte)
    assert torch.allclose(p.sum(1), torch.ones(len(Xte), dtype=p.dtype))


def test_boosting(cls_data):
    Xtr, ytr, Xte, yte = cls_data
    st = _acc(T.stump(Xtr, ytr, num_classes=3), Xte, yte)
    ada = T.AdaBoost(40, learner_depth=2).fit(Xtr, ytr)
    assert _acc(ada, Xte, yte) > st + 0.05
    lb = T.LogitBoost(25).fit(Xtr, ytr)
    assert _acc(lb, Xte, yte) > st + 0.05
    yb, ybt = (ytr == 0).long(), (yte == 0).long()
    bb = T.BrownBoost(c=3.0, max_rounds=60).fit(Xtr, yb)
    assert len(bb.alphas) > 1
    assert _acc(bb, Xte, ybt) > _acc(T.stump(Xtr, yb), Xte, ybt)


def test_tree_writable_roundtrip(cls_data):
    Xtr, ytr, Xte, _ = cls_data
    t = T.DecisionTree(max_depth=4).fit(Xtr, ytr)
    out = DataOutput()
    t.write(out)
    t2 = T.DecisionTree()
    t2.read(DataInput(out.getvalue()))
    assert torch.equal(t.predict(Xte), t2.predict(Xte))


def _rf_job(comm, X, y):
    P, r = comm.world_size, comm.rank
    n = X.shape[0]
    sl = slice(r * n // P, (r + 1) * n // P)
    f = T.DecisionForest(n_trees=10, max_depth=8, seed=3).fit_distributed(X[sl], y[sl], comm, num_classes=3)
    return len(f.trees), f.predict(X)


def test_distributed_forest(cls_data):
    Xtr, ytr, Xte, yte = cls_data
    res = launch(_rf_job, 2, args=(Xtr, ytr), timeout=300)
    assert res[0][0] == res[1][0] == 10
    assert torch.equal(res[0][1], res[1][1])  # every worker holds the same forest
    assert (res[0][1] == ytr).double().mean().item() > 0.8
