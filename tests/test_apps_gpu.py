"""The application families on the MI355X: each runs on cuda:0 and is checked against
the same code on the CPU (fp64 reference) or a closed form. Runs only on a GPU box."""
import pytest
import torch

from harp_amd.models import als as A
from harp_amd.models import apriori as AP
from harp_amd.models import ccd as CD
from harp_amd.models import graph as G
from harp_amd.models import kernels as KF
from harp_amd.models import mds as MD
from harp_amd.models import mlr as M
from harp_amd.models import nn as NN
from harp_amd.models import optim as O
from harp_amd.models import svm as S
from harp_amd.models import trees as T
from harp_amd.models.sgd_mf import synthetic_ratings
from harp_amd.ops import kmeans as K
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


def test_kmeans_min_distance_output(cuda):
    torch.manual_seed(1)
    n, d, k = 20000, 60, 500
    x = torch.rand(n, d, device=cuda) * 10
    X = K.pack_points(x, cuda)
    c = torch.rand(k, d, device=cuda) * 10
    op = K.prepare(c, X.shape[1])
    md = torch.empty(n, dtype=torch.float32, device=cuda)
    lab, _ = K.assign(X, op, want_objective=False, min_dist=md)
    xb = X[:, :d].double()
    cb = c.to(torch.bfloat16).double()
    ref = ((xb - cb[lab.long()]) ** 2).sum(1)
    assert torch.allclose(md.double(), ref, rtol=1e-3, atol=1e-2 * d)


def test_kmeans_rotation_strategy_single_gpu(cuda):
    from harp_amd.models.kmeans import KMeansConfig, run_kmeans

    g = torch.Generator().manual_seed(0)
    x = torch.rand(5000, 16, generator=g) * 10
    c0 = torch.rand(300, 16, generator=g) * 10
    a = run_kmeans(Communicator(device=cuda), KMeansConfig(5000, 300, 16, 5, "rotation"), x, c0)
    b = run_kmeans(Communicator(device=cuda), KMeansConfig(5000, 300, 16, 5, "allreduce"), x, c0)
    assert torch.allclose(a["centroids"], b["centroids"], atol=1e-2)


def test_trees_on_gpu(cuda):
    from sklearn.datasets import make_classification

    X, y = make_classification(3000, 12, n_informative=6, n_classes=3, random_state=0)
    X, y = torch.tensor(X), torch.tensor(y)
    cpu = T.DecisionTree(max_depth=6).fit(X, y)
    gpu = T.DecisionTree(max_depth=6).fit(X.to(cuda), y.to(cuda))
    agree = (cpu.predict(X) == gpu.predict(X.to(cuda)).cpu()).double().mean()
    assert agree > 0.99
    f = T.DecisionForest(n_trees=8, max_depth=8).fit(X.to(cuda), y.to(cuda))
    assert (f.predict(X.to(cuda)).cpu() == y).double().mean() > 0.85


def test_solvers_kernels_knn_on_gpu(cuda):
    g = torch.Generator().manual_seed(0)
    X = torch.randn(2000, 8, generator=g, dtype=torch.float64)
    beta = torch.randn(8, generator=g, dtype=torch.float64)
    y = X @ beta + 1.0
    r = O.lbfgs(O.MSE(X.to(cuda), y.to(cuda)), n_iterations=60)
    assert torch.allclose(r.minimum.cpu(), torch.cat([torch.ones(1, dtype=torch.float64), beta]), atol=1e-5)
    Q = X[:100]
    assert torch.allclose(KF.rbf_kernel(X.to(cuda), Q.to(cuda)).cpu(), KF.rbf_kernel(X, Q), atol=1e-10)
    lab = (X[:, 0] > 0).long()
    p_cpu = KF.KNNClassifier(5).fit(X, lab).predict(Q)
    p_gpu = KF.KNNClassifier(5).fit(X.to(cuda), lab.to(cuda)).predict(Q.to(cuda)).cpu()
    assert torch.equal(p_cpu, p_gpu)


def test_svm_nn_on_gpu(cuda):
    from sklearn.datasets import make_blobs

    X, y = make_blobs(400, 4, centers=2, cluster_std=2.5, random_state=0)
    X, y = torch.tensor(X), torch.tensor(y)
    m_cpu = S.BinarySVM(kernel="rbf", sigma=2.0).fit(X, y)
    m_gpu = S.BinarySVM(kernel="rbf", sigma=2.0).fit(X.to(cuda), y.to(cuda))
    assert torch.allclose(m_cpu.decision(X), m_gpu.decision(X.to(cuda)).cpu(), atol=1e-6)
    net = NN.MLP([4, 16, 2], device=cuda)
    Y = torch.nn.functional.one_hot(y, 2).float().to(cuda)
    Xn = ((X - X.mean(0)) / X.std(0)).float().to(cuda)
    NN.train_model_averaging(Communicator(device=cuda), net, Xn, Y, epochs=20, batch=32, lr=0.5)
    assert (net.predict(Xn).cpu() == y).double().mean() > 0.9


def test_mf_family_on_gpu(cuda):
    u, i, v = synthetic_ratings(300, 200, 6000, seed=0, true_rank=4)
    key = torch.unique(u * 200 + i)
    u, i = key // 200, key % 200
    v = torch.rand(u.numel(), dtype=torch.float64) * 4 + 1
    for fn, cfg in ((A.train_als, A.ALSConfig(factors=8, iterations=3)),
                    (CD.train_ccd, CD.CCDConfig(rank=8, iterations=3))):
        a = fn(Communicator(device="cpu"), u, i, v, 300, 200, cfg)
        b = fn(Communicator(device=cuda), u, i, v, 300, 200, cfg)
        key0 = "X" if "X" in a else "W"
        assert torch.allclose(a[key0].float(), b[key0].cpu().float(), atol=2e-3, rtol=1e-3)


def test_graph_mds_apriori_mlr_on_gpu(cuda):
    E = [(a, (a * 7 + 3) % 50) for a in range(50)] + [(a, (a + 1) % 50) for a in range(50)]
    E = sorted({(min(a, b), max(a, b)) for a, b in E if a != b})
    src = torch.tensor([a for a, b in E] + [b for a, b in E])
    dst = torch.tensor([b for a, b in E] + [a for a, b in E])
    tpl = G.Template(4, [(0, 1), (1, 2), (1, 3)])
    colors = torch.randint(0, 4, (50,), generator=torch.Generator().manual_seed(0))
    assert G.color_count(Communicator(device="cpu"), tpl, src, dst, 50, colors) == \
        G.color_count(Communicator(device=cuda), tpl, src, dst, 50, colors)
    nodes = torch.arange(50)
    pr_c = G.pagerank(Communicator(device="cpu"), src, dst, nodes, 50)
    pr_g = G.pagerank(Communicator(device=cuda), src, dst, nodes, 50)
    assert torch.allclose(pr_c, pr_g.cpu(), atol=1e-14)
    Y = torch.rand(30, 3, dtype=torch.float64)
    D = torch.cdist(Y, Y)
    W = torch.ones(30, 30, dtype=torch.float64)
    out = MD.wda_mds(Communicator(device=cuda), D, W, 0, 30, MD.MDSConfig(d=3, alpha=0.9, threshold=1e-7))
    assert out["stress"] < 1e-3
    Tm = (torch.rand(500, 10, generator=torch.Generator().manual_seed(1)) < 0.3).float()
    a = AP.apriori(Tm, 0.05, 0.5)
    b = AP.apriori(Tm.to(cuda), 0.05, 0.5)
    assert a["large_itemsets"].keys() == b["large_itemsets"].keys()
    Xs, Ys = M.synthetic_multilabel(300, 40, 3, density=0.2)
    r_c = M.train(Communicator(device="cpu"), M.CSRRows.from_dense(Xs), Ys, M.MLRConfig(batch_size=16), 3, 40)
    r_g = M.train(Communicator(device=cuda), M.CSRRows.from_dense(Xs), Ys, M.MLRConfig(batch_size=16), 3, 40)
    assert torch.allclose(r_c["W"], r_g["W"].cpu(), atol=1e-8)
