"""GPU kNN (csrc/knn.hip: hipBLASLt Q T^T + fused distance / top-k selection) vs an fp64
torch reference of the same search."""
import pytest
import torch

from harp_amd.models.kernels import KNNClassifier
from harp_amd.ops import knn as KN

pytestmark = pytest.mark.gpu


def _ref(train, queries, k):
    D = torch.cdist(queries.double(), train.double()) ** 2
    return torch.topk(D, k, dim=1, largest=False)


@pytest.mark.parametrize("k", [1, 5, 16, 32])
@pytest.mark.parametrize("n,t_tile", [(3001, 1 << 16), (20000, 4096), (37, 1 << 16)])
def test_knn_matches_reference(cuda, k, n, t_tile):
    g = torch.Generator().manual_seed(k * 7 + n)
    d = 24
    train = torch.randn(n, d, generator=g)
    queries = torch.randn(1000, d, generator=g)
    kk = min(k, n)
    rd, ri = _ref(train, queries, kk)
    od, oi = KN.knn_search(train.to(cuda), queries.to(cuda), k, q_tile=384, t_tile=t_tile)
    od, oi = od.cpu().double(), oi.cpu()
    assert od.shape == (1000, kk) and oi.dtype == torch.int64
    assert (od[:, 1:] >= od[:, :-1]).all()
    assert torch.allclose(od, rd, rtol=1e-4, atol=1e-3)
    # indices agree wherever the reference's neighbours are separated from the next one
    exact = (train[oi] - queries[:, None, :]).double().pow(2).sum(-1)
    assert torch.allclose(exact, rd, rtol=1e-4, atol=1e-3)
    assert (oi.sort(1).values == ri.sort(1).values).float().mean() > 0.99


def test_knn_ties_resolve_to_lower_index(cuda):
    train = torch.zeros(700, 8)
    train[::2] += 1.0  # 350 rows at distance 0 from the origin query, 350 at distance 8
    od, oi = KN.knn_search(train.to(cuda), torch.ones(3, 8, device=cuda), 10)
    assert torch.equal(oi.cpu(), torch.arange(0, 20, 2).expand(3, 10))
    assert od.abs().max().item() == 0.0


def test_knn_classifier_on_gpu(cuda):
    g = torch.Generator().manual_seed(3)
    centers = torch.randn(4, 16, generator=g) * 6
    y = torch.randint(0, 4, (4000,), generator=g)
    X = centers[y] + torch.randn(4000, 16, generator=g)
    clf = KNNClassifier(k=7).fit(X[:3000].to(cuda), y[:3000].to(cuda))
    pred = clf.predict(X[3000:].to(cuda)).cpu()
    ref = KNNClassifier(k=7).fit(X[:3000], y[:3000]).predict(X[3000:])
    assert (pred == ref).float().mean() > 0.995
    assert (pred == y[3000:]).float().mean() > 0.97


def test_knn_rejects_unsupported(cuda):
    t = torch.randn(100, 4, device=cuda)
    with pytest.raises(ValueError):
        KN.knn_search(t, t, 33)
    with pytest.raises(TypeError):
        KN.knn_search(t.double(), t.double(), 3)
