"""CPU kNN path (the oracle of the GPU kernel): torch distance tile + topk."""
import torch

from harp_amd.ops import knn as KN


def test_cpu_knn_matches_cdist():
    g = torch.Generator().manual_seed(0)
    train, queries = torch.randn(500, 6, generator=g), torch.randn(40, 6, generator=g)
    d, i = KN.knn_search(train, queries, 5, q_tile=16)
    rd, ri = torch.topk(torch.cdist(queries.double(), train.double()) ** 2, 5, dim=1, largest=False)
    assert torch.allclose(d.double(), rd, rtol=1e-4, atol=1e-4)
    assert torch.equal(i, ri)
    assert KN.knn_search(train[:3], queries, 5)[0].shape == (40, 3)
