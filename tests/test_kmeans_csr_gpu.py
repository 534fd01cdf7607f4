"""GPU sparse K-means step (csrc/kmeans_csr.hip) vs the fp64 torch formula on the CPU."""
import pytest
import torch

from harp_amd.models import kmeans_csr as M
from harp_amd.ops import kmeans_csr as KC

pytestmark = pytest.mark.gpu


def _sparse(n, d, density, seed):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, d, generator=g, dtype=torch.float64)
    keep = torch.rand(n, d, generator=g) < density
    keep[:: 17] = False  # some empty rows
    keep[5, :] = True  # one long row (> 64 nonzeros)
    return X * keep


@pytest.mark.parametrize("K", [5, 100, 1500])
def test_assign_accumulate_matches_torch(cuda, K):
    n, d = 4000, 300
    X = _sparse(n, d, 0.05, K)
    C = torch.rand(K, d, dtype=torch.float64, generator=torch.Generator().manual_seed(1)) * 0.3
    D = (X * X).sum(1)[:, None] + (C * C).sum(1)[None, :] - 2 * X @ C.t()
    m_ref, lab_ref = D.clamp_min(0).min(1)
    A = KC.to_device_csr(X.to_sparse_csr().to(cuda))
    lab, m, S, cnt = KC.assign_accumulate(A, C.to(cuda))
    lab, m, S, cnt = lab.cpu(), m.cpu(), S.cpu(), cnt.cpu()
    assert (lab == lab_ref).float().mean() > 0.999
    assert torch.allclose(m, m_ref, rtol=1e-10, atol=1e-9)
    onehot = torch.zeros(n, K, dtype=torch.float64)
    onehot[torch.arange(n), lab] = 1.0
    assert torch.allclose(S, onehot.t() @ X, rtol=1e-12, atol=1e-10)
    assert torch.equal(cnt, onehot.sum(0))


def test_kmeans_sparse_gpu_equals_cpu(cuda):
    X = _sparse(3000, 64, 0.2, 7)
    C0 = X[:12].clone()
    ref = M.kmeans_sparse(X.to_sparse_csr(), C0, 6)
    out = M.kmeans_sparse(X.to_sparse_csr().to(cuda), C0, 6)
    assert torch.allclose(out["centroids"].cpu(), ref["centroids"], atol=1e-10)
    assert all(abs(a - b) <= 1e-9 * abs(b) for a, b in zip(out["objective"], ref["objective"]))
    coo = M.kmeans_sparse(X.to_sparse().to(cuda), C0, 6)  # COO input takes the same kernel
    assert torch.allclose(coo["centroids"].cpu(), ref["centroids"], atol=1e-10)


def test_nan_row_gets_a_valid_label(cuda):
    """a row whose every distance is NaN must not scatter to cluster INT_MAX."""
    X = _sparse(300, 40, 0.3, 3)
    X[7, 3] = float("nan")
    C = torch.rand(9, 40, dtype=torch.float64, generator=torch.Generator().manual_seed(2))
    A = KC.to_device_csr(X.to_sparse_csr().to(cuda))
    lab, m, S, cnt = KC.assign_accumulate(A, C.to(cuda))
    torch.cuda.synchronize()
    lab = lab.cpu()
    assert int(lab.min()) >= 0 and int(lab.max()) < 9
    assert float(cnt.sum()) == 300.0
