"""Cooperative kernels under CU contention: at P > 1 RCCL kernels share the
CUs with the one-XCD eigensolver (csrc/eig.hip) and the 16-CU SMO (csrc/svm.hip). A bounded
CU hog on a second stream occupies 28 of every XCD's 32 CUs (160 KB of LDS each, so nothing
else fits there) while the cooperative kernel runs: it must either complete cooperatively
(the hog ended inside its spin budget) or take its documented fallback -- with the same
results, and never hang."""
import warnings

import pytest
import torch

from harp_amd.ops import eig as EIG
from harp_amd.ops.testutil import cu_hog

pytestmark = pytest.mark.gpu

HOG_BLOCKS = 28 * 8  # one 160-KB workgroup per CU on 28 CUs of each XCD


def _corr(cuda, n=600):
    g = torch.Generator(device=cuda).manual_seed(2)
    X = torch.rand(10 * n, n, generator=g, device=cuda, dtype=torch.float64)
    Xc = X - X.mean(0)
    C = Xc.t() @ Xc
    sd = torch.sqrt(torch.diagonal(C))
    return C / torch.outer(sd, sd)


@pytest.mark.parametrize("hog_us", [20_000, 1_000_000])
def test_eigensolver_under_contention(cuda, hog_us):
    C = _corr(cuda)
    ref_w = torch.linalg.eigvalsh(C)
    side = torch.cuda.Stream(cuda)
    torch.cuda.synchronize()
    done = cu_hog(HOG_BLOCKS, 160 * 1024, hog_us, side)
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        w = EIG.eigvalsh(C)
        lam, V = EIG.eigh(C)
    torch.cuda.synchronize()
    assert int(done.item()) == HOG_BLOCKS  # the hog drained
    fell_back = any("did not run cooperatively" in str(r.message) for r in rec)
    print(f"hog {hog_us} us: fallback={fell_back}")
    assert float((w - ref_w).abs().max()) <= 1e-12
    assert float((lam - ref_w).abs().max()) <= 1e-12
    eye = torch.eye(C.shape[0], dtype=torch.float64, device=cuda)
    assert float((V.t() @ V - eye).abs().max()) <= 1e-12
    assert float((C @ V - V * lam).abs().max()) <= 1e-11


@pytest.mark.parametrize("hog_us", [20_000, 1_000_000])
def test_coop_smo_under_contention(cuda, hog_us):
    from harp_amd.models.svm import BinarySVM, kernel_matrix

    g = torch.Generator().manual_seed(7)
    n = 12000
    y = torch.randint(0, 2, (n,), generator=g)
    X = (torch.randn(2, 16, generator=g) * 0.5)[y] + torch.randn(n, 16, generator=g)
    Xg, yg = X.double().to(cuda), y.to(cuda)
    K = kernel_matrix(Xg, Xg, "rbf", 4.0)
    base = BinarySVM(C=1.0, kernel="rbf", sigma=4.0).fit(Xg, yg, K)
    side = torch.cuda.Stream(cuda)
    torch.cuda.synchronize()
    done = cu_hog(HOG_BLOCKS, 160 * 1024, hog_us, side)
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        m = BinarySVM(C=1.0, kernel="rbf", sigma=4.0).fit(Xg, yg, K)
    torch.cuda.synchronize()
    assert int(done.item()) == HOG_BLOCKS
    fell_back = any("cooperative SMO did not run" in str(r.message) for r in rec)
    print(f"hog {hog_us} us: fallback={fell_back}, steps {m.n_iterations} vs {base.n_iterations}")
    # the one-CU kernel follows the cooperative kernel's exact trajectory
    # (tests/test_svm_gpu.py::test_coop_smo_matches_one_cu_kernel)
    assert m.n_iterations == base.n_iterations
    assert torch.equal(m.alpha, base.alpha)
