"""MFMA SYRK numerics vs torch fp64 on the same bf16-rounded data."""
import pytest
import torch

from harp_amd.ops import linalg as LA

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d", [(1000, 10), (4096, 100), (20000, 257), (3000, 1000)])
def test_gram_stats_matches_fp64(cuda, n, d):
    X = torch.rand(n, d, device=cuda) * 4 - 1
    fm = LA.FeatureMajor.from_rows(X)
    cnt, s, G = LA.gram_stats(fm)
    Xb = X.to(torch.bfloat16).double()
    assert int(cnt.item()) == n
    assert torch.allclose(s.double(), Xb.sum(0), rtol=1e-5, atol=1e-2)
    ref = Xb.t() @ Xb
    assert torch.allclose(G.double(), ref, rtol=2e-5, atol=1e-3 * ref.abs().max().item() * 1e-3 + 1e-2)


def test_feature_major_blocked_layout(cuda):
    X = torch.rand(200, 30, device=cuda)
    D = LA.FeatureMajor.from_rows(X).dense()
    assert D.shape == (128, 384)
    assert torch.equal(D[:30, :200], X.to(torch.bfloat16).t())
    assert bool((D[30, :200] == 1).all()) and int(D[31:].float().abs().sum()) == 0 and int(D[:, 200:].float().abs().sum()) == 0


def test_feature_major_uniform_and_cov(cuda):
    fm = LA.FeatureMajor.uniform(50000, 64, 0.0, 1.0, seed=3, device=cuda)
    assert fm.XT.shape == (50112 // LA.KT, 128, LA.KT)  # sample blocks; samples padded to a multiple of 192
    D = fm.dense()
    assert bool((D[64, :50000] == 1).all()) and int(D[64].float().sum()) == 50000 and int(D[65:].float().abs().sum()) == 0
    assert int(D[:, 50000:].float().abs().sum()) == 0
    cnt, s, G = LA.gram_stats(fm)
    n = cnt.item()
    mean = s.double() / n
    cov = (G.double() - n * torch.outer(mean, mean)) / (n - 1)
    assert abs(n - 50000) < 0.5
    assert torch.allclose(mean, torch.full_like(mean, 0.5), atol=0.01)
    assert torch.allclose(torch.diagonal(cov), torch.full((64,), 1 / 12, dtype=torch.float64, device=cuda), atol=0.003)
    off = cov - torch.diag(torch.diagonal(cov))
    assert off.abs().max() < 0.003


def test_covariance_gpu_matches_cpu(cuda):
    from harp_amd.models import stats as ST

    X = torch.randn(5000, 30, dtype=torch.float64) * 3 + 1
    g = ST.covariance(X.to(cuda).float())
    c = ST.covariance(X.to(torch.bfloat16).double())
    assert torch.allclose(g["covariance"].cpu(), c["covariance"], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("variant", [0])
@pytest.mark.parametrize("n,d", [(4096, 100), (20032, 700), (30016, 1000)])
def test_syrk_variants_agree(cuda, variant, n, d):
    X = torch.rand(n, d, device=cuda) * 2 - 1
    fm = LA.FeatureMajor.from_rows(X)
    G = LA.symmetrize_upper(LA.syrk_t(fm, variant=variant))
    Xb = torch.cat([X.to(torch.bfloat16).double(), torch.ones(n, 1, device=cuda, dtype=torch.float64)], 1)
    ref = Xb.t() @ Xb
    got = G[: d + 1, : d + 1].double()
    assert torch.allclose(got, ref, rtol=2e-5, atol=1e-2), (got - ref).abs().max()


@pytest.mark.parametrize("n,d", [(1, 1), (300, 5), (4096, 16), (70000, 33), (200_000, 64), (64, 64)])
def test_house_tsqr_matches_torch(cuda, n, d):
    """Hand-written fp64 Householder TSQR (csrc/tsqr.hip) vs torch / rocSOLVER QR."""
    g = torch.Generator().manual_seed(n + d)
    A = torch.randn(n, d, generator=g, dtype=torch.float64).to(cuda)
    Q, R = LA.house_tsqr(A)
    assert Q.shape == (n, d) and R.shape == (d, d)
    assert torch.allclose(Q @ R, A, atol=1e-10 * max(1.0, float(A.abs().max())))
    k = min(n, d)
    assert torch.allclose(Q[:, :k].t() @ Q[:, :k], torch.eye(k, dtype=torch.float64, device=cuda), atol=1e-10)
    assert torch.all(torch.diagonal(R) >= 0) and torch.allclose(torch.triu(R), R)
    if n >= d:
        _, Rt = torch.linalg.qr(A)
        Rt = Rt * torch.sign(torch.diagonal(Rt))[:, None]
        assert torch.allclose(R, Rt, atol=1e-9, rtol=1e-9)


def test_distributed_svd_uses_native_tsqr(cuda):
    from harp_amd.models import stats as ST

    A = torch.randn(50_000, 24, dtype=torch.float64, device=cuda)
    out = ST.svd(A)
    s_ref = torch.linalg.svdvals(A)
    assert torch.allclose(out["singularValues"], s_ref, rtol=1e-10)
    U = out["leftSingularMatrix"]
    rec = U @ torch.diag(out["singularValues"]) @ out["rightSingularMatrix"]
    assert torch.allclose(rec, A, atol=1e-9)


@pytest.mark.parametrize("d", [16, 64, 200])
def test_tsqr_auto_cholqr2_on_gpu(cuda, d):
    """GPU tsqr (method auto) = CholeskyQR2 on the fp64 matrix cores: exact QR of a
    well-conditioned tall matrix; an ill-conditioned one falls back to Householder."""
    from harp_amd.models import stats as ST

    g = torch.Generator().manual_seed(d)
    A = (torch.randn(100_000, d, generator=g, dtype=torch.float64) *
         torch.logspace(0, 2, d, dtype=torch.float64)).to(cuda)
    assert ST.cholesky_qr2(A) is not None
    out = ST.tsqr(A)
    Q, R = out["Q"], out["R"]
    assert torch.allclose(Q.t() @ Q, torch.eye(d, dtype=torch.float64, device=cuda), atol=1e-12)
    assert torch.allclose(Q @ R, A, atol=1e-9 * float(A.abs().max()))
    _, Rt = torch.linalg.qr(A)
    Rt = Rt * torch.sign(torch.diagonal(Rt))[:, None]
    assert torch.allclose(R, Rt, rtol=1e-9, atol=1e-8)
    bad = A.clone()
    bad[:, -1] = bad[:, 0] * (1 + 1e-12)  # numerically rank-deficient
    assert ST.cholesky_qr2(bad) is None
    fb = ST.tsqr(bad)
    assert torch.allclose(fb["Q"] @ fb["R"], bad, atol=1e-8 * float(bad.abs().max()))


def test_precision_policy_covariance_1e6x1000(cuda):
    """on 1e6 x 1000 U[0,1) fp32 data the fp32 mode is within 1e-6 (normwise,
    relative) of an fp64 covariance; the bf16 fast path (one bf16 operand, fp32 accumulation,
    sums from the same operand) within 3e-4; fp64 within 1e-10."""
    from harp_amd.models import stats as ST

    g = torch.Generator(device=cuda).manual_seed(9)
    X = torch.rand(1_000_000, 1000, generator=g, device=cuda, dtype=torch.float32)
    X64 = X.double()
    mu = X64.mean(0)
    ref = (X64.t() @ X64 - X64.shape[0] * torch.outer(mu, mu)) / (X64.shape[0] - 1)
    del X64
    nrm = float(ref.abs().max())
    err = {}
    for mode in ("fp32", "bf16", "fp64"):
        err[mode] = float((ST.covariance(X, dtype=mode)["covariance"] - ref).abs().max()) / nrm
    print("covariance relative error by mode:", err)
    # fp64 vs the fp64 reference: both cancel n mu mu^T in fp64 (measured 1.4e-12); bf16
    # measured 3.5e-5 (the one rounding of the operand), fp32 2.8e-7
    assert err["fp32"] <= 1e-6 and err["bf16"] <= 3e-4 and err["fp64"] <= 1e-10, err
    assert ST._policy(X, None) == "fp32"  # an fp32 input is never silently rounded to bf16
