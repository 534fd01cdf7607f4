"""EM-GMM HIP kernels (csrc/gmm.hip) vs the PyTorch fp64 E-step / statistics."""
import math
import time

import pytest
import torch

from harp_amd.models import kernels as KF
from harp_amd.ops import gmm as GM

pytestmark = pytest.mark.gpu


def _mixture(n, d, K, seed):
    g = torch.Generator().manual_seed(seed)
    mu = torch.randn(K, d, generator=g, dtype=torch.float64) * 3
    A = torch.randn(K, d, d, generator=g, dtype=torch.float64) * 0.3
    cov = A @ A.transpose(1, 2) + torch.eye(d, dtype=torch.float64)
    w = torch.rand(K, generator=g, dtype=torch.float64) + 0.5
    w = w / w.sum()
    z = torch.randint(0, K, (n,), generator=g)
    L = torch.linalg.cholesky(cov)
    X = mu[z] + (L[z] @ torch.randn(n, d, 1, generator=g, dtype=torch.float64)).squeeze(-1)
    return X, w, mu, cov


def _torch_estep(X, w, mu, cov, covariance):
    logp = KF._log_gauss(X, mu, cov, covariance) + torch.log(w)[None, :]
    lse = torch.logsumexp(logp, 1)
    return torch.exp(logp - lse[:, None]), lse.sum()


@pytest.mark.parametrize("d,K,cov_kind", [(5, 3, "full"), (16, 10, "full"), (32, 64, "full"), (40, 7, "full"), (64, 5, "full"),
                                          (12, 9, "diag")])
def test_estep_and_stats_match_torch(cuda, d, K, cov_kind):
    X, w, mu, cov = _mixture(20000, d, K, d * 100 + K)
    if cov_kind == "diag":
        cov = torch.diagonal(cov, dim1=1, dim2=2).contiguous()
    Xg, wg, mug, covg = (t.to(cuda) for t in (X, w, mu, cov))
    R, ll = GM.estep(Xg, wg, mug, covg, cov_kind)
    Rt, llt = _torch_estep(Xg, wg, mug, covg, cov_kind)
    assert (R - Rt).abs().max().item() < 1e-6
    assert abs(ll.item() - llt.item()) <= 1e-9 * abs(llt.item())
    Nk, S1, S2 = GM.stats(Xg, R, cov_kind)
    assert torch.allclose(Nk, Rt.sum(0), rtol=1e-9, atol=1e-6)
    assert torch.allclose(S1, Rt.t() @ Xg, rtol=1e-9, atol=1e-6)
    S2t = torch.einsum("nk,ni,nj->kij", Rt, Xg, Xg) if cov_kind == "full" else Rt.t() @ (Xg * Xg)
    assert torch.allclose(S2, S2t, rtol=1e-9, atol=1e-5)
    Nk2, _, S22 = GM.stats(Xg, Rt.contiguous(), cov_kind)  # a row-major R is accepted too
    assert torch.allclose(Nk2, Nk, rtol=1e-9, atol=1e-6) and torch.allclose(S22, S2t, rtol=1e-9, atol=1e-5)


def test_em_gmm_native_matches_torch_path(cuda):
    X, w, mu, cov = _mixture(30000, 6, 4, 1)
    init = {"weights": w, "means": mu + 0.5, "covariances": cov}
    a = KF.em_gmm(X.to(cuda), 4, n_iterations=25, accuracy_threshold=0, init=init)
    b = KF.em_gmm(X.to(cuda), 4, n_iterations=25, accuracy_threshold=0, init=init, estep="torch")
    assert torch.allclose(a["means"], b["means"], rtol=1e-8, atol=1e-8)
    assert torch.allclose(a["covariances"], b["covariances"], rtol=1e-8, atol=1e-8)
    assert abs(float(a["loglik"]) - float(b["loglik"])) < 1e-9 * abs(float(b["loglik"]))


def test_em_iteration_1e6(cuda):
    """N = 1e6, d = 32, K = 64: one EM iteration (E-step + statistics) matches the torch
    path; the timing is printed (the >= 10x gate lives in scripts/bench_speedups.py)."""
    X, w, mu, cov = _mixture(1_000_000, 32, 64, 5)
    Xg, wg, mug, covg = (t.to(cuda) for t in (X, w, mu, cov))

    def native():
        R, ll = GM.estep(Xg, wg, mug, covg, "full")
        return GM.stats(Xg, R, "full")

    def ref():
        Rt, _ = _torch_estep(Xg, wg, mug, covg, "full")
        return Rt.sum(0), Rt.t() @ Xg, torch.einsum("nk,ni,nj->kij", Rt, Xg, Xg)

    (nk, sx, sxx), (rk, rx, rxx) = native(), ref()
    for got, want in ((nk, rk), (sx, rx), (sxx, rxx)):
        assert float((got - want).abs().max()) <= 1e-5 * float(want.abs().max()), (got - want).abs().max()
    out = {}
    for name, fn, reps in (("native", native, 5), ("torch", ref, 2)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) / reps
    print(f"EM iteration N=1e6 d=32 K=64: native {out['native'] * 1e3:.2f} ms, torch {out['torch'] * 1e3:.1f} ms, "
          f"{out['torch'] / out['native']:.1f}x")  # ratio asserted in scripts/bench_speedups.py
