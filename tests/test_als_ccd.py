"""ALS (implicit + explicit) and MF-CCD: batched solvers vs per-row dense references,
and P=2 gloo runs vs the single-worker result (the algorithms are P-invariant)."""
import pytest
import torch

from harp_amd.models import als as A
from harp_amd.models import ccd as CD
from harp_amd.models.sgd_mf import synthetic_ratings
from harp_amd.parallel.comm import Communicator
from harp_amd.runtime.launcher import launch


def _data(nu=40, ni=30, nr=400, seed=0):
    u, i, v = synthetic_ratings(nu, ni, nr, seed=seed, true_rank=3)
    key = u * ni + i
    k, idx = torch.unique(key, return_inverse=True)
    first = torch.full((k.numel(),), len(key), dtype=torch.long).scatter_reduce(0, idx, torch.arange(len(key)), "amin")
    return u[first], i[first], v[first].double()


def _dense_rows(u, i, v, nu, F, cfg):
    f = F.shape[1]
    out = torch.zeros(nu, f, dtype=torch.float64)
    for r in range(nu):
        m = u == r
        Fi, vi = F[i[m]], v[m]
        if cfg.implicit:
            c = 1 + cfg.alpha * vi
            Am = F.t() @ F + Fi.t() @ ((c - 1)[:, None] * Fi) + cfg.lam * torch.eye(f, dtype=torch.float64)
            b = Fi.t() @ c
        else:
            Am = Fi.t() @ Fi + cfg.lam * max(int(m.sum()), 1) * torch.eye(f, dtype=torch.float64)
            b = Fi.t() @ vi
        out[r] = torch.linalg.solve(Am, b)
    return out


def test_als_solver_matches_dense():
    u, i, v = _data()
    F = torch.rand(30, 4, dtype=torch.float64)
    for implicit in (True, False):
        cfg = A.ALSConfig(factors=4, lam=0.1, alpha=2.0, implicit=implicit, block_bytes=4096)
        o = torch.argsort(u, stable=True)
        got = A.solve_rows(u[o], i[o], v[o], 40, F, cfg)
        ref = _dense_rows(u, i, v, 40, F, cfg)
        assert torch.allclose(got, ref, atol=1e-9), implicit


def test_als_implicit_loss_decreases():
    u, i, v = _data()
    cfg = A.ALSConfig(factors=4, lam=0.1, alpha=2.0, iterations=6)
    losses = []
    for n in range(1, 6):
        cfg.iterations = n
        r = A.train_als_batch(u, i, v, 40, 30, cfg)
        losses.append(A.implicit_loss(u, i, v, r["X"], r["Y"], cfg))
    assert all(b <= a + 1e-9 for a, b in zip(losses, losses[1:])), losses


def _als_job(comm, u, i, v, explicit):
    n = u.numel()
    P, r = comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    cfg = A.ALSConfig(factors=4, lam=0.1, alpha=2.0, iterations=3, implicit=not explicit)
    out = A.train_als(comm, u[sl], i[sl], v[sl], 40, 30, cfg, test=(u, i, v))
    return out["X"], out["user_ids"], out["history"][-1]["test_rmse"]


def test_als_distributed_equals_single():
    u, i, v = _data()
    for explicit in (False, True):
        cfg = A.ALSConfig(factors=4, lam=0.1, alpha=2.0, iterations=3, implicit=not explicit)
        single = A.train_als(Communicator(), u, i, v, 40, 30, cfg, test=(u, i, v))
        res = launch(_als_job, 2, args=(u, i, v, explicit), timeout=300)
        for X, ids, rm in res:
            assert torch.allclose(X, single["X"][ids], atol=1e-8)
            assert abs(rm - single["history"][-1]["test_rmse"]) < 1e-8
    # explicit ALS fits the ratings
    assert single["history"][-1]["test_rmse"] < 0.6


def _ccd_seq(u, i, v, nu, ni, k, lam, iters, W0, H0):
    """Reference-order CCD (CCDMPTask.doRowCCD / doColCCD) with explicit loops."""
    W, H = W0.clone(), H0.clone()
    for _ in range(iters):
        for r in range(nu):
            m = torch.nonzero(u == r).reshape(-1)
            res = v[m] - (W[r] * H[i[m]]).sum(1)
            for t in range(k):
                h = H[i[m], t]
                up = ((res + W[r, t] * h) * h).sum()
                down = lam * m.numel() + (h * h).sum()
                z = up / down if down > 0 else W[r, t]
                res -= (z - W[r, t]) * h
                W[r, t] = z
        for c in range(ni):
            m = torch.nonzero(i == c).reshape(-1)
            res = v[m] - (H[c] * W[u[m]]).sum(1)
            for t in range(k):
                w = W[u[m], t]
                up = ((res + H[c, t] * w) * w).sum()
                down = lam * m.numel() + (w * w).sum()
                z = up / down if down > 0 else H[c, t]
                res -= (z - H[c, t]) * w
                H[c, t] = z
    return W, H


def test_ccd_matches_sequential_reference():
    u, i, v = _data()
    cfg = CD.CCDConfig(rank=3, lam=0.05, iterations=3)
    out = CD.train_ccd(Communicator(), u, i, v, 40, 30, cfg)
    g = torch.Generator().manual_seed(0)
    W0 = torch.rand((40, 3), generator=g, dtype=torch.float64) * 3 ** -0.5
    H0 = torch.rand((30, 3), generator=g, dtype=torch.float64) * 3 ** -0.5
    W, H = _ccd_seq(u, i, v, 40, 30, 3, 0.05, 3, W0, H0)
    assert torch.allclose(out["W"], W, atol=1e-10)
    assert torch.allclose(out["H"], H, atol=1e-10)
    rm = [h["train_rmse"] for h in out["history"]]
    assert rm[-1] < rm[0]


def _ccd_job(comm, u, i, v):
    n = u.numel()
    P, r = comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    out = CD.train_ccd(comm, u[sl], i[sl], v[sl], 40, 30, CD.CCDConfig(rank=3, lam=0.05, iterations=3), test=(u, i, v))
    return out["W"], out["user_ids"], out["history"]


def test_ccd_distributed_equals_single():
    u, i, v = _data()
    single = CD.train_ccd(Communicator(), u, i, v, 40, 30, CD.CCDConfig(rank=3, lam=0.05, iterations=3))
    res = launch(_ccd_job, 3, args=(u, i, v), timeout=300)
    for W, ids, hist in res:
        assert torch.allclose(W, single["W"][ids], atol=1e-10)
        assert abs(hist[-1]["train_rmse"] - single["history"][-1]["train_rmse"]) < 1e-10


def _ccd_modes(comm, mode, S):
    from harp_amd.models.ccd import CCDConfig, train_ccd

    g = torch.Generator().manual_seed(9)
    n = 4000
    u = torch.randint(0, 150, (n,), generator=g)
    i = torch.randint(0, 60, (n,), generator=g)
    v = torch.rand(n, generator=g) * 4 + 1
    P, r = comm.world_size, comm.rank
    sl = slice(r * n // P, (r + 1) * n // P)
    res = train_ccd(comm, u[sl], i[sl], v[sl], 150, 60, CCDConfig(rank=7, iterations=6, mode=mode, slices_per_rank=S))
    return {"W": res["W"].cpu(), "uid": res["user_ids"].cpu(), "rmse": [h["train_rmse"] for h in res["history"]],
            "slab": res.get("slab_floats_per_rank")}


@pytest.mark.parametrize("S", [1, 2])
def test_ccd_rotation_mode_one_rank_equals_allgather(S):
    from harp_amd.parallel.comm import Communicator

    c = Communicator(None, torch.device("cpu"))
    a = _ccd_modes(c, "allgather", S)
    b = _ccd_modes(c, "rotation", S)
    assert torch.allclose(a["W"], b["W"], atol=1e-10)
    assert a["rmse"] == pytest.approx(b["rmse"], rel=1e-10)


@pytest.mark.parametrize("P", [2, 3])
def test_ccd_rotation_mode_multi_rank(P):
    rot = launch(_ccd_modes, P, args=("rotation", 2), timeout=300)
    ag = launch(_ccd_modes, P, args=("allgather", 2), timeout=300)
    # both descend; different (valid) dimension orders give close fits
    assert rot[0]["rmse"][-1] < rot[0]["rmse"][0]
    assert rot[0]["rmse"][-1] == pytest.approx(ag[0]["rmse"][-1], rel=0.05)
    # memory: a rank holds S slices of (m + n) x ceil(r / (S P)) floats, not a full factor
    rs = -(-7 // (2 * P))
    assert rot[0]["slab"] == 2 * (P * -(-150 // P) + P * -(-60 // P)) * rs


def test_ccd_residual_carry_equals_recompute():
    """One worker carries a phase's residuals to the other order by permutation; it must
    match recomputing them before every phase (ResTask, residual_resync=1)."""
    u, i, v = _data()
    a = CD.train_ccd(Communicator(), u, i, v, 40, 30, CD.CCDConfig(rank=3, lam=0.05, iterations=7, residual_resync=1))
    b = CD.train_ccd(Communicator(), u, i, v, 40, 30, CD.CCDConfig(rank=3, lam=0.05, iterations=7, residual_resync=3))
    assert torch.allclose(a["W"], b["W"], atol=1e-10) and torch.allclose(a["H"], b["H"], atol=1e-10)
    for ha, hb in zip(a["history"], b["history"]):
        assert abs(ha["train_rmse"] - hb["train_rmse"]) < 1e-10
