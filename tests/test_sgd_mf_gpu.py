"""GPU MF-SGD kernels vs the native sequential CPU reference / torch."""
import pytest
import torch

from harp_amd.ops import mf as MF
from harp_amd.models.sgd_mf import SGDConfig, run_sgd, synthetic_ratings
from harp_amd.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("r", [16, 48, 128])
def test_sse_matches_torch(cuda, r):
    n, nu, ni = 50000, 1000, 300
    g = torch.Generator().manual_seed(r)
    rows = torch.randint(0, nu, (n,), generator=g, dtype=torch.int32)
    cols = torch.randint(0, ni, (n,), generator=g, dtype=torch.int32)
    vals = torch.rand(n, generator=g) * 4 + 1
    W = torch.rand(nu, r, generator=g) * 0.3
    H = torch.rand(ni, r, generator=g) * 0.3
    ref = ((vals.double() - (W[rows.long()].double() * H[cols.long()].double()).sum(1)) ** 2).sum()
    got = MF.sse(rows.to(cuda), cols.to(cuda), vals.to(cuda), W.to(cuda), H.to(cuda))
    assert abs(got.item() - ref.item()) <= 1e-5 * ref.item()


def test_sgd_single_stream_matches_sequential(cuda):
    """chunk >= n -> one stream -> exactly the sequential order of the CPU reference."""
    n, nu, ni, r = 3000, 40, 30, 16
    g = torch.Generator().manual_seed(0)
    rows = torch.sort(torch.randint(0, nu, (n,), generator=g, dtype=torch.int32)).values
    cols = torch.randint(0, ni, (n,), generator=g, dtype=torch.int32)
    vals = torch.rand(n, generator=g) * 4 + 1
    W0 = torch.rand(nu, r, generator=g) * 0.3
    H0 = torch.rand(ni, r, generator=g) * 0.3
    Wc, Hc = W0.clone(), H0.clone()
    MF.sgd_update(rows, cols, vals, Wc, Hc, 0.01, 0.05)
    Wg, Hg = W0.to(cuda), H0.to(cuda)
    MF.sgd_update(rows.to(cuda), cols.to(cuda), vals.to(cuda), Wg, Hg, 0.01, 0.05, chunk=n)
    assert torch.allclose(Wg.cpu(), Wc, atol=2e-5) and torch.allclose(Hg.cpu(), Hc, atol=2e-5)


def test_sgd_gpu_converges_like_cpu(cuda):
    nu, ni = 3000, 800
    u, i, v = synthetic_ratings(nu, ni, 120000, seed=2)
    p = torch.randperm(u.numel(), generator=torch.Generator().manual_seed(0))
    k = int(0.9 * u.numel())
    train = (u[p[:k]], i[p[:k]], v[p[:k]])
    test = (u[p[k:]], i[p[k:]], v[p[k:]])
    cfg = SGDConfig(rank=32, lam=0.05, lr=0.01, epochs=10, test_every=10)
    g = run_sgd(Communicator(None, cuda), cfg, nu, ni, train, test)
    c = run_sgd(Communicator(None, torch.device("cpu")), cfg, nu, ni, train, test)
    # ~1.7k concurrent Hogwild streams on only 800 items: staleness costs a little accuracy
    assert abs(g["rmse"][-1][2] - c["rmse"][-1][2]) < 0.04, (g["rmse"], c["rmse"])
    assert g["trained"] == c["trained"] == 10 * k


def _cells(nu, ni, n, r, seed):
    g = torch.Generator().manual_seed(seed)
    rows = torch.randint(0, nu, (n,), generator=g)
    cols = torch.randint(0, ni, (n,), generator=g)
    vals = torch.rand(n, generator=g) * 4 + 1
    cid = MF.cell_layout(rows, cols, nu, ni)
    order = torch.argsort(cid * nu + rows)
    off = torch.zeros(65, dtype=torch.int64)
    off[1:] = torch.cumsum(torch.bincount(cid, minlength=64), 0)
    W0 = torch.rand(nu, r, generator=g) * 0.3
    H0 = torch.rand(ni, r, generator=g) * 0.3
    return rows[order].int(), cols[order].int(), vals[order].float(), off, W0, H0


@pytest.mark.parametrize("r", [16, 128])
def test_sgd_xcd_one_stream_per_cell_matches_cpu(cuda, r):
    """chunk >= cell size: one stream per cell, and the 8 cells of a sub-step share no user
    and no item, so the XCD-blocked kernel is deterministic and equals the CPU schedule
    (including the in-register forwarding of repeated items: 64 users x 48 items)."""
    R, C, V, off, W0, H0 = _cells(64, 48, 4000, r, 1)
    assert int((off[1:] - off[:-1]).max()) <= 128
    Wc, Hc = W0.clone(), H0.clone()
    MF.sgd_update_blocked(R, C, V, off, Wc, Hc, 0.01, 0.05)
    Wg, Hg = W0.to(cuda), H0.to(cuda)
    MF.sgd_update_blocked(R.to(cuda), C.to(cuda), V.to(cuda), off.to(cuda), Wg, Hg, 0.01, 0.05, chunk=128,
                          blocks_per_xcd=4)
    torch.cuda.synchronize()
    assert torch.allclose(Wg.cpu(), Wc, atol=2e-5) and torch.allclose(Hg.cpu(), Hc, atol=2e-5)


def test_sgd_xcd_many_streams_close_to_cpu(cuda):
    """Hogwild inside each cell (~780 streams on ~100 items per XCD): after a few passes the
    error lands close to the sequential schedule's (H rows are read from L2, so concurrent
    streams see each other's updates)."""
    R, C, V, off, W0, H0 = _cells(3000, 800, 200000, 32, 2)
    Wc, Hc = W0.clone(), H0.clone()
    Wg, Hg = W0.to(cuda), H0.to(cuda)
    Rg, Cg, Vg, og = R.to(cuda), C.to(cuda), V.to(cuda), off.to(cuda)
    for _ in range(5):
        MF.sgd_update_blocked(R, C, V, off, Wc, Hc, 0.005, 0.05)
        MF.sgd_update_blocked(Rg, Cg, Vg, og, Wg, Hg, 0.005, 0.05, chunk=32)
    torch.cuda.synchronize()
    e0 = MF.sse(R, C, V, W0, H0).item()
    e_cpu = MF.sse(R, C, V, Wc, Hc).item()
    e_gpu = MF.sse(Rg, Cg, Vg, Wg, Hg).item()
    print(f"sse initial {e0:.4g} cpu {e_cpu:.4g} gpu-xcd {e_gpu:.4g}")
    assert e_gpu < 0.5 * e0
    assert abs(e_gpu - e_cpu) < 0.1 * e_cpu, (e_gpu, e_cpu)


def test_sgd_xcd_windows_match_cpu(cuda):
    """Fixed-fraction windows (wrapping around each cell) give the CPU schedule's result."""
    R, C, V, off, W0, H0 = _cells(64, 48, 4000, 32, 3)
    host = off.tolist()
    win = MF.cell_windows(host, 0.4, epoch=2)  # starts past the middle: windows wrap
    assert any(s + l > host[c + 1] - host[c] for c, (s, l) in enumerate(zip(*win)))
    Wc, Hc = W0.clone(), H0.clone()
    nc = MF.sgd_update_blocked(R, C, V, off, Wc, Hc, 0.01, 0.05, window=win)
    Wg, Hg = W0.to(cuda), H0.to(cuda)
    ng = MF.sgd_update_blocked(R.to(cuda), C.to(cuda), V.to(cuda), off.to(cuda), Wg, Hg, 0.01, 0.05, chunk=128,
                               blocks_per_xcd=4, window=win)
    torch.cuda.synchronize()
    assert nc == ng == sum(win[1])
    assert torch.allclose(Wg.cpu(), Wc, atol=2e-5) and torch.allclose(Hg.cpu(), Hc, atol=2e-5)


# ---- wide ranks (wave-per-stream kernels; BASELINE #1 trains rank 2000) ----

@pytest.mark.parametrize("r", [260, 1000, 2000, 3000])
def test_sse_wide_rank_matches_torch(cuda, r):
    n, nu, ni = 20000, 500, 300
    g = torch.Generator().manual_seed(r)
    rows = torch.randint(0, nu, (n,), generator=g, dtype=torch.int32)
    cols = torch.randint(0, ni, (n,), generator=g, dtype=torch.int32)
    vals = torch.rand(n, generator=g) * 4 + 1
    s = 0.3 * (16.0 / r) ** 0.5
    W = torch.rand(nu, r, generator=g) * s
    H = torch.rand(ni, r, generator=g) * s
    ref = ((vals.double() - (W[rows.long()].double() * H[cols.long()].double()).sum(1)) ** 2).sum()
    got = MF.sse(rows.to(cuda), cols.to(cuda), vals.to(cuda), W.to(cuda), H.to(cuda))
    assert abs(got.item() - ref.item()) <= 1e-5 * ref.item()


@pytest.mark.parametrize("r", [512, 2000])
def test_sgd_wide_single_stream_matches_sequential(cuda, r):
    n, nu, ni = 2000, 40, 30
    g = torch.Generator().manual_seed(0)
    rows = torch.sort(torch.randint(0, nu, (n,), generator=g, dtype=torch.int32)).values
    cols = torch.randint(0, ni, (n,), generator=g, dtype=torch.int32)
    vals = torch.rand(n, generator=g) * 4 + 1
    s = 0.3 * (16.0 / r) ** 0.5
    W0 = torch.rand(nu, r, generator=g) * s
    H0 = torch.rand(ni, r, generator=g) * s
    Wc, Hc = W0.clone(), H0.clone()
    MF.sgd_update(rows, cols, vals, Wc, Hc, 0.002, 0.05)
    Wg, Hg = W0.to(cuda), H0.to(cuda)
    MF.sgd_update(rows.to(cuda), cols.to(cuda), vals.to(cuda), Wg, Hg, 0.002, 0.05, chunk=n)
    assert torch.allclose(Wg.cpu(), Wc, atol=2e-5, rtol=1e-4) and torch.allclose(Hg.cpu(), Hc, atol=2e-5, rtol=1e-4)


def test_sgd_wide_xcd_one_stream_per_cell_matches_cpu(cuda):
    """Rank 2000 through the XCD-blocked schedule, one stream per cell: equals the CPU
    schedule; strided rows (a view of a wider buffer) are honoured."""
    r = 2000
    R, C, V, off, W0, H0 = _cells(64, 48, 4000, r, 1)
    W0 *= (16.0 / r) ** 0.5
    H0 *= (16.0 / r) ** 0.5
    assert int((off[1:] - off[:-1]).max()) <= 128
    Wc, Hc = W0.clone(), H0.clone()
    MF.sgd_update_blocked(R, C, V, off, Wc, Hc, 0.002, 0.05)
    Wbuf = torch.zeros(64, r + 48, device=cuda)
    Wg = Wbuf[:, :r]
    Wg.copy_(W0)
    Hg = H0.to(cuda)
    MF.sgd_update_blocked(R.to(cuda), C.to(cuda), V.to(cuda), off.to(cuda), Wg, Hg, 0.002, 0.05, chunk=128)
    torch.cuda.synchronize()
    assert torch.allclose(Wg.cpu(), Wc, atol=2e-5, rtol=1e-4) and torch.allclose(Hg.cpu(), Hc, atol=2e-5, rtol=1e-4)
    assert bool((Wbuf[:, r:] == 0).all())  # nothing written past the rank


def test_sgd_wide_rank_model_converges(cuda):
    nu, ni = 2000, 600
    u, i, v = synthetic_ratings(nu, ni, 80000, seed=5)
    cfg = SGDConfig(rank=1000, lam=0.05, lr=0.002, epochs=6, test_every=3)
    res = run_sgd(Communicator(None, cuda), cfg, nu, ni, (u, i, v), (u[:5000], i[:5000], v[:5000]))
    rm = [x[2] for x in res["rmse"]]
    assert rm[-1] < rm[0], res["rmse"]


def test_sgd_time_budget_xcd_path(cuda):
    """Time-bounded steps on the XCD-blocked kernel: an unbounded budget trains every
    rating each epoch, a tiny one exactly one piece (a window of every cell) per step."""
    from harp_amd.models.sgd_mf import SGDConfig, SGDCollectiveMapper, synthetic_ratings
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    tr = synthetic_ratings(20000, 3000, 400_000, seed=3, device=cuda)
    out = {}
    for name, b in (("full", 1e9), ("tiny", 1e-6)):
        cfg = SGDConfig(rank=32, epochs=2, test_every=0, time_budget_ms=b, budget_pieces=8)
        m = SGDCollectiveMapper(Communicator(None, cuda), cfg, 20000, 3000, tr, None)
        m.run(KeyValReader([]))
        out[name] = m.trained
    assert out["full"] == 2 * 400_000
    assert 0.1 * 800_000 < out["tiny"] < 0.16 * 800_000


def test_sgd_one_slice_per_rank_like_two(cuda):
    """bench.py's MF-SGD record runs one H slice per rank (half the sub-step launches,
    profiles/r3_sgd_slices): every rating is still trained once per epoch and the model
    converges like the two-slice rotation."""
    from harp_amd.models.sgd_mf import SGDCollectiveMapper
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    nu, ni, n = 20000, 3000, 600000
    u, i, v = synthetic_ratings(nu, ni, n, seed=9)
    out = {}
    for S in (1, 2):
        cfg = SGDConfig(rank=128, epochs=5, test_every=0, num_slices=S, chunk=0, lr=0.005)
        m = SGDCollectiveMapper(Communicator(None, cuda), cfg, nu, ni, (u, i, v), None)
        m.init_model(KeyValReader([]))
        trained = sum(m.train_epoch(ep) for ep in range(cfg.epochs))
        m.rot.wait_all()
        torch.cuda.synchronize()
        out[S] = (trained, m._eval_ring(cfg.epochs - 1)[0])
    assert out[1][0] == out[2][0] == 5 * n
    assert abs(out[1][1] - out[2][1]) / out[2][1] < 0.01, out



@pytest.mark.parametrize("atomic", [1, 2, 3, 5])
@pytest.mark.parametrize("r", [16, 32, 48, 128])
def test_sgd_xcd_atomic_writeback_one_stream_matches_plain(cuda, r, atomic):
    """One stream per cell (no concurrency): the atomic write-back modes (W adds, H adds, hot
    H adds for flagged items) must train exactly what the plain stores train."""
    R, C, V, off, W0, H0 = _cells(64, 48, 4000, r, 2)
    out = {}
    for a in (0, atomic):
        Cf = C.clone()
        if a & MF.ATOMIC_HOT:  # every other item hot
            Cf = torch.where(Cf % 2 == 0, Cf | MF.HOT_BIT, Cf).int()
        Wg, Hg = W0.clone().to(cuda), H0.clone().to(cuda)
        MF.sgd_update_blocked(R.to(cuda), Cf.to(cuda), V.to(cuda), off.to(cuda), Wg, Hg, 0.01, 0.05, chunk=128,
                              blocks_per_xcd=1, atomic=a)
        torch.cuda.synchronize()
        out[a] = (Wg.cpu(), Hg.cpu())
    assert torch.isfinite(out[atomic][0]).all() and torch.isfinite(out[atomic][1]).all()
    assert torch.allclose(out[atomic][0], out[0][0], atol=1e-5) and torch.allclose(out[atomic][1], out[0][1], atol=1e-5)
