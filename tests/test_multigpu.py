"""Multi-GPU RCCL tests: self-activate when >= 2 HIP devices are visible (skip otherwise).

One process per GPU (``launch(..., backend="nccl")``), P = 2, 3 (odd) and
min(device_count, 8). Covers what the gloo tests cannot: device tensors through RCCL, a
``dist.new_group`` per rotation channel whose first op is a grouped send/recv, the
device-side stream wait of ``DeviceRotator.get``, K-means / MF-SGD P-invariance on the
GPU path, the RCCL watchdog turning a hung peer into a failed collective + gang restart,
and ``bench.py --gpus P`` spawning its own RCCL ranks.

Reference concurrency contract: ml/java/.../dymoro/Rotator.java:43-71 (one rotation
thread per slice = one communicator per slice here)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from harp_amd.runtime.launcher import launch

pytestmark = pytest.mark.gpu

NGPU = torch.cuda.device_count() if torch.cuda.is_available() else 0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P_LIST = sorted({p for p in (2, 3, min(NGPU, 8)) if 2 <= p <= NGPU}) or [2]
need2 = pytest.mark.skipif(NGPU < 2, reason=f"needs >= 2 GPUs ({NGPU} visible)")


def _battery(comm):
    from tests.mp_checks import collective_battery

    assert comm.backend == "nccl" and comm.device.type == "cuda"
    return collective_battery(comm)


@need2
@pytest.mark.parametrize("P", P_LIST)
def test_collective_battery_over_rccl(P):
    res = launch(_battery, P, backend="nccl", timeout=300)
    for r, checks in enumerate(res):
        bad = {k: v for k, v in checks.items() if v is not True}
        assert not bad, f"rank {r}: {bad}"


def _rotator(comm, rounds):
    from harp_amd.runtime.dymoro import DeviceRotator

    P, me = comm.world_size, comm.rank
    slabs = [torch.full((1000, 64), float(me * 10 + k), device=comm.device) for k in range(2)]
    rot = DeviceRotator(comm, slabs, name="t")
    ring = [(r + 1) % P for r in range(P)]
    seen = []
    for s in range(rounds):
        for k in range(2):
            x = rot.get(k)
            seen.append(float(x[0, 0]))
            x.add_(1000.0)  # compute on the resident slab before it moves on
            rot.start(k, ring)
    rot.wait_all()
    return seen, [float(rot.get(k)[5, 7]) for k in range(2)]


@need2
@pytest.mark.parametrize("P", P_LIST)
def test_device_rotator_ring_round_trip(P):
    res = launch(_rotator, P, args=(P,), backend="nccl", timeout=300)
    for me, (seen, final) in enumerate(res):
        for s in range(P):
            src = (me - s) % P  # slab resident at step s came from rank me - s
            for k in range(2):
                assert seen[2 * s + k] == src * 10 + k + 1000.0 * s
        # after P hops every slab is home, touched once by every rank
        assert final == [me * 10 + k + 1000.0 * P for k in range(2)]


def _kmeans(comm, strategy, x, c0):
    from harp_amd.models.kmeans import KMeansConfig, run_kmeans

    P, r = comm.world_size, comm.rank
    n = x.shape[0]
    cfg = KMeansConfig(num_points=n // P, num_centroids=c0.shape[0], dim=x.shape[1], iterations=3, strategy=strategy)
    return run_kmeans(comm, cfg, points=x[r * n // P:(r + 1) * n // P], init_centroids=c0)


@need2
@pytest.mark.parametrize("strategy", ["allreduce", "regroup_allgather", "bcast_reduce", "push_pull", "rotation"])
def test_kmeans_strategies_match_one_rank(strategy):
    P = P_LIST[-1]
    g = torch.Generator().manual_seed(3)
    x = torch.rand((P * 4096, 32), generator=g) * 100
    c0 = x[:300].clone()
    one = launch(_kmeans, 1, args=("allreduce", x, c0), backend="nccl", timeout=300)[0]
    res = launch(_kmeans, P, args=(strategy, x, c0), backend="nccl", timeout=300)
    assert res[0]["objective"] == pytest.approx(one["objective"], rel=2e-4)
    assert torch.allclose(res[0]["centroids"], one["centroids"], rtol=1e-3, atol=0.05)


def _sgd(comm, tr):
    from harp_amd.models.sgd_mf import SGDConfig, SGDCollectiveMapper
    from harp_amd.runtime.mapper import KeyValReader

    m = SGDCollectiveMapper(comm, SGDConfig(rank=32, epochs=4, test_every=2), 5000, 900, tr, None)
    m.run(KeyValReader([]))
    return m.rmse_history, m.trained


@need2
@pytest.mark.parametrize("P", P_LIST)
def test_sgd_rotation_trained_count_and_rmse(P):
    from harp_amd.models.sgd_mf import synthetic_ratings

    tr = synthetic_ratings(5000, 900, 200_000, seed=1)
    one = launch(_sgd, 1, args=(tr,), backend="nccl", timeout=300)[0]
    res = launch(_sgd, P, args=(tr,), backend="nccl", timeout=300)
    assert sum(t for _, t in res) == one[1] == 4 * 200_000
    rm_p, rm_1 = res[0][0][-1][1], one[0][-1][1]
    assert rm_p == pytest.approx(rm_1, rel=0.05)  # Hogwild order differs; the fit must not
    assert rm_p < res[0][0][0][1]


def _hang_then_resume(comm, d):
    from harp_amd.models.kmeans import KMeansConfig, run_kmeans

    g = torch.Generator().manual_seed(5)
    x = torch.rand((4096, 16), generator=g)
    P, r = comm.world_size, comm.rank
    cfg = KMeansConfig(num_points=4096 // P, num_centroids=64, dim=16, iterations=6, strategy="allreduce",
                       checkpoint_dir=str(d), checkpoint_every=1)
    return run_kmeans(comm, cfg, points=x[r * 4096 // P:(r + 1) * 4096 // P], init_centroids=x[:64].clone())


@need2
def test_rccl_watchdog_fails_the_gang_and_restart_resumes(tmp_path):
    """A rank stuck past HARP_DATA_MAX_WAIT_TIME: the survivors' RCCL collective times out
    (torch's NCCL watchdog aborts the communicator), the gang is stopped, and the job is
    restarted in FRESH processes that resume from the last checkpoint."""
    env = {"HARP_FAULT": "rank=1,iter=2,kind=hang,seconds=90", "HARP_DATA_MAX_WAIT_TIME": "10",
           "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1"}
    res = launch(_hang_then_resume, 2, args=(tmp_path,), backend="nccl", timeout=240, retries=1, env=env, grace_s=5)
    assert res[0]["start_iteration"] == 2
    ref = launch(_hang_then_resume, 2, args=(tmp_path / "ref",), backend="nccl", timeout=240)
    assert torch.allclose(res[0]["centroids"], ref[0]["centroids"], atol=1e-5)


@need2
def test_bench_spawns_rccl_ranks():
    P = P_LIST[-1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(P), "--points", "4e6",
                        "--steps", "3", "--warmup", "1", "--sgd-ratings", "4000000", "--sgd-epochs", "2"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == P and rec["config"]["parallelism"] == f"dp{P}"
    assert rec["collectives"]["allreduce"]["bytes"] > 0
    assert rec["sgd"]["updates_per_sec"] > 0


def _lda_rccl(comm, mode):
    from harp_amd.models.lda import LDACollectiveMapper, LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.runtime.mapper import KeyValReader

    push_pull = mode == "push_pull"
    doc, word = synthetic_corpus(400, 900, 8, 60, seed=11)
    # rotation_codec: the word-slice slabs cross RCCL as sparse payloads (ops/slabcodec)
    cfg = LDAConfig(num_topics=32, iterations=4, print_interval=4, block_words=128,
                    rotate_codec="on" if mode == "rotation_codec" else "off")
    cls = LDAPushPullMapper if push_pull else LDACollectiveMapper
    m = cls(comm, cfg, 400, 900, (doc, word))
    m.run(KeyValReader([]))
    return {"nk": m.nk.cpu(), "tokens": int(m.tz.numel()), "loglik": m.loglik[-1][1], "total": int(doc.numel())}


@need2
@pytest.mark.parametrize("mode", ["rotation", "rotation_codec", "push_pull"])
def test_lda_over_rccl_conserves_counts_and_learns(mode):
    """LDA-CGS on device tensors over RCCL (word-slice rotation or the push-pull PS table):
    every token sampled by exactly one rank, topic sums identical on every rank and equal to
    the token count, and the likelihood within a few % of the 1-rank run."""
    P = P_LIST[-1]
    one = launch(_lda_rccl, 1, args=(mode,), backend="nccl", timeout=300)[0]
    res = launch(_lda_rccl, P, args=(mode,), backend="nccl", timeout=300)
    assert sum(r["tokens"] for r in res) == one["total"]
    for r in res:
        assert torch.equal(r["nk"], res[0]["nk"]) and int(r["nk"].sum()) == one["total"]
    # push-pull samples every rank against one snapshot per sweep (bulk-synchronous
    # staleness): on this small corpus it trails one rank by ~5 % after 4 sweeps (gloo
    # rehearsal at P = 2); rotation by < 1 %
    assert res[0]["loglik"] == pytest.approx(one["loglik"], rel=0.15 if mode == "push_pull" else 0.05)  # P up to 8


def _ccd_rccl(comm, mode):
    from harp_amd.models.ccd import CCDConfig, train_ccd

    g = torch.Generator().manual_seed(5)
    u = torch.randint(0, 300, (30_000,), generator=g)
    i = torch.randint(0, 120, (30_000,), generator=g)
    v = torch.rand(30_000, generator=g) * 4 + 1
    P, r = comm.world_size, comm.rank
    sl = slice(r * u.numel() // P, (r + 1) * u.numel() // P)
    res = train_ccd(comm, u[sl], i[sl], v[sl], 300, 120, CCDConfig(rank=8, iterations=4, mode=mode))
    return res["history"][-1]["train_rmse"]


@need2
@pytest.mark.parametrize("mode", ["allgather", "rotation"])
def test_ccd_over_rccl_matches_one_rank(mode):
    P = P_LIST[-1]
    one = launch(_ccd_rccl, 1, args=(mode,), backend="nccl", timeout=300)[0]
    res = launch(_ccd_rccl, P, args=(mode,), backend="nccl", timeout=300)
    assert all(abs(r - res[0]) < 1e-6 for r in res)  # one allreduced RMSE
    # allgather mode is P-invariant; rotation visits the dimension slices in ring order,
    # so its trajectory differs from one rank's (gloo rehearsal: 1.1662 vs 1.1386 at P = 2)
    assert res[0] == pytest.approx(one, rel=1e-3 if mode == "allgather" else 0.06)


def _plans_rccl(comm):
    from tests.test_plans import _job, _sparse_job, _sparse_pull_job

    return _job(comm, "SUM", 2), _sparse_job(comm, True), _sparse_job(comm, False), _sparse_pull_job(comm, True), \
        _sparse_pull_job(comm, False)


@need2
def test_planned_push_pull_over_rccl():
    """Dense and sparse planned push / pull on device tables through RCCL all-to-all-v and
    all-gather agree with each other (the CPU tests pin them to the generic path)."""
    import harp_amd  # noqa: F401

    res = launch(_plans_rccl, P_LIST[-1], backend="nccl", timeout=300)
    for dense_sparse in res:
        out, sp_push, dn_push, sp_pull, dn_pull = dense_sparse
        (pd, ld), (pg, lg) = out[True], out[False]
        assert sorted(pd) == sorted(pg) and all(torch.allclose(pd[i].cpu(), pg[i].cpu()) for i in pd)
        assert all(torch.equal(sp_push[i].cpu(), dn_push[i].cpu()) for i in dn_push)
        for x, y in zip(sp_pull, dn_pull):
            assert all(torch.equal(x[i].cpu(), y[i].cpu()) for i in y)


def _pca_rccl(comm, n_per, d):
    from harp_amd.models import stats as ST
    from harp_amd.utils.metrics import Metrics

    P, r = comm.world_size, comm.rank
    blocks = [torch.rand((n_per, d), generator=torch.Generator().manual_seed(100 + q)) for q in range(P if P > 1 else 3)]
    X = (blocks[r] if P > 1 else torch.cat(blocks)).to(comm.device)
    met = Metrics(rank=r, world=P)
    res = ST.pca(X, comm, dtype="bf16", metrics=met)
    kinds = sorted({c["kind"] for c in met.collectives})
    return res["eigenvalues"].cpu(), res["eigenvectors"].cpu(), kinds


@pytest.mark.skipif(NGPU < 3, reason=f"needs >= 3 GPUs ({NGPU} visible)")
def test_pca_over_rccl_all_ranks_hold_the_same_eigenpairs():
    """stats.pca over RCCL: the MFMA SYRK partials allreduced, step 2 on the
    master, its eigenvalues + eigenvectors broadcast -- every rank holds bit-identical
    eigenpairs, equal to one rank's PCA of the concatenated rows (bf16 operands, fp32
    accumulation: summation-order differences only), and both collectives are recorded."""
    d, n_per = 200, 20000
    one = launch(_pca_rccl, 1, args=(n_per, d), backend="nccl", timeout=300)[0]
    res = launch(_pca_rccl, 3, args=(n_per, d), backend="nccl", timeout=300)
    for lam, V, kinds in res:
        assert torch.equal(lam, res[0][0]) and torch.equal(V, res[0][1])
        assert kinds == ["allreduce", "broadcast"]
        assert float((V @ V.t() - torch.eye(d, dtype=V.dtype)).abs().max()) < 1e-12
    assert float((res[0][0] - one[0]).abs().max()) < 1e-5


def _lda_fused_rccl(comm, fused):
    from harp_amd.models.lda import LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.runtime.mapper import KeyValReader

    toks = synthetic_corpus(3000, 2500, 20, 40, seed=13)
    cfg = LDAConfig(num_topics=256, alpha=0.1, beta=0.01, iterations=4, print_interval=4, block_words=256,
                    sparse_comm="on", local_server=False, seed=3, deterministic=True, fused_rows=fused)
    m = LDAPushPullMapper(comm, cfg, 3000, 2500, toks)
    m.run(KeyValReader([]))
    return {"tz": m.tz.cpu(), "ok": m.check_counts(), "fused": m.result["fused_rows"], "nk": m.nk.cpu(),
            "dedup": m.ps is not None and m.ps._dedup is not None}


@pytest.mark.skipif(NGPU < 3, reason=f"needs >= 3 GPUs ({NGPU} visible)")
def test_lda_fused_sparse_ps_over_rccl_three_ranks():
    """LDA push-pull with fused parameter-server rows over RCCL at P = 3: rows
    wanted by several ranks are encoded once and fanned out by copy_slots; in the
    deterministic sampler the fused run takes exactly the unfused run's trajectory, counts
    stay exact, and every rank holds the same topic sums."""
    a = launch(_lda_fused_rccl, 3, args=(True,), backend="nccl", timeout=300)
    b = launch(_lda_fused_rccl, 3, args=(False,), backend="nccl", timeout=300)
    assert any(r["dedup"] for r in a), "no owner-side dedup (copy_slots) exercised"
    for ra, rb in zip(a, b):
        assert ra["fused"] and not rb["fused"]
        assert ra["ok"] and rb["ok"]
        assert torch.equal(ra["tz"], rb["tz"])
        assert torch.equal(ra["nk"], a[0]["nk"])
