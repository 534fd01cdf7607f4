"""Per-iteration metrics and the bench.py driver contract.

* K-means / SGD / LDA on 2 gloo ranks write one JSONL record per iteration with phase
  times, collective bytes (non-zero: the reference never logged bytes moved), achieved
  GB/s and the xGMI-model efficiency (reference timing hooks:
  KMeansCollectiveMapper.java:191-193, SGDCollectiveMapper.java:294-298,
  RegroupCollective.java:274-295).
* ``bench.py --gpus 2`` without a torchrun environment spawns its 2 ranks itself and
  reports ``n_gpus: 2`` (KMeansLauncher.java:97-137 launches the multi-worker job)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from harp_amd.models.kmeans import KMeansConfig, KMeansCollectiveMapper
from harp_amd.runtime.launcher import launch
from harp_amd.runtime.mapper import KeyValReader
from harp_amd.utils.metrics import Metrics, ideal_collective_s, ring_allreduce_ideal_s, table_nbytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _km_job(comm, strategy, path):
    m = KMeansCollectiveMapper(comm, KMeansConfig(num_points=400, num_centroids=16, dim=8, iterations=3,
                                                  strategy=strategy),
                               metrics=Metrics(rank=comm.rank, path=f"{path}.{comm.rank}"))
    m.run(KeyValReader([]))
    return m.metrics.summary()["collectives"]


def _read(path):
    with open(path) as f:
        return [json.loads(line) for line in f]


@pytest.mark.parametrize("strategy", ["allreduce", "regroup_allgather", "bcast_reduce", "push_pull", "rotation"])
def test_kmeans_jsonl_records(tmp_path, strategy):
    path = str(tmp_path / "m.jsonl")
    summ = launch(_km_job, 2, args=(strategy, path), timeout=300)
    for r in range(2):
        recs = _read(f"{path}.{r}")
        its = [x for x in recs if x["event"] == "iteration"]
        assert [x["iter"] for x in its] == [0, 1, 2]
        for x in its:
            assert x["app"] == "kmeans" and x["world"] == 2 and x["rank"] == r
            assert x["collective_bytes"] > 0, x
            assert x["phases_ms"]["compute"] > 0
            assert x["compute_tflops"] > 0 and 0 < x["mfma_peak_frac"] < 1  # 2 n K d over the compute phase
            assert all(c["bytes"] >= 0 and c["ms"] >= 0 for c in x["collectives"])
            if strategy != "rotation":
                assert any("eff_vs_xgmi_model" in c for c in x["collectives"]), x
        assert sum(v["bytes"] for v in summ[r].values()) > 0


def test_allreduce_bytes_match_table(tmp_path):
    path = str(tmp_path / "a.jsonl")
    launch(_km_job, 2, args=("allreduce", path), timeout=300)
    rec = _read(f"{path}.0")[0]
    ar = [c for c in rec["collectives"] if c["kind"] == "allreduce"]
    assert len(ar) == 1
    kp, dp = 128, 16  # padded centroids x padded dim (fp32 partial sums)
    assert ar[0]["bytes"] == kp * dp * 4
    assert ar[0]["ideal_ms"] == pytest.approx(ring_allreduce_ideal_s(kp * dp * 4, 2) * 1e3, rel=1e-3)


def test_ideal_model_and_nbytes():
    from harp_amd.core.combiner import ArrCombiner, Operation
    from harp_amd.core.table import PackedTable, Table

    t = PackedTable(list(range(4)), torch.zeros(4, 10), combiner=ArrCombiner(Operation.SUM))
    assert table_nbytes(t) == 160
    g = Table(1, ArrCombiner(Operation.SUM))
    g.add(3, torch.zeros(5, dtype=torch.float64))
    g.add(7, torch.zeros(2, dtype=torch.int32))
    assert table_nbytes(g) == 48
    assert ideal_collective_s("allreduce", 0, 8) == 0.0
    assert ideal_collective_s("allgather", 153_000_000, 2) == pytest.approx(0.5e-3)
    assert ideal_collective_s("rotate", 153_000_000, 4) == pytest.approx(1e-3)
    assert ideal_collective_s("allreduce", 10, 1) == 0.0


def _sgd_job(comm, path):
    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings

    tr = synthetic_ratings(300, 80, 4000, seed=2)
    m = SGDCollectiveMapper(comm, SGDConfig(rank=8, epochs=2, test_every=0, xcd_blocks=False), 300, 80, tr,
                            metrics=Metrics(rank=comm.rank, path=f"{path}.{comm.rank}"))
    m.run(KeyValReader([]))
    return True


def test_sgd_jsonl_rotation_bytes(tmp_path):
    path = str(tmp_path / "s.jsonl")
    launch(_sgd_job, 2, args=(path,), timeout=300)
    recs = _read(f"{path}.0")
    assert [x["iter"] for x in recs] == [0, 1]
    for x in recs:
        rot = [c for c in x["collectives"] if c["kind"] == "rotate_wait"]
        assert rot and all(c["bytes"] > 0 for c in rot)
        assert x["trained"] > 0 and x["updates_per_s"] > 0


def _run_bench(args, env=None, rc=0):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=600, env=e, cwd=ROOT)
    assert r.returncode == rc, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_self_spawns_ranks():
    rec = _run_bench(["--gpus", "2", "--points", "2e4", "--centroids", "128", "--backend", "gloo", "--steps", "2",
                      "--warmup", "1"])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["steps"] == 2 and rec["warmup"] == 1 and rec["value"] > 0
    assert rec["sync_bytes_per_iter"] > 0
    assert "sgd" not in rec  # auto: CPU ranks skip the SGD record


def test_bench_rccl_preflight_three_ranks():
    """The self-diagnosing pre-flight at P=3 over gloo: world size seen by
    every rank, per-rank device records, a passing collective battery, a 64 MB all-reduce
    bus bandwidth and one ring send/recv per rotation channel (distinct strides at P=3)."""
    rec = _run_bench(["--gpus", "3", "--points", "3e4", "--centroids", "128", "--backend", "gloo", "--steps", "2",
                      "--warmup", "1"])
    r = rec["rccl"]
    assert r["world"] == 3 and r["world_seen"] == [3, 3, 3] and r["backend"] == "gloo"
    assert [x["rank"] for x in r["ranks"]] == [0, 1, 2]
    assert r["distinct_devices"] is False  # CPU ranks share no device
    assert set(r["battery"]) == {"all_gather_ints", "all_reduce", "broadcast", "all_gather", "reduce_scatter",
                                 "all_to_all", "ring_sendrecv", "barrier", "all_reduce_64MB"}
    assert r["battery_ok"], r["battery"]
    assert r["all_reduce_64MB"]["busbw_GBps"] > 0 and r["all_reduce_64MB"]["ms"] > 0
    ch = r["rotation_channels"]
    assert [c["channel"] for c in ch] == ["sgd-h-0", "sgd-h-1"] and [c["stride"] for c in ch] == [1, 2]
    assert all(c["ok"] and c["GBps"] > 0 for c in ch), ch


def test_bench_single_rank_with_sgd_record():
    rec = _run_bench(["--gpus", "1", "--points", "1e4", "--centroids", "128", "--steps", "2", "--warmup", "1",
                      "--sgd", "on", "--sgd-users", "2000", "--sgd-items", "300", "--sgd-ratings", "20000",
                      "--sgd-rank", "16", "--sgd-epochs", "2"])
    assert rec["n_gpus"] == 1 and rec["metric"].startswith("sec/iteration K-means")
    s = rec["sgd"]
    assert s["updates_per_sec"] > 0 and s["epochs"] == 2 and 0 < s["train_rmse"] < 2
    assert rec["rccl"]["world"] == 1 and "battery" not in rec["rccl"]


def test_bench_sgd_guard_keeps_headline_line():
    """A nested MF-SGD record that exceeds --sgd-timeout (a hung rotation peer on a real
    node) still yields exactly one JSON line: the measured K-means record with sgd.error,
    and the run exits non-zero (124) so the hang is never reported as a clean run."""
    rec = _run_bench(["--gpus", "2", "--points", "2e4", "--centroids", "128", "--backend", "gloo", "--steps", "2",
                      "--warmup", "1", "--sgd", "on", "--sgd-users", "2000", "--sgd-items", "300",
                      "--sgd-ratings", "20000", "--sgd-rank", "16", "--sgd-timeout", "0.01"], rc=124)
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    assert "timeout" in rec["sgd"]["error"]


_TINY = ["--points", "3e4", "--centroids", "128", "--backend", "gloo", "--steps", "10", "--warmup", "1",
         "--sgd", "on", "--sgd-users", "3000", "--sgd-items", "400", "--sgd-ratings", "30000", "--sgd-rank", "16",
         "--sgd-epochs", "10", "--extras", "on", "--pca-n", "6000", "--pca-d", "24", "--pca-steps", "10",
         "--lda-docs", "600", "--lda-vocab", "900", "--lda-topics", "16", "--lda-len", "20", "--lda-iters", "10"]


def _check_full_record(rec, P, slices=1):
    assert rec["n_gpus"] == P and rec["config"]["parallelism"] == f"dp{P}"
    assert rec["steps"] == 10 and rec["value"] > 0 and rec["median_s_per_iter"] > 0
    assert rec["step_s"]["n"] == 10
    assert rec["sync_bytes_per_iter"] > 0
    for name in ("sgd", "pca", "lda"):
        sub = rec[name]
        assert "error" not in sub, (name, sub)
        assert sub["n_gpus"] == P, (name, sub)
        assert sub["sync_bytes_per_iter"] > 0, (name, sub)
    s = rec["sgd"]
    assert s["updates_per_sec"] > 0 and s["epoch_s"]["n"] == 10 and 0 < s["train_rmse"] < 2
    assert s["slices_per_rank"] == slices
    assert 0 <= s["rotation_exposed_s_per_epoch"] <= s["s_per_epoch"]
    # ring mode: two slices rotate on different coprime strides (different xGMI links)
    if P > 2:
        assert len(set(s["rotation_strides"])) == slices
    p = rec["pca"]
    assert p["pass_s"]["n"] == 10 and p["max_eigenvalue"] > 0.9
    # step 2 includes eigenvectors (the reference's PCA result) through the library path
    assert p["eig_s"] is not None and p["eigvec_orth_err"] <= 1e-10 and p["eig_residual"] <= 1e-10
    lda = rec["lda"]
    assert lda["iter_s"]["n"] == 10 and lda["tokens_per_sec"] > 0 and lda["local_server"] is False
    # every nested record attributes its time per collective kind
    def kinds(sub, need):
        c = sub["collectives"]
        for k in need:
            assert k in c, (k, c)
            e = c[k]
            assert e["calls_per_iter"] > 0 and e["ms_per_iter"] >= 0 and e["bytes_per_iter"] >= 0, (k, e)
            if e["bytes_per_iter"] > 0:  # (rotate_wait is the exposed part of a transfer: no ideal)
                assert "gbps" in e and (k == "rotate_wait" or "ideal_ms_per_iter" in e), (k, e)
        return c
    kinds(lda, ("pull", "push", "allreduce"))
    assert lda["collectives"]["allreduce"]["calls_per_iter"] == 1.0
    pc = kinds(p, ("allreduce", "broadcast"))
    assert pc["allreduce"]["calls_per_iter"] == 1.0 and pc["broadcast"]["calls_per_iter"] == 1.0
    kinds(s, ("rotate_wait",))
    assert "allreduce" in rec["collectives"]


@pytest.mark.slow
def test_bench_full_records_three_ranks():
    """Every nested record (K-means, MF-SGD rotation of two slices per rank on ring strides,
    overlapped with compute, PCA, LDA push-pull with the server table remote) runs to
    completion at P=3 over gloo."""
    _check_full_record(_run_bench(["--gpus", "3", "--sgd-slices", "2"] + _TINY), 3, slices=2)


@pytest.mark.slow
def test_bench_full_records_eight_ranks():
    """Same at the 8-GPU node's world size (8 gloo ranks on the CPU), with the bench's
    default one slice per rank."""
    _check_full_record(_run_bench(["--gpus", "8"] + _TINY), 8, slices=2)  # auto: 2 slices at P > 1


def test_bench_single_rank_lda_records_collective_cost():
    """At P=1 the push-pull headline runs the pull / delta / push passes (never the
    aliased local server, which is only a nested extra on GPUs)."""
    rec = _run_bench(["--gpus", "1", "--points", "1e4", "--centroids", "128", "--steps", "2", "--warmup", "1",
                      "--sgd", "off", "--extras", "on", "--pca-n", "3000", "--pca-d", "16", "--pca-steps", "2",
                      "--lda-docs", "300", "--lda-vocab", "500", "--lda-topics", "16", "--lda-len", "20",
                      "--lda-iters", "2"])
    lda = rec["lda"]
    assert "error" not in lda and lda["tokens_per_sec"] > 0
    assert lda["comm_mode"] != "local" and lda["sync_bytes_per_iter"] >= 0
    assert lda["local_server"] is False and "local_server_alias" not in lda  # CPU: no nested alias run
    assert rec["pca"]["syrk_tflops"] is not None and rec["pca"]["n_gpus"] == 1


class _FakeEvent:
    def __init__(self, done=True):
        self.done = done

    def query(self):
        return self.done

    def elapsed_time(self, other):
        return 2.0  # ms


def test_pending_events_stay_bounded_without_metrics_path(monkeypatch):
    """Without a metrics path nothing flushes; completed event pairs must still be folded
    in as they accumulate (unbounded _pending)."""
    import harp_amd.utils.metrics as M

    m = Metrics()
    for i in range(5 * M.PENDING_SWEEP):
        m.collective("allreduce", "c", f"op{i}", 0.0, 8, events=(_FakeEvent(), _FakeEvent()))
    assert len(m._pending) < M.PENDING_SWEEP
    assert m.collectives[0]["s"] == pytest.approx(2e-3)
    # pairs still in flight are kept (in order) until the hard cap forces one sync
    synced = []
    monkeypatch.setattr(M.torch.cuda, "synchronize", lambda: synced.append(1))
    m2 = Metrics()
    for i in range(M.PENDING_HARD_CAP + 1):
        m2.collective("allreduce", "c", f"op{i}", 0.0, 8, events=(_FakeEvent(False), _FakeEvent(False)))
    assert synced and len(m2._pending) < M.PENDING_HARD_CAP
    t = M.PhaseTimer(use_events=False)
    for i in range(3 * M.PENDING_SWEEP):
        t._pending.append(("compute", _FakeEvent(), _FakeEvent()))
        M._sweep_pending(t._pending, t._fold)
    assert len(t._pending) < M.PENDING_SWEEP and t.counts["compute"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu_all_records(cuda):
    """Every nested record at P = 2 with both ranks' kernels on the GPU (gloo with host
    staging: RCCL refuses two ranks per device): the multi-rank device paths (rotation
    rings, sparse push / pull rows, PCA broadcast) run before an 8-GPU node sees them."""
    rec = _run_bench(["--gpus", "2", "--backend", "gloo", "--points", "2e5", "--centroids", "256", "--steps", "3",
                      "--warmup", "1", "--sgd", "on", "--sgd-users", "20000", "--sgd-items", "3000",
                      "--sgd-ratings", "400000", "--sgd-epochs", "3", "--extras", "on", "--pca-n", "2e5",
                      "--pca-d", "200", "--pca-steps", "3", "--lda-docs", "5000", "--lda-vocab", "8000",
                      "--lda-topics", "256", "--lda-len", "40", "--lda-iters", "3"])
    assert rec["n_gpus"] == 2 and rec["dtype"] == "bf16"
    for name in ("sgd", "pca", "lda"):
        assert "error" not in rec[name], (name, rec[name])
        assert rec[name]["n_gpus"] == 2 and rec[name]["sync_bytes_per_iter"] > 0
