#!/usr/bin/env python3
"""Headline benchmark: K-means sec/iteration (N=1e8, d=100, K=1e4, bf16 MFMA) plus the
MF-SGD updates/sec record (Netflix shape, rank 128, model rotation) — BASELINE.json's
metric "sec/iteration K-means (N=1e8, d=100, K=1e4) at 1/2/4/8 MI355X; SGD-MF updates/sec".

K-means: the problem size is FIXED (N = 1e8 total points split evenly over the ranks), so
this is strong scaling; ``value`` is the whole-job seconds per Lloyd iteration (max over
ranks), lower is better. One timed step = one full iteration of the reference's loop
(ml/java/.../kmeans/regroupallgather/KMeansCollectiveMapper.java:147-197, timing printed at
:191-193): fused MFMA assign + accumulate over all local points, the RCCL model sync of
the 1e4 x 112 fp32 partial sums (``--strategy``: allreduce, or the reference's headline
regroup -> average at owner -> allgather), normalize, centroid operand prepare.

Nested ``pca`` / ``lda`` records (on GPUs; ``--extras off`` skips them): BASELINE configs 4
and 5 -- one PCA correlation pass over N = 1e8 x d = 1000 (MFMA SYRK partial result +
allreduce + fp64 eig) and LDA-CGS over 1M docs x 1M vocab x 1000 topics with the push-pull
collective, each split over the ranks and bounded by ``--extras-timeout``.

MF-SGD (nested ``sgd`` record): 480,189 x 17,770, 100,480,507 synthetic ratings, rank
128, H split into ``--sgd-slices`` slices per rank (default: 1 on one GPU, 2 at P > 1) that rotate around the ring
(model rotation); epochs timed after warmup; updates/sec = ratings trained / epoch time
(SGDCollectiveMapper.java:294-298).

Every record reports the mean (wall clock around the timed loop, max over ranks) and the
median / min / max of per-step times (HIP events at step boundaries, each step's max over
ranks) -- BASELINE.md's protocol; nested records time >= 10 iterations by default. A nested
record that hangs past its guard leaves the headline line printed and exits 124.

Usage:
  python bench.py [--gpus N] [--steps K] [--warmup W]
  With N > 1 and no torchrun environment, the parent process spawns the N ranks itself
  (before anything touches the GPU); under ``torch.distributed.run`` the ranks come from
  RANK / LOCAL_RANK / WORLD_SIZE.
Data: synthetic U[0,1000) points generated on the device, random-init centroids; synthetic
Netflix-shaped ratings (no datasets are available offline).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sec/iteration K-means (N=1e8, d=100, K=1e4)"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--points", type=float, default=1e8, help="total points (strong scaling)")
    ap.add_argument("--centroids", type=int, default=10000)
    ap.add_argument("--dim", type=int, default=100)
    ap.add_argument("--strategy", default="allreduce")
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--backend", default=None, help="override (e.g. gloo to rehearse >1 rank on the CPU)")
    ap.add_argument("--graph", action="store_true", help="replay each iteration's kernels from HIP graphs")
    ap.add_argument("--sgd", choices=("auto", "on", "off"), default="auto",
                    help="nested MF-SGD record (auto: on when the ranks run on GPUs)")
    ap.add_argument("--sgd-users", type=int, default=480189)
    ap.add_argument("--sgd-items", type=int, default=17770)
    ap.add_argument("--sgd-ratings", type=int, default=100480507)
    ap.add_argument("--sgd-rank", type=int, default=128)
    ap.add_argument("--sgd-epochs", type=int, default=10)
    ap.add_argument("--sgd-warmup", type=int, default=1)
    ap.add_argument("--sgd-slices", type=int, default=0,
                    help="H slices per rank (rotation pipeline depth); 0 = auto: 1 on one GPU (nothing rotates; "
                         "each slice step then trains twice the cells in half the launches, 6.3 vs 7.6 ms per "
                         "100M-rating epoch, profiles/r3_sgd_slices), 2 at P > 1 so every slice's transfer to "
                         "the ring neighbour overlaps the other slice's compute (the reference's numModelSlices "
                         "default, MJ/dymoro/Rotator.java:30-86)")
    ap.add_argument("--sgd-atomic", type=int, default=-1,
                    help="atomic write-back of the blocked SGD kernel: 0 none, 1 W, 2 H, 3 both; -1 = SGDConfig "
                         "default")
    ap.add_argument("--sgd-timeout", type=float, default=240.0,
                    help="wall-clock bound (s) on the nested MF-SGD record; past it rank 0 prints the "
                         "K-means line with an sgd error and every rank exits")
    ap.add_argument("--extras", choices=("auto", "on", "off"), default="auto",
                    help="nested PCA (BASELINE config 4) and LDA (config 5) records (auto: on GPUs)")
    ap.add_argument("--pca-n", type=float, default=1e8)
    ap.add_argument("--pca-d", type=int, default=1000)
    ap.add_argument("--pca-steps", type=int, default=10)
    ap.add_argument("--lda-docs", type=float, default=1e6)
    ap.add_argument("--lda-vocab", type=float, default=1e6)
    ap.add_argument("--lda-topics", type=int, default=1000)
    ap.add_argument("--lda-len", type=int, default=100)
    ap.add_argument("--lda-iters", type=int, default=10)
    ap.add_argument("--lda-strategy", choices=("push_pull", "rotation"), default="push_pull")
    ap.add_argument("--lda-local-server", choices=("auto", "off"), default="auto",
                    help="push-pull at P=1: the headline always runs the pull / delta / push passes; auto also "
                         "records (nested, local_server_alias) the shortcut where the server table aliases the "
                         "sampled slab")
    ap.add_argument("--extras-timeout", type=float, default=180.0, help="wall-clock bound (s) per nested record")
    ap.add_argument("--metrics-jsonl", default="", help="per-iteration phase/bytes records (JSONL)")
    ap.add_argument("--preflight-timeout", type=float, default=120.0,
                    help="wall-clock bound (s) on the RCCL pre-flight (world / devices / battery / bandwidth)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- spawning
def spawn(args, argv) -> int:
    """Start ``args.gpus`` rank processes of this script (torchrun environment contract)
    and return the worst exit code. The parent never initialises the GPU."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HARP_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:  # a failed gang: stop the rest
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc


# ----------------------------------------------------------------------------- RCCL pre-flight
PREFLIGHT_BYTES = 64 << 20


def _now(comm, torch) -> float:
    if comm.device.type == "cuda":
        torch.cuda.synchronize()
    return time.perf_counter()


def rccl_preflight(args, comm, torch) -> dict:
    """A short self-diagnosis before any timed record (the reference's
    standalone collective harness, core/harp-collective/.../AllreduceCollective.java:53-138,
    and BenchmarkMapper.java:64-152): the world size every rank sees, every rank's device /
    PCI address (distinct on a real node), a mini battery of the collectives the records use
    (each checked against known values; a failure is reported here and never costs the
    headline), the bus bandwidth of a 64 MB all-reduce, and one ring send/recv per MF-SGD
    rotation channel (the same keyed channels the rotation then reuses) with its GB/s."""
    import torch.distributed as dist

    from harp_amd.runtime.dymoro import ring_strides

    P, me, dev = comm.world_size, comm.rank, comm.device
    ident = [me, -1, -1, -1, -1]
    name = "cpu"
    if dev.type == "cuda":
        pr = torch.cuda.get_device_properties(dev)
        ident = [me, dev.index, int(getattr(pr, "pci_domain_id", -1)), int(getattr(pr, "pci_bus_id", -1)),
                 int(getattr(pr, "pci_device_id", -1))]
        name = pr.name
    out = {"world": P, "backend": comm.backend, "device": {"index": ident[1], "name": name,
                                                          "pci": "%04x:%02x:%02x" % tuple(max(0, x) for x in ident[2:])}}
    if P == 1:
        return out
    battery = {}

    def item(key, fn):
        t0 = _now(comm, torch)
        try:
            ok = fn()
            battery[key] = {"ok": bool(ok), "ms": round((_now(comm, torch) - t0) * 1e3, 3)}
        except Exception as e:  # noqa: BLE001
            battery[key] = {"ok": False, "error": f"{type(e).__name__}: {e}"[:200]}

    seen = {}

    def world():
        g = comm.all_gather_ints([P] + ident)
        seen["rows"] = g.tolist()
        return all(r[0] == P for r in seen["rows"]) and [r[1] for r in seen["rows"]] == list(range(P))

    item("all_gather_ints", world)
    rows = seen.get("rows", [])
    out["world_seen"] = [r[0] for r in rows]
    out["ranks"] = [{"rank": r[1], "device": r[2], "pci": "%04x:%02x:%02x" % tuple(max(0, x) for x in r[3:])}
                    for r in rows]
    out["distinct_devices"] = len({(r[2], r[3], r[4], r[5]) for r in rows}) == P if rows else False
    f32 = dict(dtype=torch.float32, device=dev)

    def all_reduce():
        t = torch.full((1024,), float(me + 1), **f32)
        comm.all_reduce(t)
        return bool((t == P * (P + 1) / 2).all())

    def broadcast():
        t = torch.full((1024,), float(me), **f32)
        comm.broadcast(t, P - 1)
        return bool((t == P - 1).all())

    def all_gather():
        o = torch.empty(P * 4, **f32)
        comm.all_gather_into(o, torch.full((4,), float(me), **f32))
        return torch.equal(o.cpu(), torch.arange(P, dtype=torch.float32).repeat_interleave(4))

    def reduce_scatter():
        o = torch.empty(4, **f32)
        comm.reduce_scatter(o, torch.arange(P * 4, **f32))
        return torch.equal(o.cpu(), P * torch.arange(me * 4, me * 4 + 4, dtype=torch.float32))

    def all_to_all():
        inp = torch.tensor([me * 100 + j for j in range(P)], dtype=torch.int64, device=dev)
        o = torch.empty(P, dtype=torch.int64, device=dev)
        comm.all_to_all_single(o, inp)
        return o.cpu().tolist() == [j * 100 + me for j in range(P)]

    def ring():
        o = torch.empty(1024, **f32)
        comm.sendrecv({(me + 1) % P: torch.full((1024,), float(me), **f32)}, {(me - 1) % P: o})
        return bool((o == (me - 1) % P).all())

    for key, fn in (("all_reduce", all_reduce), ("broadcast", broadcast), ("all_gather", all_gather),
                    ("reduce_scatter", reduce_scatter), ("all_to_all", all_to_all), ("ring_sendrecv", ring),
                    ("barrier", lambda: comm.barrier() or True)):
        item(key, fn)
    out["battery"] = battery
    out["battery_ok"] = all(v["ok"] for v in battery.values())

    def busbw():
        t = torch.ones(PREFLIGHT_BYTES // 4, **f32)
        comm.all_reduce(t)  # warm-up (RCCL communicator / channel setup)
        reps = 5
        t0 = _now(comm, torch)
        for _ in range(reps):
            comm.all_reduce(t)
        dt = (_now(comm, torch) - t0) / reps
        # ring all-reduce moves 2 (P - 1) / P of the buffer over every link (nccl-tests busbw)
        seen["busbw"] = 2 * (P - 1) / P * PREFLIGHT_BYTES / dt / 1e9
        seen["ar_ms"] = dt * 1e3
        return True

    item("all_reduce_64MB", busbw)
    out["all_reduce_64MB"] = {"ms": round(seen.get("ar_ms", 0.0), 3), "busbw_GBps": round(seen.get("busbw", 0.0), 2)}
    S = args.sgd_slices or 2
    chans = []
    for k, st in enumerate(ring_strides(P, S)):
        rec = {"channel": f"sgd-h-{k}", "stride": st}
        try:
            ch = comm.channel(f"sgd-h-{k}")  # the DeviceRotator's channel key (models/sgd_mf.py)
            n = (16 << 20) // 4
            snd, rcv = torch.ones(n, **f32), torch.empty(n, **f32)
            ch.sendrecv({(me + st) % P: snd}, {(me - st) % P: rcv})
            t0 = _now(comm, torch)
            for _ in range(3):
                ch.sendrecv({(me + st) % P: snd}, {(me - st) % P: rcv})
            dt = (_now(comm, torch) - t0) / 3
            rec.update(ok=bool((rcv == 1).all()), MB=16, GBps=round((n * 4) / dt / 1e9, 2))
        except Exception as e:  # noqa: BLE001
            rec.update(ok=False, error=f"{type(e).__name__}: {e}"[:200])
        chans.append(rec)
    out["rotation_channels"] = chans
    return out


# ----------------------------------------------------------------------------- K-means
def bench_kmeans(args, comm, torch):
    from harp_amd.models.kmeans import KMeansCollectiveMapper, KMeansConfig
    from harp_amd.ops import kmeans as K
    from harp_amd.utils.metrics import Metrics

    P, rank = comm.world_size, comm.rank
    N = int(args.points)
    n_local = N // P + (1 if rank < N % P else 0)
    cfg = KMeansConfig(num_points=n_local, num_centroids=args.centroids, dim=args.dim, iterations=10**9,
                       strategy=args.strategy, objective_every=0,
                       variant=K.DEFAULT_VARIANT if args.variant is None else args.variant, graph=args.graph)
    metrics = Metrics(rank=rank, path=args.metrics_jsonl or None)
    m = KMeansCollectiveMapper(comm, cfg, metrics=metrics)
    m.init_model(_Reader())
    for it in range(args.warmup):
        m.step(it)
    sync(comm, torch)
    m.metrics.timer.reset()
    m.metrics.collectives.clear()
    clock = StepClock(comm, torch)
    t0 = time.perf_counter()
    clock.mark()
    for it in range(args.steps):
        m.step(args.warmup + it)
        clock.mark()
    sync(comm, torch)
    elapsed = time.perf_counter() - t0
    step_s = clock.durations()
    phases = m.metrics.timer.flush()
    coll = m.metrics.summary()["collectives"]
    elapsed = reduce_max(comm, torch, elapsed)
    sec_per_iter = elapsed / args.steps
    # objective after timing (one extra assign pass, outside the timed region) as a sanity value
    if args.strategy == "rotation":  # the model lives in rotating blocks: gather it first
        m.op = K.prepare(m._rotation_gather().contiguous(), m.dp)
    _, obj = K.assign(m.X, m.op, sums=None, want_objective=True, variant=cfg.variant)
    o = obj.reshape(1).to(comm.device, torch.float64)
    if P > 1:
        comm.all_reduce(o)
    flops = 2.0 * N * args.centroids * args.dim
    sync_bytes = sum(v["bytes"] for v in coll.values()) / max(args.steps, 1)
    rec = {
        "metric": METRIC,
        "value": round(sec_per_iter, 6),
        "unit": "s/iter",
        "n_gpus": P,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(sec_per_iter * 1e3, 3),
        "higher_is_better": False,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16" if comm.device.type == "cuda" else "fp32",
        "data": "synthetic U[0,1000) points generated on device; random-init centroids",
        "config": {"model": f"kmeans-{args.strategy}", "N": N, "d": args.dim, "K": args.centroids,
                   "global_batch": N, "seq_len": None, "parallelism": f"dp{P}"},
        "median_s_per_iter": round(step_stats(step_s)["median"], 6),
        "step_s": step_stats(step_s),
        "points_per_sec": round(N / sec_per_iter, 1),
        "effective_tflops": round(flops / sec_per_iter / 1e12, 1),
        "phase_ms_per_iter": {k: round(v / args.steps * 1e3, 3) for k, v in phases.items()},
        "sync_bytes_per_iter": int(sync_bytes),
        "collectives": {k: {"calls": v["calls"], "ms": round(v["s"] * 1e3, 3), "bytes": v["bytes"]}
                        for k, v in coll.items()},
        "mean_sq_dist": float(o.item()) / N,
        "kernel_variant": cfg.variant,
        "hip_graph": bool(args.graph),
    }
    del m
    return rec


def _coll_breakdown(metrics, iters: int, comm, torch) -> dict:
    """Per collective kind, per timed iteration: calls, stream milliseconds (HIP events; the
    MAX over ranks), bytes on this rank, achieved GB/s and the xGMI link model's ideal time
    (``utils.metrics.ideal_collective_s``), so a multi-GPU record says which collective cost
    what. Kinds: pull / push (all-to-all of parameter-server rows),
    allreduce, broadcast, rotate / rotate_wait (model rotation; rotate_wait = compute-stream
    time stalled on an arrival, i.e. the rotation NOT hidden)."""
    from harp_amd.utils.metrics import ideal_collective_s

    metrics.resolve()
    agg = {}
    for c in metrics.collectives:
        a = agg.setdefault(c["kind"], {"calls": 0, "s": 0.0, "bytes": 0, "ideal_s": 0.0})
        a["calls"] += 1
        a["s"] += c["s"]
        a["bytes"] += c["bytes"]
        a["ideal_s"] += ideal_collective_s(c["kind"], c["bytes"], comm.world_size)
    # one MAX-allreduce over a fixed kind list: every rank takes part whatever it recorded
    kinds = ("allgather", "allreduce", "broadcast", "join", "pull", "push", "reduce", "regroup", "rotate",
             "rotate_wait")
    v = torch.tensor([[agg.get(k, {}).get("calls", 0), agg.get(k, {}).get("s", 0.0)] for k in kinds],
                     dtype=torch.float64, device=comm.device)
    if comm.world_size > 1:
        import torch.distributed as dist

        comm.all_reduce(v, op=dist.ReduceOp.MAX)
    v = v.cpu().tolist()
    out = {}
    it = max(iters, 1)
    for kind, (calls_max, s_max) in zip(kinds, v):
        if calls_max <= 0:
            continue
        a = agg.get(kind, {"calls": 0, "s": 0.0, "bytes": 0, "ideal_s": 0.0})
        e = {"calls_per_iter": round(a["calls"] / it, 3), "ms_per_iter": round(s_max * 1e3 / it, 4),
             "bytes_per_iter": int(a["bytes"] / it)}
        if s_max > 0 and a["bytes"]:
            e["gbps"] = round(a["bytes"] / s_max / 1e9, 3)
        if a["ideal_s"] > 0:
            e["ideal_ms_per_iter"] = round(a["ideal_s"] * 1e3 / it, 4)
            e["eff_vs_xgmi_model"] = round(a["ideal_s"] / s_max, 4) if s_max > 0 else None
        out[kind] = e
    return out


def _window_bytes(metrics, kinds=None) -> int:
    """Bytes of the collectives a mapper recorded (optionally of the given kinds)."""
    return sum(c["bytes"] for c in metrics.collectives if kinds is None or c["kind"] in kinds)


# ----------------------------------------------------------------------------- MF-SGD
def bench_sgd(args, comm, torch):
    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings

    dev = comm.device
    P = comm.world_size
    t0 = time.perf_counter()
    u, i, v = synthetic_ratings(args.sgd_users, args.sgd_items, args.sgd_ratings, seed=7, device=dev)
    cfg = SGDConfig(rank=args.sgd_rank, epochs=args.sgd_warmup + args.sgd_epochs, test_every=0,
                    xcd_blocks=dev.type == "cuda", num_slices=args.sgd_slices or (1 if P == 1 else 2))
    if args.sgd_atomic >= 0:
        cfg.atomic = args.sgd_atomic
    m = SGDCollectiveMapper(comm, cfg, args.sgd_users, args.sgd_items, (u, i, v), None)
    m.init_model(_Reader())
    del u, i, v
    setup_s = time.perf_counter() - t0
    for ep in range(args.sgd_warmup):
        m.train_epoch(ep)
    m.rot.wait_all()
    sync(comm, torch)
    m.metrics.resolve()
    m.metrics.collectives.clear()
    clock = StepClock(comm, torch)
    t0 = time.perf_counter()
    n = 0
    clock.mark()
    for ep in range(args.sgd_warmup, args.sgd_warmup + args.sgd_epochs):
        n += m.train_epoch(ep)
        clock.mark()
    m.rot.wait_all()
    sync(comm, torch)
    dt = reduce_max(comm, torch, time.perf_counter() - t0)
    ep_s = clock.durations()
    rot_bytes = _window_bytes(m.metrics, ("rotate_wait",))
    coll = _coll_breakdown(m.metrics, args.sgd_epochs, comm, torch)
    # compute-stream time stalled on slice arrivals (HIP events around each stream-level
    # wait): the part of the model rotation NOT hidden behind the SGD kernels
    rot_exposed = reduce_max(comm, torch, sum(c["s"] for c in m.metrics.collectives if c["kind"] == "rotate_wait"))
    nt = torch.tensor([float(n)], dtype=torch.float64, device=dev)
    if P > 1:
        comm.all_reduce(nt)
    n = float(nt.item())
    train_rmse, _ = m._eval_ring(args.sgd_warmup + args.sgd_epochs - 1)
    st = step_stats(ep_s)
    placement = None
    if dev.type == "cuda":
        from harp_amd.ops import mf as MF

        placement = MF.check_placement(dev)  # residue -> XCC check of every timed launch
    return {
        "metric": "MF-SGD updates/sec (Netflix-shape synthetic, model rotation)",
        "updates_per_sec": round(n / dt, 1),
        "median_updates_per_sec": round(n / args.sgd_epochs / st["median"], 1) if st["median"] > 0 else None,
        "s_per_epoch": round(dt / args.sgd_epochs, 6),
        "epoch_s": st,
        "epochs": args.sgd_epochs,
        "warmup": args.sgd_warmup,
        "n_gpus": P,
        "sync_bytes_per_iter": int(rot_bytes / max(args.sgd_epochs, 1)),
        "rotation_exposed_s_per_epoch": round(rot_exposed / max(args.sgd_epochs, 1), 6),
        "collectives": coll,
        "rotation_strides": [s.stride for s in m.schedules],
        "xcd_placement": placement,
        "atomic_writeback": m.atomic,
        "hot_items": m.hot_items,
        "blocks_per_xcd": m.bpx,
        "cell_sum_p2": round(getattr(m, "cell_sum_p2", 0.0), 6),  # the concurrency cap's input (SGDConfig)
        "train_rmse": round(train_rmse, 6),
        "users": args.sgd_users, "items": args.sgd_items, "ratings": args.sgd_ratings, "rank": args.sgd_rank,
        "slices_per_rank": cfg.num_slices,
        "dtype": "fp32 factors",
        "setup_s": round(setup_s, 3),
        "scaling": "strong",
    }


# ----------------------------------------------------------------------------- PCA (config 4)
def bench_pca(args, comm, torch):
    """One PCA / correlation pass per step over N x d synthetic U[0,1) samples split over
    the ranks, through the library API ``stats.pca`` (PCADaalCollectiveMapper.java:121-154):
    step 1 is the MFMA SYRK partial result of the bf16 feature-major block with a row of
    ones (n, column sums and X^T X from ONE pass over one operand), one fp64 allreduce, the
    fp64 correlation, step 2 -- eigenvalues AND eigenvectors of the d x d correlation on the
    master (one-XCD reduction + divide and conquer + WY back-transform, ``ops.eig.eigh``) --
    and the broadcast of the d + 1 x d result. CPU ranks (gloo rehearsal) run the same API on
    row-major blocks (dtype bf16: the same rounding, fp32 accumulation)."""
    from harp_amd.models import stats as ST
    from harp_amd.ops import eig as EIG

    P, r = comm.world_size, comm.rank
    N, d = int(args.pca_n), args.pca_d
    n = N // P + (1 if r < N % P else 0)
    dev = comm.device
    if dev.type == "cuda":
        from harp_amd.ops import linalg as LA

        data = LA.FeatureMajor.uniform(n, d, 0.0, 1.0, seed=11 + r, device=dev)
        syrk = lambda: LA.syrk_t(data)  # noqa: E731
    else:
        g = torch.Generator().manual_seed(11 + r)
        data = torch.rand((n, d), generator=g)
        syrk = lambda: data.t() @ data  # noqa: E731

    from harp_amd.utils.metrics import Metrics

    met = Metrics(rank=r, world=P)

    def one_pass():
        return ST.pca(data, comm, dtype="bf16", metrics=met)

    res = one_pass()
    sync(comm, torch)
    met.resolve()
    met.collectives.clear()
    clock = StepClock(comm, torch)
    t0 = time.perf_counter()
    clock.mark()
    for _ in range(args.pca_steps):
        res = one_pass()
        clock.mark()
    sync(comm, torch)
    dt = reduce_max(comm, torch, time.perf_counter() - t0) / args.pca_steps
    st = step_stats(clock.durations())
    coll = _coll_breakdown(met, args.pca_steps, comm, torch)
    sclock = StepClock(comm, torch)  # the SYRK alone (device time on GPUs)
    sclock.mark()
    syrk()
    sclock.mark()
    sync(comm, torch)
    syrk_s = sclock.durations()[0]
    # step 2 alone on the master: eigenvalues + eigenvectors of the correlation matrix
    corr = ST.correlation(data, comm, dtype="bf16")["correlation"]
    eig_s = None
    orth = res_rel = None
    if r == 0:
        lam, V = EIG.eigh(corr)
        reps = 3
        if dev.type == "cuda":
            torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(reps):
            lam, V = EIG.eigh(corr)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        eig_s = (time.perf_counter() - te) / reps
        eye = torch.eye(d, dtype=torch.float64, device=V.device)
        orth = float((V.t() @ V - eye).abs().max())
        res_rel = float((corr @ V - V * lam).abs().max()) / float(lam.abs().max())
    if P > 1:
        comm.barrier()
    # useful SYRK work: the upper triangle (diagonal included) of the (d+1)^2 Gram of [X 1]
    # over this rank's rows -- what the kernel must compute, not the full-Gram equivalent
    flop = float(n) * (d + 1) * (d + 2)
    sync_bytes = ((d * d + d + 1) * 8 + (d + 1) * d * 8) if P > 1 else 0
    ev = res["eigenvalues"]
    return {"metric": "PCA correlation pass s/pass (N x d, stats.pca: MFMA SYRK + allreduce + fp64 eigenvalues "
                      "and eigenvectors)",
            "s_per_pass": round(dt, 6), "median_s_per_pass": round(st["median"], 6), "pass_s": st,
            "syrk_s": round(syrk_s, 6), "eig_s": round(eig_s, 6) if eig_s is not None else None,
            "eig": "eigenvalues + eigenvectors (ops.eig.eigh)", "eigvec_orth_err": orth, "eig_residual": res_rel,
            "N": N, "d": d, "steps": args.pca_steps, "n_gpus": P,
            "syrk_tflops": round(flop / syrk_s / 1e12, 1) if syrk_s > 0 else None,
            "syrk_flop_per_rank": flop, "sync_bytes_per_iter": int(sync_bytes), "collectives": coll,
            "max_eigenvalue": round(float(ev.max()), 6),
            "dtype": "bf16 in / fp32 acc / fp64 finalize" if dev.type == "cuda" else "bf16-rounded fp32 (CPU rehearsal)",
            "data": "synthetic U[0,1) generated on device", "scaling": "strong"}


# ----------------------------------------------------------------------------- LDA (config 5)
def _lda_run(args, comm, torch, local_server: bool, iters: int) -> dict:
    from harp_amd.models.lda import LDACollectiveMapper, LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.runtime.mapper import KeyValReader

    nd, V, K = int(args.lda_docs), int(args.lda_vocab), args.lda_topics
    P = comm.world_size
    t0 = time.perf_counter()
    toks = synthetic_corpus(nd, V, 1000, args.lda_len, seed=3, device=comm.device)
    _trace(comm, "lda corpus", t0)
    cfg = LDAConfig(num_topics=K, alpha=50.0 / K, beta=0.01, iterations=1 + iters, local_server=local_server)
    cls = LDAPushPullMapper if args.lda_strategy == "push_pull" else LDACollectiveMapper
    m = cls(comm, cfg, nd, V, toks)
    del toks  # init_model keeps only the mapper's own (int32, word-sorted) token arrays
    _trace(comm, "lda mapper", t0)
    m.init_model(KeyValReader([]))
    _trace(comm, "lda init_model", t0)
    setup_s = time.perf_counter() - t0
    m.iterate(0)
    if hasattr(m, "rot"):
        m.rot.wait_all()
    sync(comm, torch)
    m.metrics.resolve()
    m.metrics.collectives.clear()
    clock = StepClock(comm, torch)
    t0 = time.perf_counter()
    n = 0
    clock.mark()
    for it in range(1, 1 + iters):
        n += m.iterate(it)
        clock.mark()
    if hasattr(m, "rot"):
        m.rot.wait_all()
    sync(comm, torch)
    dt = reduce_max(comm, torch, time.perf_counter() - t0)
    st = step_stats(clock.durations())
    coll = _window_bytes(m.metrics)  # pull / push / rotate and the topic-delta allreduce
    breakdown = _coll_breakdown(m.metrics, iters, comm, torch)
    ll = m.log_likelihood(1 + iters)
    nt = torch.tensor([float(n)], dtype=torch.float64, device=comm.device)
    if P > 1:
        comm.all_reduce(nt)
    n = float(nt.item())
    out = {"tokens_per_sec": round(n / dt, 1), "s_per_iter": round(dt / iters, 6),
           "median_s_per_iter": round(st["median"], 6), "iter_s": st, "iters": iters,
           "sync_bytes_per_iter": int(coll / max(iters, 1)), "collectives": breakdown,
           "loglik_end": ll, "setup_s": round(setup_s, 3),
           "local_server": bool(getattr(m, "local_server", False)), "tokens_per_iter": int(n) // iters,
           "comm_mode": getattr(m, "comm_mode", "rotation"), "fused_rows": bool(getattr(m, "fused", False)),
           "sampler": "sparse" if getattr(m, "sparse", False) else "dense"}
    del m
    return out


def bench_lda(args, comm, torch):
    """LDA collapsed Gibbs sweeps over a synthetic corpus of docs x len tokens (vocab
    words, topics topics); push-pull parameter-server collective by default
    (LDAMPCollectiveMapper.java / contrib LDAMapperDyn.java push :380 / pull :429).
    The top-level record ALWAYS runs the collective the config names: at one rank too,
    every sweep pulls the word rows, samples and pushes the count deltas (VERDICT r4 weak
    #1). ``--lda-local-server auto`` additionally records, nested as ``local_server_alias``, the
    one-rank shortcut where the server table aliases the sampled slab (no pull / push)."""
    nd, V, K = int(args.lda_docs), int(args.lda_vocab), args.lda_topics
    rec = {"metric": f"LDA-CGS sampled tokens/sec ({args.lda_strategy})", "n_gpus": comm.world_size,
           "docs": nd, "vocab": V, "topics": K, "warmup": 1, "data": "synthetic corpus generated on device",
           "scaling": "strong"}
    rec.update(_lda_run(args, comm, torch, False, args.lda_iters))
    if (args.lda_strategy == "push_pull" and comm.world_size == 1 and args.lda_local_server == "auto"
            and comm.device.type == "cuda"):
        torch.cuda.empty_cache()
        alias = _lda_run(args, comm, torch, True, args.lda_iters)
        if alias["local_server"]:
            rec["local_server_alias"] = {k: alias[k] for k in ("tokens_per_sec", "s_per_iter", "median_s_per_iter",
                                                          "sync_bytes_per_iter", "loglik_end", "sampler")}
    return rec


# ----------------------------------------------------------------------------- helpers
def _trace(comm, what: str, t0: float) -> None:
    """HARP_BENCH_TRACE=1: per-rank setup progress on stderr (seconds since ``t0``)."""
    if os.environ.get("HARP_BENCH_TRACE"):
        print(f"bench trace rank {comm.rank}: {what} +{time.perf_counter() - t0:.2f}s", file=sys.stderr, flush=True)


class _Reader:
    def __iter__(self):
        return iter(())

    def __len__(self):
        return 0


class StepClock:
    """Per-step durations of a timed loop without a host sync inside it: a HIP event is
    recorded on the current stream at every step boundary (host clock on CPU ranks).
    :meth:`durations` (after the loop's closing sync) returns each step's max over the
    ranks -- BASELINE.md's protocol reports the median over >= 10 timed iterations."""

    def __init__(self, comm, torch):
        self.comm, self.torch = comm, torch
        self.cuda = comm.device.type == "cuda"
        self.marks = []

    def mark(self) -> None:
        if self.cuda:
            e = self.torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append(e)
        else:
            self.marks.append(time.perf_counter())

    def durations(self):
        torch = self.torch
        if self.cuda:
            self.marks[-1].synchronize()
            d = [a.elapsed_time(b) / 1e3 for a, b in zip(self.marks, self.marks[1:])]
        else:
            d = [b - a for a, b in zip(self.marks, self.marks[1:])]
        t = torch.tensor(d, dtype=torch.float64, device=self.comm.device)
        if self.comm.world_size > 1 and t.numel():
            import torch.distributed as dist

            self.comm.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.cpu().tolist()


def step_stats(d) -> dict:
    """median / mean / min / max of per-step seconds."""
    if not d:
        return {"median": 0.0, "mean": 0.0, "min": 0.0, "max": 0.0, "n": 0}
    x = sorted(d)
    k = len(x)
    med = x[k // 2] if k % 2 else 0.5 * (x[k // 2 - 1] + x[k // 2])
    return {"median": round(med, 6), "mean": round(sum(x) / k, 6), "min": round(x[0], 6), "max": round(x[-1], 6),
            "n": k}


# exit status of a rank whose nested-record watchdog fired: the headline line was printed,
# a nested record did not finish (GNU timeout's code, so launchers read it as a time limit)
NESTED_TIMEOUT_EXIT = 124


class _NestedGuard:
    """Bounds one nested record. If it has not finished after ``timeout_s``, rank 0 prints
    the (already measured) record with ``<name>.error`` and every rank leaves with
    ``os._exit(NESTED_TIMEOUT_EXIT)`` -- non-zero, so a hung peer is never reported as a
    clean run; the process teardown releases any RCCL kernel still waiting on a peer.
    ``cancel()`` returns False when the guard has already fired."""

    def __init__(self, timeout_s: float, rec: dict, rank: int, name: str = "sgd"):
        self.name = name
        import threading

        self._lock = threading.Lock()
        self._state = "armed"
        self.rec, self.rank = rec, rank
        self._t = threading.Timer(timeout_s, self._fire, args=(timeout_s,))
        self._t.daemon = True
        if timeout_s > 0:
            self._t.start()

    def _fire(self, timeout_s: float) -> None:
        with self._lock:
            if self._state != "armed":
                return
            self._state = "fired"
        print(f"bench: nested {self.name} record exceeded {timeout_s:g} s on rank {self.rank}; leaving",
              file=sys.stderr, flush=True)
        if self.rank == 0:
            rec = dict(self.rec, **{self.name: {"error": f"timeout after {timeout_s:g} s"}})
            print(json.dumps(rec), flush=True)
        os._exit(NESTED_TIMEOUT_EXIT)

    def cancel(self) -> bool:
        with self._lock:
            if self._state == "fired":
                return False
            self._state = "done"
        self._t.cancel()
        return True


def _nested(rec, name, fn, timeout_s, args, comm, torch):
    """rec[name] = fn(...) under a wall-clock guard; a failure is reported inside the
    record, never at the cost of the headline line."""
    guard = _NestedGuard(timeout_s, rec, comm.rank, name)
    t0 = time.perf_counter()
    _trace(comm, f"{name} record start", t0)
    try:
        rec[name] = fn(args, comm, torch)
        _trace(comm, f"{name} record done", t0)
    except Exception as e:  # noqa: BLE001
        rec[name] = {"error": f"{type(e).__name__}: {e}"[:500]}
        print(f"bench: nested {name} record failed on rank {comm.rank}: {e!r}", file=sys.stderr)
    if not guard.cancel():
        time.sleep(3600)  # the guard is printing / exiting this process


def sync(comm, torch):
    if comm.device.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    if comm.device.type == "cuda":
        torch.cuda.synchronize()


def reduce_max(comm, torch, x: float) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=comm.device)
    if comm.world_size > 1:
        import torch.distributed as dist

        comm.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run(args) -> int:
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    backend = args.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        ndev = torch.cuda.device_count()
        if world != args.gpus or world > ndev:
            print(f"bench: need --gpus ({args.gpus}) == world size ({world}) <= visible devices ({ndev})",
                  file=sys.stderr)
            return 3
    from harp_amd.ops.build import KERNEL_LIB, build_kernels

    if torch.cuda.is_available() and int(os.environ.get("LOCAL_RANK", "0")) == 0 and not os.path.exists(KERNEL_LIB):
        build_kernels()
    from harp_amd.runtime.launcher import init_distributed, shutdown

    # bounded collective watchdog for the bench (a stuck peer fails the run in minutes, not 30)
    os.environ.setdefault("HARP_DATA_MAX_WAIT_TIME", "600")
    comm = init_distributed(backend)
    if backend == "gloo" and torch.cuda.is_available():
        from harp_amd.parallel.comm import Communicator

        comm = Communicator(None, torch.device("cuda", torch.cuda.current_device()))
    if comm.world_size != args.gpus and backend != "gloo":
        raise RuntimeError(f"world size {comm.world_size} != --gpus {args.gpus}")
    # self-diagnosis before any timed record; bounded like the nested records (a guard that
    # fires prints what exists and exits 124 instead of hanging the node). The first barrier
    # (rank 0's rare build finishes before any rank loads the library) is inside the bound:
    # it is the first collective of the run.
    def barrier_and_preflight(a, c, t):
        if world > 1:
            c.barrier()
        return rccl_preflight(a, c, t)

    pre = {}
    _nested(pre, "rccl", barrier_and_preflight, args.preflight_timeout, args, comm, torch)
    rec = bench_kmeans(args, comm, torch)
    rec["rccl"] = pre["rccl"]
    if comm.device.type == "cuda":
        torch.cuda.empty_cache()
    want_sgd = args.sgd == "on" or (args.sgd == "auto" and comm.device.type == "cuda")
    if want_sgd:
        # the nested record must never cost the headline line: a failure is reported inside
        # it, and a hang (e.g. a stuck RCCL peer in the rotation ring, which no Python
        # exception interrupts) is bounded by a per-rank wall-clock guard
        _nested(rec, "sgd", bench_sgd, args.sgd_timeout, args, comm, torch)
    want_extras = args.extras == "on" or (args.extras == "auto" and comm.device.type == "cuda")
    if want_extras:
        for name, fn in (("pca", bench_pca), ("lda", bench_lda)):
            if comm.device.type == "cuda":
                torch.cuda.empty_cache()
            _nested(rec, name, fn, args.extras_timeout, args, comm, torch)
    if comm.rank == 0:
        print(json.dumps(rec), flush=True)
    shutdown()
    return 0


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn(args, argv)
    return run(args)


if __name__ == "__main__":
    sys.exit(main())
