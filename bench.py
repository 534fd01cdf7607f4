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
128, H split into 2 slices per rank that rotate around the ring (model rotation); epochs
timed after warmup; updates/sec = ratings trained / epoch time
(SGDCollectiveMapper.java:294-298).

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
    ap.add_argument("--sgd-epochs", type=int, default=5)
    ap.add_argument("--sgd-warmup", type=int, default=1)
    ap.add_argument("--sgd-slices", type=int, default=2, help="H slices per rank (rotation pipeline depth)")
    ap.add_argument("--sgd-timeout", type=float, default=240.0,
                    help="wall-clock bound (s) on the nested MF-SGD record; past it rank 0 prints the "
                         "K-means line with an sgd error and every rank exits")
    ap.add_argument("--extras", choices=("auto", "on", "off"), default="auto",
                    help="nested PCA (BASELINE config 4) and LDA (config 5) records (auto: on GPUs)")
    ap.add_argument("--pca-n", type=float, default=1e8)
    ap.add_argument("--pca-d", type=int, default=1000)
    ap.add_argument("--pca-steps", type=int, default=3)
    ap.add_argument("--lda-docs", type=float, default=1e6)
    ap.add_argument("--lda-vocab", type=float, default=1e6)
    ap.add_argument("--lda-topics", type=int, default=1000)
    ap.add_argument("--lda-len", type=int, default=100)
    ap.add_argument("--lda-iters", type=int, default=3)
    ap.add_argument("--lda-strategy", choices=("push_pull", "rotation"), default="push_pull")
    ap.add_argument("--extras-timeout", type=float, default=180.0, help="wall-clock bound (s) per nested record")
    ap.add_argument("--metrics-jsonl", default="", help="per-iteration phase/bytes records (JSONL)")
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
    t0 = time.perf_counter()
    for it in range(args.steps):
        m.step(args.warmup + it)
    sync(comm, torch)
    elapsed = time.perf_counter() - t0
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


# ----------------------------------------------------------------------------- MF-SGD
def bench_sgd(args, comm, torch):
    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings

    dev = comm.device
    t0 = time.perf_counter()
    u, i, v = synthetic_ratings(args.sgd_users, args.sgd_items, args.sgd_ratings, seed=7, device=dev)
    cfg = SGDConfig(rank=args.sgd_rank, epochs=args.sgd_warmup + args.sgd_epochs, test_every=0,
                    xcd_blocks=dev.type == "cuda", num_slices=args.sgd_slices)
    m = SGDCollectiveMapper(comm, cfg, args.sgd_users, args.sgd_items, (u, i, v), None)
    m.init_model(_Reader())
    del u, i, v
    setup_s = time.perf_counter() - t0
    for ep in range(args.sgd_warmup):
        m.train_epoch(ep)
    m.rot.wait_all()
    sync(comm, torch)
    t0 = time.perf_counter()
    n = 0
    for ep in range(args.sgd_warmup, args.sgd_warmup + args.sgd_epochs):
        n += m.train_epoch(ep)
    m.rot.wait_all()
    sync(comm, torch)
    dt = reduce_max(comm, torch, time.perf_counter() - t0)
    nt = torch.tensor([float(n)], dtype=torch.float64, device=dev)
    if comm.world_size > 1:
        comm.all_reduce(nt)
    n = float(nt.item())
    train_rmse, _ = m._eval_ring(args.sgd_warmup + args.sgd_epochs - 1)
    return {
        "metric": "MF-SGD updates/sec (Netflix-shape synthetic, model rotation)",
        "updates_per_sec": round(n / dt, 1),
        "s_per_epoch": round(dt / args.sgd_epochs, 6),
        "epochs": args.sgd_epochs,
        "warmup": args.sgd_warmup,
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
    the ranks: MFMA SYRK partial result (G = [X 1]^T [X 1], upper tiles), one allreduce,
    fp64 correlation + eigenvalues (PCADaalCollectiveMapper.java:121-147)."""
    from harp_amd.models.common import reduce_partials
    from harp_amd.ops import linalg as LA

    P, r = comm.world_size, comm.rank
    N, d = int(args.pca_n), args.pca_d
    n = N // P + (1 if r < N % P else 0)
    fm = LA.FeatureMajor.uniform(n, d, 0.0, 1.0, seed=11 + r, device=comm.device)

    def one_pass():
        G = LA.syrk_t(fm)
        Gs = LA.symmetrize_upper(reduce_partials(comm, {"g": G}, dtype=torch.float32)["g"]).double()
        cnt = Gs[d, d]
        mean = Gs[:d, d] / cnt
        cov = (Gs[:d, :d] - cnt * torch.outer(mean, mean)) / (cnt - 1)
        sd = torch.diagonal(cov).sqrt()
        return torch.linalg.eigvalsh(cov / torch.outer(sd, sd))

    one_pass()
    sync(comm, torch)
    t0 = time.perf_counter()
    for _ in range(args.pca_steps):
        ev = one_pass()
    sync(comm, torch)
    dt = reduce_max(comm, torch, time.perf_counter() - t0) / args.pca_steps
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    LA.syrk_t(fm)
    e.record()
    e.synchronize()
    syrk_s = reduce_max(comm, torch, s.elapsed_time(e) / 1e3)
    del fm
    return {"metric": "PCA correlation pass s/pass (N x d, MFMA SYRK + allreduce + fp64 eig)", "s_per_pass": round(dt, 6),
            "syrk_s": round(syrk_s, 6), "N": N, "d": d, "steps": args.pca_steps,
            "gram_equiv_tflops": round(2.0 * N * d * d / P / syrk_s / 1e12, 1),
            "max_eigenvalue": round(float(ev.max()), 6), "dtype": "bf16 in / fp32 acc / fp64 finalize",
            "data": "synthetic U[0,1) generated on device", "scaling": "strong"}


# ----------------------------------------------------------------------------- LDA (config 5)
def bench_lda(args, comm, torch):
    """LDA collapsed Gibbs sweeps over a synthetic corpus of docs x len tokens (vocab
    words, topics topics); push-pull parameter-server collective by default
    (LDAMPCollectiveMapper.java / contrib LDAMapperDyn.java push :380 / pull :429)."""
    from harp_amd.models.lda import LDACollectiveMapper, LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.runtime.mapper import KeyValReader

    nd, V, K = int(args.lda_docs), int(args.lda_vocab), args.lda_topics
    t0 = time.perf_counter()
    toks = synthetic_corpus(nd, V, 1000, args.lda_len, seed=3, device=comm.device)
    cfg = LDAConfig(num_topics=K, alpha=50.0 / K, beta=0.01, iterations=1 + args.lda_iters)
    cls = LDAPushPullMapper if args.lda_strategy == "push_pull" else LDACollectiveMapper
    m = cls(comm, cfg, nd, V, toks)
    m.init_model(KeyValReader([]))
    del toks
    setup_s = time.perf_counter() - t0
    m.iterate(0)
    if hasattr(m, "rot"):
        m.rot.wait_all()
    sync(comm, torch)
    t0 = time.perf_counter()
    n = 0
    for it in range(1, 1 + args.lda_iters):
        n += m.iterate(it)
    if hasattr(m, "rot"):
        m.rot.wait_all()
    sync(comm, torch)
    dt = reduce_max(comm, torch, time.perf_counter() - t0)
    ll = m.log_likelihood(1 + args.lda_iters)
    nt = torch.tensor([float(n)], dtype=torch.float64, device=comm.device)
    if comm.world_size > 1:
        comm.all_reduce(nt)
    n = float(nt.item())
    del m
    return {"metric": f"LDA-CGS sampled tokens/sec ({args.lda_strategy})", "tokens_per_sec": round(n / dt, 1),
            "s_per_iter": round(dt / args.lda_iters, 6), "iters": args.lda_iters, "warmup": 1,
            "docs": nd, "vocab": V, "topics": K, "tokens_per_iter": int(n) // args.lda_iters,
            "loglik_end": ll, "setup_s": round(setup_s, 3), "data": "synthetic corpus generated on device",
            "scaling": "strong"}


# ----------------------------------------------------------------------------- helpers
class _Reader:
    def __iter__(self):
        return iter(())

    def __len__(self):
        return 0


class _NestedGuard:
    """Bounds one nested record. If it has not finished after ``timeout_s``, rank 0 prints
    the (already measured) record with ``<name>.error`` and every rank leaves with
    ``os._exit(0)`` — the process teardown releases any RCCL kernel still waiting on a
    peer. ``cancel()`` returns False when the guard has already fired."""

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
        os._exit(0)

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
    try:
        rec[name] = fn(args, comm, torch)
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
    if world > 1:
        comm.barrier()  # rank 0's (rare) build finishes before any rank loads the library
    rec = bench_kmeans(args, comm, torch)
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
