#!/usr/bin/env python3
"""Headline benchmark: K-means sec/iteration, N=1e8 points, d=100, K=1e4, bf16 MFMA.

BASELINE.json metric: "sec/iteration K-means (N=1e8, d=100, K=1e4) at 1/2/4/8 MI355X".
The problem size is FIXED (N = 1e8 total points split evenly over the ranks), so this is
strong scaling; ``value`` is the whole-job seconds per Lloyd iteration (max over ranks),
lower is better. One timed step = one full iteration of the reference's regroup/allgather
-> here allreduce K-means loop: fused MFMA assign + accumulate over all local points,
RCCL model sync of the 1e4 x 112 fp32 partial sums, normalize, centroid operand prepare.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
Data: synthetic U[0,1000) points generated on the device, random-init centroids
(no datasets are available offline).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sec/iteration K-means (N=1e8, d=100, K=1e4)"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--points", type=float, default=1e8, help="total points (strong scaling)")
    ap.add_argument("--centroids", type=int, default=10000)
    ap.add_argument("--dim", type=int, default=100)
    ap.add_argument("--strategy", default="allreduce")
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--backend", default=None, help="override (e.g. gloo to rehearse >1 rank on one GPU)")
    ap.add_argument("--graph", action="store_true", help="replay each iteration's kernels from HIP graphs")
    args = ap.parse_args()

    import torch

    from harp_amd.ops.build import KERNEL_LIB, build_kernels

    if int(os.environ.get("LOCAL_RANK", "0")) == 0 and not os.path.exists(KERNEL_LIB):
        build_kernels()
    from harp_amd.models.kmeans import KMeansCollectiveMapper, KMeansConfig
    from harp_amd.ops import kmeans as K
    from harp_amd.runtime.launcher import init_distributed, shutdown
    from harp_amd.runtime.mapper import KeyValReader

    world = int(os.environ.get("WORLD_SIZE", "1"))
    backend = args.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    comm = init_distributed(backend)
    if backend == "gloo" and torch.cuda.is_available():
        from harp_amd.parallel.comm import Communicator

        comm = Communicator(None, torch.device("cuda", torch.cuda.current_device()))
    if world > 1:
        comm.barrier()  # rank 0's (rare) build finishes before any rank loads the library
    P, rank = comm.world_size, comm.rank
    N = int(args.points)
    n_local = N // P + (1 if rank < N % P else 0)
    cfg = KMeansConfig(num_points=n_local, num_centroids=args.centroids, dim=args.dim, iterations=10**9,
                       strategy=args.strategy, objective_every=0,
                       variant=K.DEFAULT_VARIANT if args.variant is None else args.variant, graph=args.graph)
    m = KMeansCollectiveMapper(comm, cfg)
    m.init_model(KeyValReader([]))
    for it in range(args.warmup):
        m.step(it)

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        comm.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    sync()
    m.metrics.timer.reset()
    t0 = time.perf_counter()
    for it in range(args.steps):
        m.step(args.warmup + it)
    sync()
    elapsed = time.perf_counter() - t0
    phases = m.metrics.timer.flush()
    t = torch.tensor([elapsed], dtype=torch.float64, device=comm.device)
    if P > 1:
        import torch.distributed as dist

        comm.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    sec_per_iter = elapsed / args.steps
    # objective after timing (one extra assign pass, outside the timed region) as a sanity value
    _, obj = K.assign(m.X, m.op, sums=None, want_objective=True, variant=cfg.variant)
    o = obj.reshape(1).to(comm.device, torch.float64)
    if P > 1:
        comm.all_reduce(o)
    flops = 2.0 * N * args.centroids * args.dim
    if rank == 0:
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
            "dtype": "bf16",
            "data": "synthetic U[0,1000) points generated on device; random-init centroids",
            "config": {"model": f"kmeans-{args.strategy}", "N": N, "d": args.dim, "K": args.centroids,
                       "global_batch": N, "seq_len": None, "parallelism": f"dp{P}"},
            "points_per_sec": round(N / sec_per_iter, 1),
            "effective_tflops": round(flops / sec_per_iter / 1e12, 1),
            "phase_ms_per_iter": {k: round(v / args.steps * 1e3, 3) for k, v in phases.items()},
            "mean_sq_dist": float(o.item()) / N,
            "kernel_variant": cfg.variant,
            "hip_graph": bool(args.graph),
        }
        print(json.dumps(rec), flush=True)
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
