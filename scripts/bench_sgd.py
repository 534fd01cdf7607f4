#!/usr/bin/env python3
"""MF-SGD updates/sec on a Netflix-shaped synthetic problem (480,189 x 17,770, ~100.5M
ratings, rank 128) with H model rotation (2 slices per worker) — BASELINE.json's second
metric. Strong scaling: the rating set is fixed, users are partitioned over the ranks.

python scripts/bench_sgd.py [--epochs 3] [--warmup 1]   (N GPUs: under torchrun)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=480189)
    ap.add_argument("--items", type=int, default=17770)
    ap.add_argument("--ratings", type=int, default=100480507)
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--lr", type=float, default=0.002)
    ap.add_argument("--lam", type=float, default=0.05)
    ap.add_argument("--layout", choices=("xcd", "flat"), default="xcd")
    ap.add_argument("--skew", type=float, default=2.0, help="item popularity skew (1 = uniform)")
    ap.add_argument("--blocks-per-xcd", type=int, default=128)
    ap.add_argument("--conflicts-per-rating", type=float, default=0.0,
                    help="SGDConfig concurrency cap (0 = use --blocks-per-xcd as is)")
    ap.add_argument("--variant", type=int, default=0, help="kernel variant: 0 (per-sub-step launches), 1 (flow)")
    ap.add_argument("--slices", type=int, default=1,
                    help="H slices per rank (rotation slice steps per epoch; 1 as in bench.py, profiles/r3_sgd_slices)")
    a = ap.parse_args()
    import torch

    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings
    from harp_amd.runtime.launcher import init_distributed, shutdown
    from harp_amd.runtime.mapper import KeyValReader

    comm = init_distributed()
    dev = comm.device
    t0 = time.perf_counter()
    u, i, v = synthetic_ratings(a.users, a.items, a.ratings, seed=7, device=dev, skew=a.skew)
    gen_s = time.perf_counter() - t0
    cfg = SGDConfig(rank=a.rank, lam=a.lam, lr=a.lr, epochs=a.warmup + a.epochs, chunk=a.chunk, test_every=0,
                    xcd_blocks=a.layout == "xcd", blocks_per_xcd=a.blocks_per_xcd, conflicts_per_rating=a.conflicts_per_rating,
                    kernel_variant=a.variant, num_slices=a.slices)
    m = SGDCollectiveMapper(comm, cfg, a.users, a.items, (u, i, v), None)
    m.init_model(KeyValReader([]))
    del u, i, v
    for ep in range(a.warmup):
        m.train_epoch(ep)
    m.rot.wait_all()
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for ep in range(a.warmup, a.warmup + a.epochs):
        n += m.train_epoch(ep)
    m.rot.wait_all()
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tot = torch.tensor([float(n), dt], dtype=torch.float64, device=dev)
    if comm.world_size > 1:
        import torch.distributed as dist

        n_all = tot[:1].clone()
        comm.all_reduce(n_all)
        t_all = tot[1:].clone()
        comm.all_reduce(t_all, op=dist.ReduceOp.MAX)
        n, dt = float(n_all.item()), float(t_all.item())
    tr, _ = m._eval_ring(a.warmup + a.epochs - 1)
    if comm.rank == 0:
        print(json.dumps({"metric": f"MF-SGD updates/sec (Netflix-shape synthetic, rank {a.rank}, model rotation)",
                          "value": n / dt, "unit": "updates/s", "n_gpus": comm.world_size, "epochs": a.epochs,
                          "s_per_epoch": dt / a.epochs, "train_rmse": tr, "data_gen_s": gen_s,
                          "ratings": a.ratings, "rank": a.rank, "dtype": "fp32 factors",
                          "layout": a.layout, "skew": a.skew, "chunk": a.chunk, "blocks_per_xcd": a.blocks_per_xcd, "variant": a.variant, "slices": a.slices}), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
