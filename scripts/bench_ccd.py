#!/usr/bin/env python3
"""MF-CCD bench: Netflix-shape synthetic (480,189 x 17,770, ~100M ratings), rank 120
(the reference's clueweb CCD rank), lambda 0.1: seconds per iteration (row + column
phase + residual recomputes) and updates/s (= 2 * nnz * rank coordinate updates / s).

python scripts/bench_ccd.py [--users 480189 --items 17770 --ratings 1e8 --rank 120 --iters 3]
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
    ap.add_argument("--ratings", type=float, default=1e8)
    ap.add_argument("--rank", type=int, default=120)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--mode", default="allgather", choices=["allgather", "rotation"])
    ap.add_argument("--resync", type=int, default=10, help="CCDConfig.residual_resync (1 = recompute every phase)")
    a = ap.parse_args()
    import torch

    from harp_amd.models.ccd import CCDConfig, train_ccd
    from harp_amd.models.sgd_mf import synthetic_ratings
    from harp_amd.runtime.launcher import init_distributed, shutdown

    comm = init_distributed()
    u, i, v = synthetic_ratings(a.users, a.items, int(a.ratings), seed=0, device=comm.device)
    P, me = comm.world_size, comm.rank
    n = u.numel()
    sl = slice(me * n // P, (me + 1) * n // P)
    t0 = time.perf_counter()
    out = train_ccd(comm, u[sl], i[sl], v[sl], a.users, a.items,
                    CCDConfig(rank=a.rank, lam=0.1, iterations=a.iters + 1, mode=a.mode,
                                                                  residual_resync=a.resync))
    wall = time.perf_counter() - t0
    its = [h["time_s"] for h in out["history"][1:]]
    s_it = sorted(its)[len(its) // 2]
    if me == 0:
        print(json.dumps({"metric": "MF-CCD seconds/iteration", "value": s_it, "unit": "s/iter", "n_gpus": P,
                          "rank": a.rank, "nnz": n, "mode": a.mode, "residual_resync": a.resync,
                          "peak_hbm_gb": torch.cuda.max_memory_allocated() / 2**30 if torch.cuda.is_available() else None, "coord_updates_per_s": 2 * n * a.rank / s_it,
                          "train_rmse": [h["train_rmse"] for h in out["history"]], "wall_s": wall}), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
