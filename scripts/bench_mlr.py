#!/usr/bin/env python3
"""MLR (contrib, one-vs-rest logistic regression) SGD pass on an rcv1-shaped synthetic
shard: one-launch HIP pass (csrc/mlr.hip) vs the torch mini-batch loop on the same GPU."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=23149)     # rcv1 (lyrl2004) training docs
    ap.add_argument("--dim", type=int, default=47236)
    ap.add_argument("--topics", type=int, default=103)
    ap.add_argument("--nnz-per-row", type=int, default=75)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--alpha", type=float, default=1.0)
    args = ap.parse_args()
    import torch

    from harp_amd.models import mlr as M

    dev = torch.device("cuda", 0)
    n, d, T, z = args.rows, args.dim, args.topics, args.nnz_per_row
    g = torch.Generator(device=dev).manual_seed(0)
    cols = torch.randint(0, d, (n, z), device=dev, generator=g).sort(1).values.reshape(-1)
    vals = torch.rand(n * z, device=dev, generator=g, dtype=torch.float64) / z ** 0.5
    X = M.CSRRows(torch.arange(0, n * z + 1, z, device=dev), cols, vals, d)
    Y = (torch.rand(n, T, device=dev, generator=g) < 0.1).float()
    W0 = torch.zeros((T, d + 1), dtype=torch.float64, device=dev)

    def timed(fn, reps):
        W = W0.clone()
        fn(W)
        torch.cuda.synchronize()
        W = W0.clone()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(W)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps, W

    tn, Wn = timed(lambda W: M._sgd_pass(W, X, Y, args.alpha, args.batch), 5)
    tt, Wt = timed(lambda W: M._sgd_pass_torch(W, X, Y, args.alpha, args.batch), 1)
    Wn1 = W0.clone()
    M._sgd_pass(Wn1, X, Y, args.alpha, args.batch)
    Wt1 = W0.clone()
    M._sgd_pass_torch(Wt1, X, Y, args.alpha, args.batch)
    print(json.dumps({"metric": "MLR SGD pass seconds (rcv1-shaped shard, fp64)", "value": tn, "unit": "s",
                      "n_gpus": 1, "rows": n, "dim": d, "topics": T, "nnz": n * z, "batch": args.batch,
                      "native_s": tn, "torch_s": tt, "speedup_vs_torch": tt / tn,
                      "alpha": args.alpha,
                      "max_abs_diff_one_pass": float((Wn1 - Wt1).abs().max()), "max_abs_w": float(Wt1.abs().max()),
                      "bias_range": [float(Wt1[:, 0].min()), float(Wt1[:, 0].max())]}))


if __name__ == "__main__":
    main()
