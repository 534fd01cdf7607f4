#!/usr/bin/env python3
"""kNN search benchmark: fused GEMM + top-k selection (csrc/knn.hip) vs the torch path
(distance tile + torch.topk), same fp32 GEMM underneath. Synthetic Gaussian rows."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train", type=int, default=1_000_000)
    ap.add_argument("--queries", type=int, default=16384)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from harp_amd.ops import knn as KN

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    T = torch.randn(args.train, args.dim, device=dev, generator=g)
    Q = torch.randn(args.queries, args.dim, device=dev, generator=g)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps, out

    tn, (dn, in_) = timed(lambda: KN.knn_search(T, Q, args.k))
    tt, (dt, it) = timed(lambda: KN._torch_search(T, Q, args.k, 8192))
    gemm_s, _ = timed(lambda: [Q[a:a + 8192] @ T[b:b + 65536].t() for a in range(0, args.queries, 8192)
                               for b in range(0, args.train, 65536)])
    agree = float((dn - dt).abs().max().item())
    print(json.dumps({"metric": "kNN search seconds (exact, fp32)", "value": tn, "unit": "s", "n_gpus": 1,
                      "train": args.train, "queries": args.queries, "dim": args.dim, "k": args.k,
                      "native_s": tn, "torch_topk_s": tt, "gemm_only_s": gemm_s, "speedup_vs_torch": tt / tn,
                      "max_abs_dist_diff": agree}))


if __name__ == "__main__":
    main()
