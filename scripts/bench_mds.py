#!/usr/bin/env python3
"""WDA-MDS SMACOF step on one GPU: fused B(Z) X / stress row kernels (csrc/mds.hip) vs the
torch formulation (Gram GEMM + distance / mask / B tensors). Synthetic 3-D point cloud."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from harp_amd.models import mds as MD
    from harp_amd.parallel.comm import Communicator

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    Y = torch.rand(args.n, args.dim, device=dev, generator=g, dtype=torch.float64)
    D = torch.cdist(Y, Y)
    W = torch.ones_like(D)
    X = torch.rand(args.n, args.dim, device=dev, generator=g, dtype=torch.float64)
    rows = MD._Rows(Communicator(None, dev), D, W, 0)
    T = 0.01

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps, out

    bc_n, B1 = timed(lambda: rows.bc(X, T, args.dim))
    st_n, s1 = timed(lambda: rows.stress(X, T, args.dim))
    step_n, _ = timed(lambda: MD._cg(rows, X, rows.bc(X, T, args.dim), 20))
    rows._native = lambda X: False
    bc_t, B2 = timed(lambda: rows.bc(X, T, args.dim))
    st_t, s2 = timed(lambda: rows.stress(X, T, args.dim))
    print(json.dumps({"metric": "WDA-MDS B(Z)X seconds (fp64 row block)", "value": bc_n, "unit": "s", "n_gpus": 1,
                      "n": args.n, "dim": args.dim, "bc_native_s": bc_n, "bc_torch_s": bc_t,
                      "stress_native_s": st_n, "stress_torch_s": st_t, "bc_speedup": bc_t / bc_n,
                      "stress_speedup": st_t / st_n, "smacof_step_native_s": step_n,
                      "bc_max_rel_diff": float((B1 - B2).abs().max() / B2.abs().max()),
                      "stress_rel_diff": float(abs(s1 - s2) / s2)}))


if __name__ == "__main__":
    main()
