#!/usr/bin/env python3
"""Sparse (CSR) K-means iteration, fp64: fused HIP E-step + accumulate (csrc/kmeans_csr.hip)
vs the torch formulation (sparse-dense product, [n, K] distances, one-hot SpMM). Synthetic
rows with a fixed number of random nonzeros."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=10_000)
    ap.add_argument("--nnz-per-row", type=int, default=50)
    ap.add_argument("--centroids", type=int, default=100)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    import torch

    from harp_amd.models import kmeans_csr as M
    from harp_amd.ops import kmeans_csr as KC

    dev = torch.device("cuda", 0)
    n, d, z, K = args.rows, args.dim, args.nnz_per_row, args.centroids
    g = torch.Generator(device=dev).manual_seed(0)
    cols = torch.randint(0, d, (n * z,), device=dev, generator=g)
    rows = torch.arange(n, device=dev).repeat_interleave(z)
    vals = torch.rand(n * z, device=dev, generator=g, dtype=torch.float64)
    X = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (n, d)).coalesce().to_sparse_csr()
    C = torch.rand(K, d, device=dev, dtype=torch.float64, generator=g) * 0.01
    A = KC.to_device_csr(X)

    def native():
        return KC.assign_accumulate(A, C)

    def torch_path():
        D = M.sq_dist(X, C)
        m, lab = D.min(1)
        onehot = torch.zeros((n, K), dtype=torch.float64, device=dev)
        onehot[torch.arange(n, device=dev), lab] = 1.0
        S = torch.sparse.mm(X.to_sparse_coo().t(), onehot).t()
        return lab, m, S, onehot.sum(0)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.iters, out

    tn, (lab, m, S, cnt) = timed(native)
    tt, (lab2, m2, S2, cnt2) = timed(torch_path)
    print(json.dumps({"metric": "sparse K-means E-step + accumulate seconds (fp64)", "value": tn, "unit": "s",
                      "n_gpus": 1, "rows": n, "dim": d, "nnz": int(X.values().numel()), "K": K, "native_s": tn,
                      "torch_s": tt, "speedup_vs_torch": tt / tn,
                      "label_agreement": float((lab == lab2).double().mean()),
                      "objective_rel_diff": float(abs(m.sum() - m2.sum()) / m2.sum()),
                      "sums_max_abs_diff": float((S - S2).abs().max())}))


if __name__ == "__main__":
    main()
