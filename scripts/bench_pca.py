#!/usr/bin/env python3
"""Covariance/correlation-PCA partial-result bench (BASELINE config #4: N=1e8 x d=1000):
time per pass of the MFMA SYRK partial (X^T X + column sums + n from one GEMM) plus the
allreduce and the fp64 finalize/eigendecomposition. Strong scaling over ranks.

python scripts/bench_pca.py [--n 1e8] [--d 1000] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--d", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--splits", type=int, default=0)
    a = ap.parse_args()
    import torch

    from harp_amd.models.common import reduce_partials
    from harp_amd.ops import linalg as LA
    from harp_amd.ops import eig as EIG
    from harp_amd.runtime.launcher import init_distributed, shutdown

    comm = init_distributed()
    P, r = comm.world_size, comm.rank
    N = int(a.n)
    n = N // P + (1 if r < N % P else 0)
    fm = LA.FeatureMajor.uniform(n, a.d, 0.0, 1.0, seed=11 + r, device=comm.device)
    torch.cuda.synchronize()

    def one_pass():
        G = LA.syrk_t(fm, num_splits=a.splits, variant=a.variant)
        part = reduce_partials(comm, {"g": G}, dtype=torch.float32)
        Gs = LA.symmetrize_upper(part["g"]).double()
        d = a.d
        cnt = Gs[d, d]
        mean = Gs[:d, d] / cnt
        cov = (Gs[:d, :d] - cnt * torch.outer(mean, mean)) / (cnt - 1)
        sd = torch.diagonal(cov).sqrt()
        corr = cov / torch.outer(sd, sd)
        return EIG.eigvalsh(corr)  # one-XCD tridiagonalisation + multisection (csrc/eig.hip)

    for _ in range(a.warmup):
        one_pass()
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ev = one_pass()
    torch.cuda.synchronize()
    comm.barrier()
    dt = (time.perf_counter() - t0) / a.steps
    t_syrk = None
    if r == 0:
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        LA.syrk_t(fm, num_splits=a.splits, variant=a.variant)
        e.record()
        e.synchronize()
        t_syrk = s.elapsed_time(e) / 1e3
    if r == 0:
        # useful work: the upper triangle (diagonal included) of the (d+1)^2 Gram of [X 1]
        flop = float(n) * (a.d + 1) * (a.d + 2)
        print(json.dumps({"metric": "PCA/covariance partial-result pass (N x d, MFMA SYRK + allreduce + eig)",
                          "value": dt, "unit": "s/pass", "n_gpus": P, "N": N, "d": a.d,
                          "syrk_s_local": t_syrk, "syrk_tflops_local": flop / t_syrk / 1e12,
                          "max_eigenvalue": float(ev.max()), "dtype": "bf16 in / fp32 acc / fp64 finalize"}), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
