"""ALS half-iteration (all user rows solved against the item factors) on one GPU: the
native normal-equation kernel (``csrc/als.hip``) + batched Cholesky vs the torch
outer-product / index_add formulation. Synthetic MovieLens-20M-like shape."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from harp_amd.models import als as A
from harp_amd.ops import als as OA


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=138000)
    ap.add_argument("--items", type=int, default=27000)
    ap.add_argument("--nnz", type=float, default=2e7)
    ap.add_argument("--factors", type=int, default=64)
    ap.add_argument("--implicit", type=int, default=1)
    ap.add_argument("--native-only", action="store_true", help="skip the torch comparison (profiling)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    nnz = int(a.nnz)
    rows = torch.sort(torch.randint(0, a.users, (nnz,), device=dev, generator=g)).values
    cols = (torch.rand(nnz, device=dev, generator=g) ** 2 * a.items).long().clamp_max(a.items - 1)
    vals = torch.randint(1, 6, (nnz,), device=dev, generator=g).float()
    F = torch.randn(a.items, a.factors, device=dev, generator=g) * 0.1
    cfg = A.ALSConfig(factors=a.factors, implicit=bool(a.implicit), alpha=1.0, lam=0.1)

    def run():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x = A.solve_rows(rows, cols, vals, a.users, F, cfg)
        torch.cuda.synchronize()
        return x, time.perf_counter() - t0

    run()
    xn, tn = run()
    print("native %.4f s" % tn, flush=True)
    if a.native_only:
        return
    OA.available = lambda t: False  # torch formulation
    run()
    xt, tt = run()
    d = float((xn - xt).abs().max())
    print(json.dumps({"metric": "ALS half-iteration seconds (user solve)", "value": tn, "unit": "s",
                      "torch_s": tt, "speedup": tt / tn, "users": a.users, "items": a.items, "nnz": nnz,
                      "factors": a.factors, "implicit": bool(a.implicit), "max_abs_diff_vs_torch": d,
                      "n_gpus": 1}), flush=True)


if __name__ == "__main__":
    main()
