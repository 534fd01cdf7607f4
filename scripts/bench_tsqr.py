#!/usr/bin/env python3
"""Tall-skinny QR: hand-written fp64 Householder TSQR panel kernels (csrc/tsqr.hip),
torch.linalg.qr (rocSOLVER geqrf + orgqr) and CholeskyQR2 (models/stats.py, the GPU default)
on the same fp64 matrix.

python scripts/bench_tsqr.py [--n 4e6] [--d 64] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=4e6)
    ap.add_argument("--ds", default="16,32,64")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from harp_amd.models import stats as ST
    from harp_amd.ops import linalg as LA

    n = int(a.n)
    for d in [int(x) for x in a.ds.split(",")]:
        A = torch.randn(n, d, dtype=torch.float64, device="cuda")
        res = {}
        def chol():
            o = ST.cholesky_qr2(A)
            return o["Q"], o["R"]

        for name, fn in (("native", lambda: LA.house_tsqr(A)), ("torch", lambda: torch.linalg.qr(A)),
                         ("cholqr2", chol)):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                Q, R = fn()
            torch.cuda.synchronize()
            res[name] = (time.perf_counter() - t0) / a.reps
        Q, R = LA.house_tsqr(A)
        err = float((Q @ R - A).abs().max())
        orth = float((Q.t() @ Q - torch.eye(d, dtype=torch.float64, device="cuda")).abs().max())
        Qc, Rc = chol()
        orth_c = float((Qc.t() @ Qc - torch.eye(d, dtype=torch.float64, device="cuda")).abs().max())
        print(json.dumps({"metric": "TSQR (Q and R) seconds", "n": n, "d": d, "native_s": res["native"],
                          "torch_s": res["torch"], "cholqr2_s": res["cholqr2"], "cholqr2_orth": orth_c,
                          "speedup": res["torch"] / res["native"],
                          "max_abs_QR_minus_A": err, "max_abs_QtQ_minus_I": orth}), flush=True)


if __name__ == "__main__":
    main()
