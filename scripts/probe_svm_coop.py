#!/usr/bin/env python3
"""Device SMO per-step time at n = 20k / 40k RBF (the speed test's data) for the one-CU
kernel and the cooperative kernel over 2-16 CUs (HARP_SVM_COOP_NB)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from harp_amd.models.svm import BinarySVM, kernel_matrix


def data(n, d, seed, spread):
    g = torch.Generator().manual_seed(seed)
    c = torch.randn(2, d, generator=g) * spread
    y = torch.randint(0, 2, (n,), generator=g)
    return (c[y] + torch.randn(n, d, generator=g)).double(), y


def main():
    dev = torch.device("cuda:0")
    for n in (20000, 40000):
        X, y = data(n, 16, 3, 0.25)
        Xg, yg = X.to(dev), y.to(dev)
        K = kernel_matrix(Xg, Xg, "rbf", 4.0)
        for nb in (0, 2, 4, 8, 16):
            if (nb == 0 and n > 32768) or (nb and n > 4096 * nb):
                continue
            os.environ["HARP_SVM_COOP_NB"] = str(nb)
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                m = BinarySVM(C=1.0, kernel="rbf", sigma=4.0).fit(Xg, yg, K)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t = min(ts)
            print(json.dumps({"n": n, "cus": nb or 1, "kernel": "coop" if nb else "one-cu", "steps": m.n_iterations,
                              "s": round(t, 4), "us_per_step": round(t / m.n_iterations * 1e6, 2),
                              "objective": m.dual_objective()}), flush=True)


if __name__ == "__main__":
    main()
