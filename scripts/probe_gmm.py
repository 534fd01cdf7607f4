#!/usr/bin/env python3
"""EM-GMM kernel timings at N = 1e6, d = 32, K = 64 (full covariance): E-step and
statistics separately, HIP events, 20 repetitions each."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from harp_amd.ops import gmm as GM


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    n, d, K = 1_000_000, int(os.environ.get("D", 32)), int(os.environ.get("K", 64))
    mu = torch.randn(K, d, generator=g, dtype=torch.float64) * 3
    A = torch.randn(K, d, d, generator=g, dtype=torch.float64) * 0.3
    cov = A @ A.transpose(1, 2) + torch.eye(d, dtype=torch.float64)
    w = torch.full((K,), 1.0 / K, dtype=torch.float64)
    X = (mu[torch.randint(0, K, (n,), generator=g)] + torch.randn(n, d, generator=g, dtype=torch.float64))
    X, w, mu, cov = X.to(dev), w.to(dev), mu.to(dev), cov.to(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    R, _ = GM.estep(X, w, mu, cov, "full")
    GM.stats(X, R, "full")
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("estep", lambda: GM.estep(X, w, mu, cov, "full")), ("stats", lambda: GM.stats(X, R, "full"))):
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_ms"] = round(e0.elapsed_time(e1) / 20, 3)
    res.update({"n": n, "d": d, "K": K})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
