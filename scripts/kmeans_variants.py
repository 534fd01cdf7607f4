"""Interleaved A/B timing of the K-means assign kernel variants (one process, n rounds).

python scripts/kmeans_variants.py [--n 1e8] [--k 10000] [--d 100] [--rounds 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from harp_amd.ops import kmeans as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--k", type=int, default=10000)
    ap.add_argument("--d", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--acc", default="none,atomic,bucket")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = int(a.n)
    dev = torch.device("cuda", 0)
    X = K.generate_points(n, a.d, 0, 1000, seed=1, device=dev)
    c = torch.rand(a.k, a.d, device=dev) * 1000
    op = K.prepare(c, X.shape[1])
    sums = torch.zeros((K.padded_k(a.k), X.shape[1]), dtype=torch.float32, device=dev)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    variants = [int(v) for v in a.variants.split(",")]
    res = {}
    for _ in range(a.rounds):
        for v in variants:
            for acc in a.acc.split(","):
                kw = dict(sums=None if acc == "none" else sums, labels=lab, want_objective=False, variant=v,
                          accumulate=acc if acc != "none" else "bucket")
                K.assign(X, op, **kw)
                s, e = torch.cuda.Event(True), torch.cuda.Event(True)
                s.record()
                K.assign(X, op, **kw)
                e.record()
                e.synchronize()
                res.setdefault(f"v{v}+{acc}", []).append(s.elapsed_time(e))
    flops = 2.0 * n * a.k * a.d
    out = {k: {"ms_min": min(v), "ms_med": sorted(v)[len(v) // 2], "tflops": flops / (min(v) / 1e3) / 1e12}
           for k, v in res.items()}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
