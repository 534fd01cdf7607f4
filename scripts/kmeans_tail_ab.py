#!/usr/bin/env python3
"""A/B of the assign kernel's swept rows in one process: K = 1e4 rounded to 32 (10,016, the
default) vs the full 128-row padding (10,112). python scripts/kmeans_tail_ab.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from harp_amd.ops import kmeans as K

    n, d, k = 100_000_000, 100, 10_000
    X = K.generate_points(n, d, seed=1, device="cuda")
    c = torch.rand(k, d, device="cuda") * 1000
    op = K.prepare(c, X.shape[1])
    labels = torch.empty(n, dtype=torch.int32, device="cuda")
    default = K.swept_k
    out = {}
    for name, fn in (("k32", default), ("k128", lambda o: o.Cm2.shape[0]), ("k32_again", default)):
        K.swept_k = fn
        K.assign(X, op, labels=labels, want_objective=False)
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(5):
            K.assign(X, op, labels=labels, want_objective=False)
        e.record()
        e.synchronize()
        out[name + "_ms"] = round(s.elapsed_time(e) / 5, 3)
        out[name + "_labels_max"] = int(labels.max().item())
    K.swept_k = default
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
