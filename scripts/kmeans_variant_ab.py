#!/usr/bin/env python3
"""A/B of assign-kernel variants in one process (N = 1e8, d = 100, K = 1e4): time per
assign and label agreement with the first variant. python scripts/kmeans_variant_ab.py [d=100] 14 13 14"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from harp_amd.ops import kmeans as K

    args = [a for a in sys.argv[1:] if not a.startswith("d=")]
    variants = [int(v) for v in args] or [14, 13, 14]
    d = int(next((a[2:] for a in sys.argv[1:] if a.startswith("d=")), 100))
    n, k = 100_000_000, 10_000
    X = K.generate_points(n, d, seed=1, device="cuda")
    c = torch.rand(k, d, device="cuda") * 1000
    op = K.prepare(c, X.shape[1])
    ref = None
    out = []
    for v in variants:
        labels = torch.empty(n, dtype=torch.int32, device="cuda")
        _, obj = K.assign(X, op, labels=labels, want_objective=True, variant=v)
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(5):
            K.assign(X, op, labels=labels, want_objective=False, variant=v)
        e.record()
        e.synchronize()
        if ref is None:
            ref = labels.clone()
        out.append({"variant": v, "ms": round(s.elapsed_time(e) / 5, 3), "objective": float(obj),
                    "label_agreement": float((labels == ref).float().mean())})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
