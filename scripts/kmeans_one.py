"""Run ONE K-means assign variant a few times (for rocprofv3 --pmc runs).

python scripts/kmeans_one.py --variant 6 [--n 1e8 --k 10000 --d 100 --reps 2]
"""
import argparse
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
    ap.add_argument("--variant", type=int, default=K.DEFAULT_VARIANT)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = int(a.n)
    X = K.generate_points(n, a.d, 0, 1000, seed=1, device=dev)
    c = torch.rand(a.k, a.d, device=dev) * 1000
    op = K.prepare(c, X.shape[1])
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(a.reps):
        K.assign(X, op, labels=lab, want_objective=False, variant=a.variant)
    torch.cuda.synchronize()
    print("ok", a.variant)


if __name__ == "__main__":
    main()
