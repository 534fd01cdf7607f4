#!/usr/bin/env python3
"""Host-side (Python) cost of one MF-SGD slice step: cProfile over epochs of the 8-GPU
per-rank share (12.5M Netflix-shape ratings) run on one GPU with 16 slices, i.e. the 16
slice steps an 8-rank, 2-slice rotation takes per epoch.

python scripts/sgd_host_profile.py [--slices 16] [--epochs 10]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ratings", type=int, default=12560063)
    ap.add_argument("--slices", type=int, default=16)
    ap.add_argument("--epochs", type=int, default=10)
    a = ap.parse_args()
    import torch

    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    dev = torch.device("cuda")
    u, i, v = synthetic_ratings(480189, 17770, a.ratings, seed=7, device=dev)
    cfg = SGDConfig(rank=128, epochs=10**6, test_every=0, xcd_blocks=True, num_slices=a.slices)
    m = SGDCollectiveMapper(Communicator(None, dev), cfg, 480189, 17770, (u, i, v), None)
    m.init_model(KeyValReader([]))
    for ep in range(3):
        m.train_epoch(ep)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = []
    pr = cProfile.Profile()
    for ep in range(a.epochs):
        h0 = time.perf_counter()
        pr.enable()
        m.train_epoch(3 + ep)
        pr.disable()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.epochs
    print(f"epoch wall {wall * 1e3:.3f} ms, host issue {sum(host) / len(host) * 1e3:.3f} ms "
          f"({a.slices} slice steps: {sum(host) / len(host) / a.slices * 1e6:.1f} us host per step)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
