#!/usr/bin/env python3
"""Does replaying an MF-SGD epoch from a HIP graph shorten the per-launch floor at small
per-rank shares? One GPU, the 8-GPU rank share (12.56M Netflix-shape ratings, 16 slice
steps = 128 XCD sub-step launches per epoch): eager epochs vs graph replays.
python scripts/probe_sgd_graph.py [--ratings 12560063] [--slices 16]"""
import argparse
import contextlib
import json
import os
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

    dev = torch.device("cuda", 0)
    comm = Communicator(None, dev)
    u, i, v = synthetic_ratings(480189, 17770, a.ratings, seed=7, device=dev)
    cfg = SGDConfig(rank=128, epochs=100, test_every=0, xcd_blocks=True, num_slices=a.slices)
    m = SGDCollectiveMapper(comm, cfg, 480189, 17770, (u, i, v), None)
    m.init_model(KeyValReader([]))

    class _NoTimer:
        @contextlib.contextmanager
        def phase(self, name):
            yield

    m.metrics.timer = _NoTimer()
    out = {"ratings": a.ratings, "slices": a.slices}
    for ep in range(2):
        m.train_epoch(ep)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for ep in range(a.epochs):
        m.train_epoch(2 + ep)
    torch.cuda.synchronize()
    out["eager_ms_per_epoch"] = (time.perf_counter() - t0) / a.epochs * 1e3
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m.train_epoch(50)  # warm the allocator on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.train_epoch(51)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.epochs):
        g.replay()
    torch.cuda.synchronize()
    out["graph_ms_per_epoch"] = (time.perf_counter() - t0) / a.epochs * 1e3
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
