#!/usr/bin/env python3
"""A/B of the MF-SGD XCD kernel's triple staging: register loads between barriers (0) vs
LDS-DMA double buffer (1), alternating in one process on one model.
python scripts/probe_sgd_stage.py [--ratings 100480507] [--slices 2]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ratings", type=int, default=100480507)
    ap.add_argument("--slices", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=5)
    a = ap.parse_args()
    import torch

    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings
    from harp_amd.ops import _lib
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    _lib.register({"harp_mf_set_stage_dma": [_lib.c_int]})
    lib = _lib.kernels()
    dev = torch.device("cuda", 0)
    u, i, v = synthetic_ratings(480189, 17770, a.ratings, seed=7, device=dev)
    cfg = SGDConfig(rank=128, epochs=1000, test_every=0, xcd_blocks=True, num_slices=a.slices)
    m = SGDCollectiveMapper(Communicator(None, dev), cfg, 480189, 17770, (u, i, v), None)
    m.init_model(KeyValReader([]))
    out = {"ratings": a.ratings, "slices": a.slices}
    ep = 0
    for rep in range(2):
        for dma in (0, 1):
            lib.harp_mf_set_stage_dma(dma)
            m.train_epoch(ep)
            ep += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.epochs):
                m.train_epoch(ep)
                ep += 1
            torch.cuda.synchronize()
            out[f"dma{dma}_run{rep}_ms"] = round((time.perf_counter() - t0) / a.epochs * 1e3, 3)
    out["train_rmse_after"] = m._eval_ring(ep - 1)[0]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
