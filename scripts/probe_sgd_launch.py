#!/usr/bin/env python3
"""Where does an XCD sub-step launch's time go at the 8-GPU rank share? Times one slice
pass (8 sub-step launches of mf_sgd_xcd_kernel) over a Netflix-share slice (60k users x
1,110 items, 785k ratings) while the trained fraction of every cell varies from 0 (blocks
exit at once: the launch floor) to 1, for a few launch geometries."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from harp_amd.models.sgd_mf import _Buckets, synthetic_ratings
from harp_amd.ops import mf as MF


def main():
    dev = torch.device("cuda:0")
    nu, ni, n = 60000, 1110, 785000
    u, i, v = synthetic_ratings(nu, ni, n, seed=7, skew=2.0)
    b = _Buckets(u, i, v, torch.zeros(ni, dtype=torch.int64), torch.arange(ni), 1, dev, cells=(nu, ni))
    rows, cols, vals = b.rows, b.cols, b.vals
    off, host = b.cell_off[0].contiguous(), b.cell_off_host[0]
    W = torch.rand(nu, 128, device=dev) * 0.1
    H = torch.rand(ni, 128, device=dev) * 0.1
    out = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for bpx in (128, 32):
        for var in (0, 2):
            for f in (0.0, 0.02, 0.125, 0.5, 1.0):
                win = None
                if f < 1.0:
                    w = MF.cell_windows(host, f, 0)
                    if f == 0.0:
                        w = ([0] * 64, [0] * 64)
                    win = w
                for _ in range(5):
                    MF.sgd_update_blocked(rows, cols, vals, off, W, H, 1e-4, 0.05, chunk=8, blocks_per_xcd=bpx,
                                          variant=var, window=win, host_off=host)
                torch.cuda.synchronize()
                reps = 50
                e0.record()
                for _ in range(reps):
                    MF.sgd_update_blocked(rows, cols, vals, off, W, H, 1e-4, 0.05, chunk=8, blocks_per_xcd=bpx,
                                          variant=var, window=win, host_off=host)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1000 / reps / 8
                rec = {"blocks_per_xcd": bpx, "variant": var, "fraction": f, "us_per_substep": round(us, 2)}
                out.append(rec)
                print(json.dumps(rec), flush=True)
    # reference: a trivial 1024-block kernel
    x = torch.zeros(1024 * 256, device=dev)
    for _ in range(10):
        x.add_(1.0)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(400):
        x.add_(1.0)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"trivial_kernel_us": round(e0.elapsed_time(e1) * 1000 / 400, 2)}))


if __name__ == "__main__":
    main()
