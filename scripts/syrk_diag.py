#!/usr/bin/env python3
"""SYRK bottleneck split (csrc/syrk.hip harp_syrk_diag): time the default 256-tile kernel
with (0) everything, (1) no global loads after the first stage, (2) no MFMA, (3) loads +
barriers only, (4) L2-hot loads (every stage re-reads the first), on the PCA shape. python scripts/syrk_diag.py [--n 1e8] [--d 1000]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--d", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--modes", default="0,1,2,3,4", help="DIAG modes of csrc/syrk.hip (0-5)")
    a = ap.parse_args()
    import torch

    from harp_amd.ops import _lib
    from harp_amd.ops import linalg as LA

    _lib.register({"harp_syrk_diag": [_lib.c_void_p, _lib.c_long, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_int,
                                      _lib.c_int, _lib.c_int, _lib.c_void_p]})
    fm = LA.FeatureMajor.uniform(int(a.n), a.d, 0.0, 1.0, seed=11, device="cuda")
    G = torch.zeros((fm.d_pad, fm.d_pad), dtype=torch.float32, device="cuda")
    lib = _lib.kernels()
    out = {"n": int(a.n), "d": a.d}
    for mode in [int(m) for m in a.modes.split(",")]:
        def run():
            _lib.check(lib.harp_syrk_diag(fm.XT.data_ptr(), fm.ld, fm.ld, fm.d_pad, G.data_ptr(), G.stride(0),
                                          a.splits, mode, _lib.stream_ptr(G.device)), "syrk_diag")
        run()
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(a.reps):
            run()
        e.record()
        e.synchronize()
        out[f"mode{mode}_s"] = s.elapsed_time(e) / 1e3 / a.reps
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
