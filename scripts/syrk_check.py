#!/usr/bin/env python3
"""SYRK variant agreement: every variant's upper triangle vs an fp32 torch reference of the
same bf16 operands. python scripts/syrk_check.py [--n 96000] [--d 1000] [--variants 0,1]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=96000)
    ap.add_argument("--d", type=int, default=1000)
    ap.add_argument("--variants", default="0")
    a = ap.parse_args()
    import torch

    from harp_amd.ops import linalg as LA

    torch.manual_seed(0)
    X = torch.randn(a.n, a.d, device="cuda").to(torch.bfloat16)
    fm = LA.FeatureMajor.from_rows(X)
    ref = X.float().t() @ X.float()
    out = {"n": a.n, "d": a.d}
    for v in [int(x) for x in a.variants.split(",")]:
        G = LA.symmetrize_upper(LA.syrk_t(fm, variant=v))[: a.d, : a.d]
        err = (G - ref).abs().max().item() / ref.abs().max().item()
        out[f"v{v}_relerr"] = err
    print(json.dumps(out), flush=True)
    assert all(v < 1e-4 for k, v in out.items() if k.endswith("relerr")), out


if __name__ == "__main__":
    main()
