#!/usr/bin/env python3
"""One-XCD eigensolver time vs workgroup count (HARP_EIG_NB) and matrix size."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from harp_amd.ops import eig as EIG


def main():
    dev = torch.device("cuda:0")
    for n in (256, 1000, 2048):
        g = torch.Generator(device=dev).manual_seed(0)
        M = torch.randn(n, n, generator=g, device=dev, dtype=torch.float64)
        C = (M + M.t()) / 2
        for nb in (8, 16, 32):
            os.environ["HARP_EIG_NB"] = str(nb)
            EIG.eigvalsh(C)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                EIG.eigvalsh(C)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / 5
            print(json.dumps({"n": n, "nb": nb, "ms": round(t * 1e3, 3), "us_per_column": round(t / n * 1e6, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()


def stamps():
    dev = torch.device("cuda:0")
    n = 1000
    g = torch.Generator(device=dev).manual_seed(0)
    M = torch.randn(n, n, generator=g, device=dev, dtype=torch.float64)
    C = (M + M.t()) / 2
    os.environ["HARP_EIG_NB"] = "32"
    st = torch.zeros(9, dtype=torch.int64, device=dev)
    EIG.eigvalsh(C, st)
    torch.cuda.synchronize()
    cyc = st.tolist()
    names = ["v", "p_rest", "arrive1", "w", "update", "arrive2", "p_loads", "p_sync1", "p_reduce"]
    tot = sum(cyc)
    print(json.dumps({"n": n, "stamp_cycles": dict(zip(names, cyc)),
                      "share": {k: round(c / tot, 3) for k, c in zip(names, cyc)}}))


if os.environ.get("STAMPS"):
    stamps()
