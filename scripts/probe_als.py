#!/usr/bin/env python3
"""ALS kernel split: the fused build + in-LDS Cholesky solve vs the build alone (A / rhs
mode) on the bench shape (138k x 27k, 2e7 implicit ratings, f = 64), one 131,072-row block.
python scripts/probe_als.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from harp_amd.ops import als as OA

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    users, items, nnz, f = 138000, 27000, 20_000_000, 64
    rows = torch.sort(torch.randint(0, users, (nnz,), device=dev, generator=g)).values
    cols = (torch.rand(nnz, device=dev, generator=g) ** 2 * items).long().clamp_max(items - 1)
    vals = torch.randint(1, 6, (nnz,), device=dev, generator=g).float()
    F = torch.randn(items, f, device=dev, generator=g) * 0.1
    crow = torch.searchsorted(rows, torch.arange(users + 1, dtype=rows.dtype, device=dev)).contiguous()
    G = F.t() @ F
    m = 1 << 17
    X = torch.empty(m, f, device=dev)
    info = torch.empty(m, dtype=torch.int32, device=dev)
    A = torch.empty(m, f, f, device=dev)
    rhs = torch.empty(m, f, device=dev)

    def t(fn, reps=3):
        fn()
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / reps

    out = {"rows": m, "f": f}
    out["fused_solve_ms"] = t(lambda: OA.normal_equations(crow, cols, vals, F, G, True, 1.0, 0.1, False, None, None, 0,
                                                          X=X, info=info))
    from harp_amd.ops import _lib
    _lib.register({"harp_als_set_build_dma": [_lib.c_int]})
    lib = _lib.kernels()
    ref = {}
    for dma in (0, 1):
        lib.harp_als_set_build_dma(dma)
        out[f"build_only_dma{dma}_ms"] = t(lambda: OA.normal_equations(crow, cols, vals, F, G, True, 1.0, 0.1, False,
                                                                       A, rhs, 0))
        ref[dma] = (A[:1000].clone(), rhs[:1000].clone())
    out["dma_max_abs_diff_A"] = float((ref[0][0] - ref[1][0]).abs().max())
    out["dma_max_abs_diff_rhs"] = float((ref[0][1] - ref[1][1]).abs().max())
    out["ratings_in_block"] = int(crow[m] - crow[0])
    OA.normal_equations(crow, cols, vals, F, G, True, 1.0, 0.1, False, A, rhs, 0)
    for v in (0, 1):
        out[f"wave_solve_v{v}_ms"] = t(lambda: OA.chol_solve(A, rhs, X, info, variant=v))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
