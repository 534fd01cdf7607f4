#!/usr/bin/env python3
"""Where to run the PCA finalize (eigvalsh of the d x d correlation matrix): GPU fp64 /
fp32 vs CPU fp64, d = 1000. python scripts/probe_eig.py"""
import json
import time

import torch


def timeit(fn, reps=5, cuda=True):
    fn()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    if cuda:
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    d = 1000
    g = torch.Generator().manual_seed(0)
    A = torch.randn(4 * d, d, generator=g, dtype=torch.float64)
    C = (A.t() @ A) / (4 * d)
    out = {"d": d, "torch_threads": torch.get_num_threads()}
    Cg = C.cuda()
    out["gpu_fp64_eigvalsh_ms"] = timeit(lambda: torch.linalg.eigvalsh(Cg))
    out["gpu_fp32_eigvalsh_ms"] = timeit(lambda: torch.linalg.eigvalsh(Cg.float()))
    out["cpu_fp64_eigvalsh_ms"] = timeit(lambda: torch.linalg.eigvalsh(C), cuda=False)
    out["gpu_to_cpu_fp64_eigvalsh_ms"] = timeit(lambda: torch.linalg.eigvalsh(Cg.cpu()))
    out["gpu_fp64_eigh_ms"] = timeit(lambda: torch.linalg.eigh(Cg))
    out["cpu_fp64_eigh_ms"] = timeit(lambda: torch.linalg.eigh(C), cuda=False)
    for lib in ("magma", "cusolver"):
        try:
            torch.backends.cuda.preferred_linalg_library(lib)
            out[f"gpu_fp64_eigvalsh_{lib}_ms"] = timeit(lambda: torch.linalg.eigvalsh(Cg))
        except Exception as e:  # noqa: BLE001
            out[f"gpu_fp64_eigvalsh_{lib}_ms"] = f"{type(e).__name__}: {e}"[:120]
    torch.backends.cuda.preferred_linalg_library("default")
    ref = torch.linalg.eigvalsh(C)
    out["fp32_max_rel_err"] = float(((torch.linalg.eigvalsh(Cg.float()).double().cpu() - ref).abs() / ref.abs().max()).max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
