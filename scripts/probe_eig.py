#!/usr/bin/env python3
"""Symmetric eigensolvers for the PCA pass's 1000 x 1000 fp64 correlation matrix on one
MI355X: torch (rocSOLVER syevd) vs rocSOLVER's Jacobi (syevj) and divide-and-conquer Jacobi
(syevdj) called directly, eigenvalues only and with vectors. Times after warm-up."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

EV_ORIG, EV_NONE = 211, 213
FILL_UPPER = 121
ESORT_ASC = 252


def main():
    dev = torch.device("cuda:0")
    n = int(os.environ.get("N", 1000))
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.rand(20 * n, n, generator=g, device=dev, dtype=torch.float64)
    Xc = X - X.mean(0)
    C = (Xc.t() @ Xc)
    sd = torch.sqrt(torch.diagonal(C))
    C = (C / torch.outer(sd, sd)).contiguous()
    ref = torch.linalg.eigvalsh(C)
    rb = ctypes.CDLL("librocblas.so")
    rs = ctypes.CDLL("librocsolver.so")
    h = ctypes.c_void_p()
    assert rb.rocblas_create_handle(ctypes.byref(h)) == 0
    rb.rocblas_set_stream(h, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    W = torch.empty(n, dtype=torch.float64, device=dev)
    E = torch.empty(n, dtype=torch.float64, device=dev)
    resid = torch.empty(1, dtype=torch.float64, device=dev)
    sweeps = torch.zeros(1, dtype=torch.int32, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run(name, fn, reps=5):
        A = C.clone()
        fn(A)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            A = C.clone()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            w = fn(A)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        err = float((torch.sort(w)[0] - ref).abs().max())
        print(json.dumps({"solver": name, "n": n, "ms": round(min(ts) * 1e3, 3), "max_abs_err": err}), flush=True)

    run("torch.eigvalsh", lambda A: torch.linalg.eigvalsh(A))
    run("torch.eigh", lambda A: torch.linalg.eigh(A)[0])

    def syevd(ev):
        def f(A):
            st = rs.rocsolver_dsyevd(h, ev, FILL_UPPER, n, p(A), n, p(W), p(E), p(info))
            assert st == 0, st
            return W
        return f

    def syevj(ev):
        def f(A):
            st = rs.rocsolver_dsyevj(h, ESORT_ASC, ev, FILL_UPPER, n, p(A), n, ctypes.c_double(0.0), p(resid), 100,
                                     p(sweeps), p(W), p(info))
            assert st == 0, st
            return W
        return f

    def syevdj(ev):
        def f(A):
            st = rs.rocsolver_dsyevdj(h, ev, FILL_UPPER, n, p(A), n, p(W), p(info))
            assert st == 0, st
            return W
        return f

    for name, ev in (("none", EV_NONE), ("vectors", EV_ORIG)):
        run(f"rocsolver_dsyevd/{name}", syevd(ev))
        run(f"rocsolver_dsyevj/{name}", syevj(ev))
        run(f"rocsolver_dsyevdj/{name}", syevdj(ev))
    print(json.dumps({"jacobi_sweeps": int(sweeps.item())}))


if __name__ == "__main__":
    main()
