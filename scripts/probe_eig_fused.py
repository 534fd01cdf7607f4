"""A/B of the one-XCD eigensolver reductions (HARP_EIG_VARIANT fused vs twopass) on the PCA
pass's 1000 x 1000 correlation matrix and random symmetric matrices; rocSOLVER for scale."""
import sys
import time

import torch

sys.path.insert(0, ".")
from harp_amd.ops import eig as EIG  # noqa: E402


def corr(n, N=20000):
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.rand(N, n, generator=g, device="cuda", dtype=torch.float64)
    Xc = X - X.mean(0)
    C = Xc.t() @ Xc
    sd = torch.sqrt(torch.diagonal(C))
    return C / torch.outer(sd, sd)


def timed(fn, C, reps=10):
    fn(C)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn(C)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for n in (1000, 2048, 500):
    C = corr(n)
    ref = torch.linalg.eigvalsh(C)
    row = {"n": n, "rocsolver_ms": round(timed(torch.linalg.eigvalsh, C), 3)}
    for v, ku in (("twopass", 8), ("fused", 8)):
        EIG.VARIANT, EIG.KU = v, ku
        w = EIG.eigvalsh(C)
        tag = v
        row[tag + "_ms"] = round(timed(EIG.eigvalsh, C), 3)
        row[tag + "_err"] = float((w - ref).abs().max())
    print(row, flush=True)
