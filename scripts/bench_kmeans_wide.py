"""K-means assign at wide rows: N = 1e7, K = 1e3, d = 1000 (VERDICT r3 target: >= 1.2 PF
useful, 2 N K d flops). Prints ms per assign and the useful rate."""
import sys
import time

import torch

sys.path.insert(0, ".")
from harp_amd.ops import kmeans as K  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
Kc = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
d = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
X = K.generate_points(N, d, 0.0, 1000.0, seed=1, device="cuda")
c = torch.rand(Kc, d, device="cuda") * 1000
op = K.prepare(c, X.shape[1])
lab = torch.empty(N, dtype=torch.int32, device="cuda")
variants = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
for var, mode in [(v, "assign") for v in variants] + [(variants[0], "assign+sums")]:
    K.WIDE_VARIANT = var
    sums = torch.zeros((K.padded_k(Kc), X.shape[1]), dtype=torch.float32, device="cuda") if mode != "assign" else None
    K.assign(X, op, sums=sums, labels=lab)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        if sums is not None:
            sums.zero_()
        K.assign(X, op, sums=sums, labels=lab)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"variant {var} {mode}: N={N} K={Kc} d={d} dp={X.shape[1]}: {dt * 1e3:.2f} ms, {2.0 * N * Kc * d / dt / 1e12:.0f} TFLOP/s "
          "useful", flush=True)
