"""eigh of the PCA pass's 1000 x 1000 correlation matrix, repeated (for rocprofv3 kernel stats)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from harp_amd.ops import eig as EIG  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.rand(20 * n, n, generator=g, device="cuda", dtype=torch.float64)
Xc = X - X.mean(0)
C = Xc.t() @ Xc
sd = torch.sqrt(torch.diagonal(C))
C = C / torch.outer(sd, sd)
for name, fn in (("harp eigh", EIG.eigh), ("rocSOLVER eigh", torch.linalg.eigh), ("harp eigvalsh", EIG.eigvalsh)):
    fn(C)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        fn(C)
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms", flush=True)
