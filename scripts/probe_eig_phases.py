"""Phase split of the fused one-XCD reduction (workgroup 0, thread 0 cycle sums per phase:
w + column update, Householder vector, trailing pass, arrival) at several n."""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
from harp_amd.ops import _lib  # noqa: E402
from harp_amd.ops import eig as EIG  # noqa: E402

k = _lib.kernels()
k.harp_eig_fused_stamps.argtypes = [ctypes.c_void_p]
k.harp_eig_fused_stamps.restype = None
for n in [int(a) for a in sys.argv[1:]] or [500, 1000, 1536]:
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.rand(20 * n, n, generator=g, device="cuda", dtype=torch.float64)
    Xc = X - X.mean(0)
    C = Xc.t() @ Xc
    sd = torch.sqrt(torch.diagonal(C))
    C = (C / torch.outer(sd, sd)).contiguous()
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    EIG.eigvalsh(C, native=True)
    torch.cuda.synchronize()
    k.harp_eig_fused_stamps(st.data_ptr())
    t0 = time.perf_counter()
    EIG.eigvalsh(C, native=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    k.harp_eig_fused_stamps(None)
    ph = st.tolist()
    tot = max(sum(ph), 1)
    names = ["w+column", "householder", "pass", "arrival"]
    print(f"n={n}: eigvalsh {dt * 1e3:.2f} ms; cycles/column " +
          ", ".join(f"{nm} {v / (n - 2):.0f} ({100 * v / tot:.0f}%)" for nm, v in zip(names, ph)), flush=True)
