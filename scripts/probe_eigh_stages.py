"""Stage times of ops.eig.eigh at n = 1000 (reduction, D&C tridiagonal eigenvectors,
compact-WY back-transform), CUDA events, median of 10 after 3 warm-ups."""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from harp_amd.ops import eig as E  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
X = torch.randn(4 * n, n, generator=g, dtype=torch.float64)
C = (X.t() @ X / (4 * n)).to(dev)
k = E._lib.kernels()
stages = {"sytrd": [], "dc": [], "back": [], "total": []}
for it in range(13):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    nb = int(k.harp_eig_workgroups(n, E.NB_DEFAULT))
    A = C.contiguous().clone()
    ws = torch.zeros(int(k.harp_eig_ws_ints()), dtype=torch.int32, device=dev)
    wsd = torch.zeros(3 * n + 4, dtype=torch.float64, device=dev)
    d = torch.empty(n, dtype=torch.float64, device=dev)
    e = torch.zeros(n, dtype=torch.float64, device=dev)
    Vt = torch.zeros((n, n), dtype=torch.float64, device=dev)
    tau = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ev[0].record()
    E._lib.check(k.harp_sytrd_fused(A.data_ptr(), n, n, d.data_ptr(), e.data_ptr(), Vt.data_ptr(), tau.data_ptr(), nb,
                                    ws.data_ptr(), wsd.data_ptr(), E._lib.stream_ptr(dev)), "sytrd")
    ev[1].record()
    lam, Z = E.eigh_tridiag(d, e[:n - 1])
    ev[2].record()
    V = E.back_transform(Vt, tau, Z)
    ev[3].record()
    torch.cuda.synchronize()
    if it >= 3:
        stages["sytrd"].append(ev[0].elapsed_time(ev[1]))
        stages["dc"].append(ev[1].elapsed_time(ev[2]))
        stages["back"].append(ev[2].elapsed_time(ev[3]))
        stages["total"].append(ev[0].elapsed_time(ev[3]))
print({k: round(statistics.median(v), 3) for k, v in stages.items()}, "ms")
lam_ref = torch.linalg.eigvalsh(C)
print("eigenvalue err", float((lam - lam_ref).abs().max()), "orth", float((V.t() @ V - torch.eye(n, device=dev, dtype=torch.float64)).abs().max()))
