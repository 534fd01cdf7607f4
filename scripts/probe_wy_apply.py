"""Forms of the eigh back-transform X = Z - M (V^T Z) (ops/eig.py apply_wy) at n = 1000 with
Z handed over as Z^T contiguous (what eigh_tridiag returns): CUDA-event medians per form.
python scripts/probe_wy_apply.py [n]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
m = n - 2
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
Zt = torch.randn(n, n, generator=g, device=dev, dtype=torch.float64)
# V^T and M^T with the layouts ops.eig.wy_factor produces (its triangular solve decides M^T's)
from harp_amd.ops import eig as E  # noqa: E402

Vt = torch.triu(torch.randn(n, n, generator=g, device=dev, dtype=torch.float64), 1) / n ** 0.5
tau = torch.full((n,), 1.0, device=dev, dtype=torch.float64)
Vm, Mt = E.wy_factor(Vt, tau)
Mtc = Mt.contiguous()
Vc = Vm.t().contiguous()  # V (n x m) row-major
print("Mt strides", Mt.stride(), "Vm strides", Vm.stride(), file=sys.stderr)


def a():  # current: Z as a transposed view
    Z = Zt.t()
    return torch.addmm(Z, Mt.t(), Vm @ Z, alpha=-1)


def b():  # V^T Z formed as (Z^T V)^T
    Z = Zt.t()
    return torch.addmm(Z, Mt.t(), (Zt @ Vm.t()).t(), alpha=-1)


def c():  # X^T = Z^T - (Z^T V) M^T, all row-major, X as a view
    return torch.addmm(Zt, Zt @ Vm.t(), Mt, alpha=-1).t()


def d():  # c in place on a copy of Z^T (the copy stands in for the fresh buffer)
    W = Zt.clone()
    return W.addmm_(Zt @ Vm.t(), Mt, alpha=-1).t()


def e():  # d with M^T made row-major (off the critical path, on wy_factor's stream)
    W = Zt.clone()
    return W.addmm_(Zt @ Vm.t(), Mtc, alpha=-1).t()


def g():  # e with V row-major as well
    W = Zt.clone()
    return W.addmm_(Zt @ Vc, Mtc, alpha=-1).t()


def f():  # a with M^T row-major
    Z = Zt.t()
    return torch.addmm(Z, Mtc.t(), Vm @ Z, alpha=-1)


ref = a()
rec = {"n": n}
for name, fn in (("a_view", a), ("b_zt_v", b), ("c_rowmajor", c), ("d_inplace_incl_clone", d),
                 ("e_inplace_mt_rowmajor_incl_clone", e), ("f_view_mt_rowmajor", f),
                 ("g_inplace_v_mt_rowmajor_incl_clone", g)):
    out = fn()
    err = float((out - ref).abs().max() / ref.abs().max())
    for _ in range(3):
        fn()
    ts = []
    for _ in range(15):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    rec[name] = {"ms": round(ts[len(ts) // 2], 4), "max_diff": err}
W = Zt.clone()
for _ in range(3):
    torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    W.copy_(Zt)
e.record()
e.synchronize()
rec["clone_ms"] = round(s.elapsed_time(e) / 10, 4)
print(json.dumps(rec))
