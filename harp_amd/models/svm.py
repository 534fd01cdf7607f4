"""Support vector machines: SMO (C-SVC), one-vs-one multiclass, cascade SVM.

Reference: ml/daal/.../daal_svm/{multidensebatch, multicsrbatch} (DAAL svm ``boser``
SMO with ``C``, ``accuracyThreshold``, ``tau``, ``maxIterations``, linear / RBF kernel,
wrapped in ``multi_class_classifier`` one-against-one) and
contrib/src/main/java/edu/iu/svm/SVMMapper.java:100-222 (iterative cascade: every
mapper trains libsvm on its local data plus the current global SV set; the SVs are
serialised as libsvm text lines in ONE ``HarpString`` partition and allreduced with the
string-concatenating ``HarpStringPlus`` combiner, then de-duplicated in a HashSet).

MI355X design: SMO with second-order working-set selection (Fan, Chen & Lin 2005); the
kernel matrix of the training block is one GEMM (+ fused RBF epilogue) kept resident
(a 60k-row fp64 Gram is 29 GB — nothing on a 288 GB device). On the GPU the whole solve
runs in ``csrc/svm.hip`` (:func:`smo_device`), no host round trip per SMO step: a large
machine is split over 16 CUs of one XCD (gradient, alphas and its slice of kernel row i
in registers, two cross-workgroup reductions per step through the XCD's L2; up to 8
machines at once, one per XCD), many small ones run one 1024-thread workgroup each, and
the K(K-1)/2 one-vs-one machines of a multiclass problem train concurrently in ONE
launch over the shared Gram matrix. The PyTorch loop below is the CPU path and the oracle. The
cascade keeps the reference's wire format: SV lines travel through the generic
(variable-length Writable) allreduce path.
"""
from __future__ import annotations

import os
import warnings
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..core.combiner import PartitionCombiner, PartitionStatus
from ..ops import _lib
from ..core.table import Table
from ..core.writable import DataInput, DataOutput, Writable
from ..parallel import collectives as CL
from ..parallel.comm import Communicator
from . import kernels as KF


def kernel_matrix(X, Y, kernel: str = "linear", sigma: float = 1.0, k: float = 1.0, b: float = 0.0):
    if kernel == "linear":
        return KF.linear_kernel(X, Y, k, b)
    if kernel == "rbf":
        return KF.rbf_kernel(X, Y, sigma)
    raise ValueError(kernel)


_lib.register({
    "harp_svm_max_rows": [],
    "harp_svm_coop_ws_ints": [],
    "harp_svm_coop_xcd_ints": [],
    "harp_svm_coop_max_rows": [_lib.c_int],
    # K, ldk, ids, moff, nm, max_n, y, kd, a, g, iters, C, eps, tau, max_iter, NB, ident, ws, stream
    "harp_svm_smo_coop": [_lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int,
                          _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_double,
                          _lib.c_double, _lib.c_double, _lib.c_int, _lib.c_int, _lib.c_int, _lib.c_void_p,
                          _lib.c_void_p],
    # K, ldk, ids, moff, nm, max_n, y, kd, a, g, iters, C, eps, tau, max_iter, ident, stream
    "harp_svm_smo": [_lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p,
                     _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_double, _lib.c_double,
                     _lib.c_double, _lib.c_int, _lib.c_int, _lib.c_void_p],
})


# machines of at least COOP_MIN_ROWS rows are split over several CUs of one XCD each (XCD x
# trains machines x, x + 8, ...; csrc/svm.hip smo_coop_kernel) when there are at most
# COOP_MAX_MACHINES of them (more small machines fill the chip better one CU each);
# HARP_SVM_COOP_NB overrides the CU count per machine (0 = off)
COOP_MIN_ROWS = 4096
COOP_MAX_NB = 16
COOP_MAX_MACHINES = 16


def coop_workgroups(max_n: int, machines: int = 1) -> int:
    """CUs per machine for the cooperative kernel (<= 4 elements per thread, <= 16 CUs), or
    0 for the one-CU-per-machine kernel."""
    one_cu_max = int(_lib.kernels().harp_svm_max_rows())
    env = os.environ.get("HARP_SVM_COOP_NB")
    if env is not None:
        try:
            nb = int(env)
        except ValueError:
            nb = -1
        if not 0 <= nb <= COOP_MAX_NB:
            warnings.warn(f"HARP_SVM_COOP_NB={env!r} is outside [0, {COOP_MAX_NB}]: cooperative SMO off")
            nb = 0
    elif max_n < COOP_MIN_ROWS or (machines > COOP_MAX_MACHINES and max_n <= one_cu_max):
        return 0
    else:
        nb = COOP_MAX_NB
    if nb <= 0 or max_n > 4096 * nb:
        return 0
    return nb


def _max_rows() -> int:
    k = _lib.kernels()
    return max(int(k.harp_svm_max_rows()), int(k.harp_svm_coop_max_rows(COOP_MAX_NB)))


def native_smo_ok(K: torch.Tensor, n: int, machines: int = 1) -> bool:
    """The device solver takes fp64 GPU Gram matrices with machines of <= 65536 rows (the
    cooperative kernel at 16 CUs; the one-CU kernel takes <= 32768)."""
    return (K.device.type == "cuda" and K.dtype == torch.float64 and K.dim() == 2 and K.stride(1) == 1
            and _lib.use_native(K) and 0 < n <= _max_rows())


def _smo_coop(K, ids, moff, nm, max_n, y, kd, C, eps, tau, max_iter, ident, nb):
    """All machines over ``nb`` CUs each; None if some XCD could not run its machines
    cooperatively (fewer than nb workgroups there, or a wait gave up)."""
    dev = K.device
    k = _lib.kernels()
    ws = torch.zeros(int(k.harp_svm_coop_ws_ints()), dtype=torch.int32, device=dev)
    a = torch.zeros_like(y)
    g = -torch.ones_like(y)
    iters = torch.zeros(nm, dtype=torch.int32, device=dev)
    st = k.harp_svm_smo_coop(K.data_ptr(), K.stride(0), ids.data_ptr(), moff.data_ptr(), nm, max_n, y.data_ptr(),
                             kd.data_ptr(), a.data_ptr(), g.data_ptr(), iters.data_ptr(), float(C), float(eps),
                             float(tau), int(max_iter), nb, 1 if ident else 0, ws.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(st, "svm_smo_coop")
    w = ws.view(8, int(k.harp_svm_coop_xcd_ints()))[:, :4].tolist()
    bad = [x for x in range(min(nm, 8)) if w[x][0] < nb or w[x][3] != 0]
    if bad:
        warnings.warn(f"cooperative SMO did not run on {nb} CUs of XCDs {bad} (claims / errors "
                      f"{[(w[x][0], w[x][3]) for x in bad]}); using the one-CU kernel")
        return None
    return a, g, iters.tolist()


def smo_device(K: torch.Tensor, machines: Sequence[Tuple[torch.Tensor, torch.Tensor]], C: float, eps: float,
               tau: float, max_iter: int, ident: bool = False) -> Optional[List[Tuple[torch.Tensor, torch.Tensor, int]]]:
    """Train every binary machine ``(idx, y)`` (rows / columns ``idx`` of the fp64 Gram
    ``K``, labels +-1) with the device SMO, all machines in one launch. ``ident``: one
    machine over all of K (idx = 0..n-1, no index indirection). Returns per machine
    (alpha, gradient G = Q alpha - e, SMO steps), or None when no device kernel can take
    the machines (the caller runs the PyTorch loop)."""
    dev = K.device
    idx = [m[0].to(dev, torch.int32) for m in machines]
    ys = [m[1].to(dev, torch.float64).reshape(-1) for m in machines]
    sizes = [int(i.numel()) for i in idx]
    moff = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0).tolist()), dtype=torch.int64, device=dev)
    ids = torch.cat(idx).contiguous()
    y = torch.cat(ys).contiguous()
    kd = torch.diagonal(K)[ids.long()].contiguous()
    a = torch.zeros_like(y)
    g = -torch.ones_like(y)
    nb = coop_workgroups(max(sizes), len(machines))
    r = _smo_coop(K, ids, moff, len(machines), max(sizes), y, kd, C, eps, tau, max_iter, ident, nb) if nb else None
    if r is not None:
        a, g, it = r
        out, o = [], 0
        for k, n in enumerate(sizes):
            out.append((a[o:o + n], g[o:o + n], it[k]))
            o += n
        return out
    if max(sizes) > int(_lib.kernels().harp_svm_max_rows()):
        # only the cooperative kernel takes machines this large, and it could not run (a
        # transient co-residency failure, or coop switched off): the caller falls back to
        # the PyTorch SMO loop instead of aborting the fit
        warnings.warn(f"device SMO: {max(sizes)} rows per machine exceed the one-CU kernel's "
                      f"{int(_lib.kernels().harp_svm_max_rows())} and the cooperative kernel did not run; "
                      "falling back to the PyTorch SMO loop")
        return None
    iters = torch.zeros(len(machines), dtype=torch.int32, device=dev)
    st = _lib.kernels().harp_svm_smo(K.data_ptr(), K.stride(0), ids.data_ptr(), moff.data_ptr(), len(machines),
                                     max(sizes), y.data_ptr(), kd.data_ptr(), a.data_ptr(), g.data_ptr(),
                                     iters.data_ptr(), float(C), float(eps), float(tau), int(max_iter),
                                     1 if ident else 0, _lib.stream_ptr(dev))
    _lib.check(st, "svm_smo")
    it = iters.tolist()
    out, o = [], 0
    for k, n in enumerate(sizes):
        out.append((a[o:o + n], g[o:o + n], it[k]))
        o += n
    return out


class BinarySVM:
    """C-SVC trained by SMO with WSS-2; labels in {-1, +1} (or {0,1} mapped)."""

    def __init__(self, C: float = 1.0, kernel: str = "linear", sigma: float = 1.0, accuracy_threshold: float = 1e-3,
                 tau: float = 1e-6, max_iterations: int = 100000, solver: str = "auto"):
        self.C, self.kernel, self.sigma = C, kernel, sigma
        self.eps, self.tau, self.max_iter = accuracy_threshold, tau, max_iterations
        self.solver = solver  # "auto": the device SMO for GPU Gram matrices; "torch": the oracle loop

    def fit(self, X: torch.Tensor, y: torch.Tensor, K: Optional[torch.Tensor] = None) -> "BinarySVM":
        Xd = X.double() if not (X.is_sparse or X.layout == torch.sparse_csr) else X.double()
        yv = y.double().reshape(-1)
        if bool(((yv == 0) | (yv == 1)).all()):
            yv = 2 * yv - 1
        n = yv.numel()
        K = kernel_matrix(Xd, Xd, self.kernel, self.sigma) if K is None else K.double()
        if self.solver != "torch" and native_smo_ok(K, n):
            ar = torch.arange(n, device=K.device)
            res = smo_device(K.contiguous(), [(ar, yv)], self.C, self.eps, self.tau, self.max_iter,
                             ident=K.shape[0] == n)
            if res is not None:
                a, G, steps = res[0]
                return self._finish(Xd, yv, a, G, steps)
        Kd = torch.diagonal(K).clone()
        a = torch.zeros(n, dtype=torch.float64, device=K.device)
        G = -torch.ones(n, dtype=torch.float64, device=K.device)
        Cc, tau = self.C, self.tau
        pos = yv > 0
        it = 0
        for it in range(self.max_iter):
            mg = -yv * G
            up = (pos & (a < Cc)) | (~pos & (a > 0))
            low = (pos & (a > 0)) | (~pos & (a < Cc))
            mu = torch.where(up, mg, torch.full_like(mg, -float("inf")))
            i = int(mu.argmax())
            m = float(mu[i])
            Mv = float(torch.where(low, mg, torch.full_like(mg, float("inf"))).min())
            if m - Mv < self.eps:
                break
            bt = m - mg  # > 0 for candidates
            at = Kd[i] + Kd - 2 * K[i]
            at = torch.where(at > 0, at, torch.full_like(at, tau))
            score = torch.where(low & (mg < m), -(bt * bt) / at, torch.full_like(bt, float("inf")))
            j = int(score.argmin())
            yi, yj = float(yv[i]), float(yv[j])
            aij = float(at[j])
            delta = float(bt[j]) / aij
            ai, aj = float(a[i]), float(a[j])
            lim_i = Cc - ai if yi > 0 else ai
            lim_j = aj if yj > 0 else Cc - aj
            delta = max(0.0, min(delta, lim_i, lim_j))
            dai, daj = yi * delta, -yj * delta
            a[i] += dai
            a[j] += daj
            # G += Q[:, i] dai + Q[:, j] daj,  Q = y y^T K
            G += yv * (yi * dai * K[i] + yj * daj * K[j])
        return self._finish(Xd, yv, a, G, it)

    def _finish(self, Xd, yv, a, G, steps: int) -> "BinarySVM":
        """Bias from the free SVs (or the violating-pair midpoint) and the SV set."""
        Cc = self.C
        pos = yv > 0
        self.n_iterations = steps + 1
        self.alpha, self.grad = a, G
        free = (a > 1e-12) & (a < Cc - 1e-12)
        yG = yv * G
        if bool(free.any()):
            rho = float(yG[free].mean())
        else:
            mg = -yG
            up = (pos & (a < Cc)) | (~pos & (a > 0))
            low = (pos & (a > 0)) | (~pos & (a < Cc))
            m = float(torch.where(up, mg, torch.full_like(mg, -float("inf"))).max())
            Mv = float(torch.where(low, mg, torch.full_like(mg, float("inf"))).min())
            rho = -(m + Mv) / 2
        self.bias = -rho
        sv = a > 1e-12
        self.sv_index = torch.nonzero(sv).reshape(-1)
        self.sv = Xd.to_dense()[sv] if (Xd.is_sparse or Xd.layout == torch.sparse_csr) else Xd[sv]
        self.coef = (a * yv)[sv]
        return self

    def dual_objective(self) -> float:
        """0.5 a^T Q a - e^T a = 0.5 a^T (G - e) with G = Q a - e."""
        return float(0.5 * (self.alpha * (self.grad - 1.0)).sum())

    def decision(self, X):
        Kx = kernel_matrix(X.double(), self.sv, self.kernel, self.sigma)
        return Kx @ self.coef + self.bias

    def predict(self, X):
        return (self.decision(X) > 0).long()


class MultiClassSVM:
    """One-against-one multiclass (DAAL multi_class_classifier with SVM two-class
    learners): K(K-1)/2 binary machines on a shared kernel matrix, majority vote."""

    def __init__(self, num_classes: int, **svm_kw):
        self.K, self.kw = num_classes, svm_kw
        self.machines: Dict[Tuple[int, int], BinarySVM] = {}

    def fit(self, X, y):
        yl = y.long().reshape(-1)
        Xd = X.double()
        Kfull = kernel_matrix(Xd, Xd, self.kw.get("kernel", "linear"), self.kw.get("sigma", 1.0))
        Xdense = Xd.to_dense() if (Xd.is_sparse or Xd.layout == torch.sparse_csr) else Xd
        pairs = []
        for a in range(self.K):
            for b in range(a + 1, self.K):
                idx = torch.nonzero((yl == a) | (yl == b)).reshape(-1)
                if idx.numel() == 0:
                    continue
                pairs.append(((a, b), idx, torch.where(yl[idx] == a, 1.0, -1.0).double()))
        if pairs and self.kw.get("solver", "auto") != "torch" and native_smo_ok(Kfull, max(p[1].numel() for p in pairs),
                                                                                     machines=len(pairs)):
            # all one-vs-one machines in ONE device launch over the shared Gram matrix
            proto = BinarySVM(**self.kw)
            res = smo_device(Kfull.contiguous(), [(idx, yy) for _, idx, yy in pairs], proto.C, proto.eps, proto.tau,
                             proto.max_iter)
            if res is not None:
                for (key, idx, yy), (al, G, steps) in zip(pairs, res):
                    self.machines[key] = BinarySVM(**self.kw)._finish(Xdense[idx], yy.to(al.device), al, G, steps)
                return self
        for key, idx, yy in pairs:
            self.machines[key] = BinarySVM(**self.kw).fit(Xdense[idx], yy, Kfull[idx][:, idx])
        return self

    def predict(self, X):
        votes = torch.zeros((X.shape[0], self.K), dtype=torch.float64, device=X.device)
        ar = torch.arange(X.shape[0], device=X.device)
        for (a, b), m in self.machines.items():
            win = torch.where(m.decision(X) > 0, a, b)
            votes[ar, win] += 1
        return votes.argmax(1)


# ---------------------------------------------------------------- cascade SVM (contrib)
class HarpString(Writable):
    """One UTF-8 string payload (contrib svm HarpString)."""

    def __init__(self, s: str = ""):
        self.s = s

    def write(self, out: DataOutput) -> None:
        b = self.s.encode("utf-8")
        out.write_int(len(b))
        out.write_bytes(b)

    def read(self, inp: DataInput) -> None:
        n = inp.read_int()
        self.s = inp.read_bytes(n).decode("utf-8")


class HarpStringPlus(PartitionCombiner):
    """Concatenate the strings of two partitions with the same id (contrib svm)."""

    def combine(self, cur, new) -> PartitionStatus:
        a, b = cur, new
        if a.s and b.s and not a.s.endswith("\n"):
            a.s += "\n"
        a.s += b.s
        return PartitionStatus.COMBINED


def _lines(X: torch.Tensor, y: torch.Tensor) -> List[str]:
    """libsvm text rows ``label idx:val ...`` (1-based indices, nonzeros only)."""
    out = []
    Xc = X.double().cpu()
    for i in range(Xc.shape[0]):
        nz = torch.nonzero(Xc[i]).reshape(-1).tolist()
        feats = " ".join(f"{j + 1}:{float(Xc[i, j])!r}" for j in nz)
        out.append(f"{float(y[i])!r} {feats}".rstrip())
    return out


def _parse(lines: Sequence[str], dim: int) -> Tuple[torch.Tensor, torch.Tensor]:
    X = torch.zeros((len(lines), dim), dtype=torch.float64)
    y = torch.zeros(len(lines), dtype=torch.float64)
    for r, ln in enumerate(lines):
        tok = ln.split()
        y[r] = float(tok[0])
        for t in tok[1:]:
            j, v = t.split(":")
            X[r, int(j) - 1] = float(v)
    return X, y


def cascade_svm(comm: Communicator, X: torch.Tensor, y: torch.Tensor, iterations: int = 3, C: float = 1.0,
                kernel: str = "linear", sigma: float = 1.0, eps: float = 1e-3) -> Dict[str, object]:
    """Iterative cascade: local data + global SVs -> local SVM -> allreduce SV lines
    (HarpStringPlus) -> de-duplicate. Returns the final SV set (identical on every worker)
    and a model trained on it."""
    dim = X.shape[1]
    local = _lines(X, y)
    base = dict.fromkeys(local)
    svs: Dict[str, None] = {}
    sizes = []
    for it in range(iterations):
        cur = dict(base)
        for s in svs:
            cur.setdefault(s)
        cl = list(cur)
        Xc, yc = _parse(cl, dim)
        m = BinarySVM(C, kernel, sigma, eps).fit(Xc.to(X.device), yc.to(X.device))
        mine = "\n".join(cl[i] for i in m.sv_index.tolist())
        t = Table(0, HarpStringPlus())
        t.add(0, HarpString(mine))
        if not CL.allreduce(comm, t):
            raise IOError("cascade SVM allreduce failed")
        svs = dict.fromkeys(ln for ln in t[0].s.split("\n") if ln)
        sizes.append(len(svs))
    Xs, ys = _parse(list(svs), dim)
    model = BinarySVM(C, kernel, sigma, eps).fit(Xs.to(X.device), ys.to(X.device))
    return {"support_vectors": list(svs), "sizes": sizes, "model": model}
