"""Symmetric eigen-decomposition of the PCA pass's d x d fp64 correlation matrix.

* the Householder tridiagonalisation: up to n = 1024 the chip-wide register-resident form
  (``csrc/eig_ll.hip``: rows of the matrix in the VGPRs of ceil(n / 8) workgroups, panel-deferred
  two-sided updates, one data-tagged granule exchange per column); above that, or if that
  launch could not get its workgroups co-resident, the one-XCD cooperative form
  (``csrc/eig.hip``);
* :func:`eigvalsh`: the reduction + multisection (``csrc/eig.hip``);
* :func:`eigh`: eigenvalues AND eigenvectors -- the same reduction keeping its reflectors,
  divide and conquer on the tridiagonal (``csrc/tridiag_dc.hip``: Cuppen merges with
  Gu-Eisenstat vectors, host reference ``ops/tridiag_dc.py``), and the back-transform
  X = Q Z = Z - V T (V^T Z) with the compact-WY triangle T^-1 = diag(1/tau) + striu(V^T V)
  as rocBLAS GEMMs and one triangular solve.

Reference: the DAAL PCA correlation step 3 (eigen-decomposition on the master),
ml/daal/src/main/java/edu/iu/daal_pca/cordensedistr/PCADaalCollectiveMapper.java:121-147.
"""
from __future__ import annotations

import os
import warnings

import torch

from . import _lib

_lib.register({
    "harp_eig_ws_ints": [],
    "harp_eig_max_n": [],
    "harp_eig_workgroups": [_lib.c_int, _lib.c_int],
    # A, lda, n, d, e, w, nb_max, ws, wsd, stamps, stream
    "harp_eig_sym": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                     _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    # A, lda, n, d, e, V, tau, nb_max, ws, wsd, stream
    "harp_sytrd_fused": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                         _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    "harp_dc_max_n": [],
    "harp_dc_prep_stamps": [_lib.c_void_p],
    "harp_dc_wave_stamps": [_lib.c_void_p],
    "harp_dc_ws_doubles": [_lib.c_int],
    # dmod, n, w, perm (int64), stream
    "harp_dc_order": [_lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    # d, e, n, dmod, Q, ws, perm, stream
    "harp_dc_setup": [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                      _lib.c_void_p, _lib.c_void_p],
    # dmod, e, n, Q, merges, level_off, level_smax, level_full, nlevels, ws, stream
    "harp_dc_tridiag": [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                        _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
    # A, lda, n, d, e, w, nb_max, ws, wsd, stream
    "harp_eig_sym_fused": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                           _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    # d, e, n, w, stream
    "harp_tridiag_eigvals": [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
    "harp_sytrd_ll_max_n": [],
    "harp_sytrd_ll_gran_words": [],
    "harp_sytrd_ll_workgroups": [_lib.c_int],
    "harp_sytrd_ll_stamps": [_lib.c_void_p],
    "harp_sytrd_ll_trace": [_lib.c_void_p],
    # A, lda, n, d, e, V, ldv, tau, ws, gran, stream
    "harp_sytrd_ll": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                      _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
})

NB_DEFAULT = 32  # workgroups (CUs) of XCD 0
# reduction form: "ll" (chip-wide, register-resident rows, granule exchange; n <= 1024, else
# "fused"), "fused" (one XCD, one pass over the trailing block and one arrival per column,
# look-ahead Householder vector) or "twopass" (matrix-vector pass + rank-2 update pass)
VARIANT = os.environ.get("HARP_EIG_VARIANT", "ll")


# crossover to rocSOLVER: the one-XCD reduction costs n steps of ~10-25 us and loses to the
# blocked dsyevd near n = 1.9k (eigh: n = 1000 11.7 vs 23-27 ms, 1536 29.2 vs 36.3, 1792
# 40.6 vs 44.1, 2048 57.3 vs 51.7; profiles/r4_eigh/crossover.log, time_barriers10.log)
NATIVE_MAX_N = int(os.environ.get("HARP_EIG_NATIVE_MAX", "1856"))


def usable(C: torch.Tensor, native: bool | None = None) -> bool:
    """The native kernels take C: fp64 square on a GPU, within the kernels' size limit and
    (``native=None``) at most NATIVE_MAX_N; ``native=True`` ignores the crossover (tests),
    ``native=False`` never takes them."""
    if native is False:
        return False
    ok = (C.device.type == "cuda" and C.dtype == torch.float64 and C.dim() == 2 and C.shape[0] == C.shape[1]
          and _lib.use_native(C) and 0 < C.shape[0] <= int(_lib.kernels().harp_eig_max_n()))
    return ok and (native is True or C.shape[0] <= NATIVE_MAX_N)


def eigvalsh(C: torch.Tensor, stamps: torch.Tensor | None = None, native: bool | None = None) -> torch.Tensor:
    """Ascending eigenvalues of the symmetric matrix ``C`` (fp64 on a GPU up to
    NATIVE_MAX_N: the one-XCD kernels; otherwise, or if the cooperative launch could not
    claim its workgroups, torch.linalg.eigvalsh). ``native``: see :func:`usable`."""
    if not usable(C, native if stamps is None else True):
        return torch.linalg.eigvalsh(C)
    n = C.shape[0]
    dev = C.device
    k = _lib.kernels()
    nb_max = int(os.environ.get("HARP_EIG_NB", NB_DEFAULT))
    nb = int(k.harp_eig_workgroups(n, nb_max))
    if nb < 1:
        return torch.linalg.eigvalsh(C)
    if VARIANT == "ll" and stamps is None:
        r = sytrd_ll(C, vectors=False, check=False)
        if r is not None:
            d, e, ws = r[0], r[1], r[4]
            w = torch.empty(n, dtype=torch.float64, device=dev)
            _lib.check(k.harp_tridiag_eigvals(d.data_ptr(), e.data_ptr(), n, w.data_ptr(), _lib.stream_ptr(dev)),
                       "tridiag_eigvals")
            if _ll_ok(ws):
                return w
    A = C.contiguous().clone()  # symmetric: row-major storage is the column-major matrix
    ws = torch.zeros(int(k.harp_eig_ws_ints()), dtype=torch.int32, device=dev)
    wsd = torch.zeros(3 * n + 4, dtype=torch.float64, device=dev)
    d = torch.empty(n, dtype=torch.float64, device=dev)
    e = torch.empty(n, dtype=torch.float64, device=dev)
    w = torch.empty(n, dtype=torch.float64, device=dev)
    if VARIANT in ("fused", "ll") and stamps is None:
        st = k.harp_eig_sym_fused(A.data_ptr(), n, n, d.data_ptr(), e.data_ptr(), w.data_ptr(), nb, ws.data_ptr(),
                                  wsd.data_ptr(), _lib.stream_ptr(dev))
    else:
        st = k.harp_eig_sym(A.data_ptr(), n, n, d.data_ptr(), e.data_ptr(), w.data_ptr(), nb_max, ws.data_ptr(),
                            wsd.data_ptr(), _lib.ptr(stamps), _lib.stream_ptr(dev))
    _lib.check(st, "eig_sym")
    claims, _, err = ws[:3].tolist()
    if claims < nb or err:
        warnings.warn(f"one-XCD eigensolver did not run cooperatively (claims {claims}/{nb}, error {err}); "
                      "using torch.linalg.eigvalsh")
        return torch.linalg.eigvalsh(C)
    return w


def ll_usable(n: int) -> bool:
    """The chip-wide reduction takes n <= harp_sytrd_ll_max_n() (1024) with one workgroup per
    8 rows, all co-resident (one per CU)."""
    k = _lib.kernels()
    return 0 < n <= int(k.harp_sytrd_ll_max_n())


_LL_WARNED = [False]


def _ll_ok(ws: torch.Tensor) -> bool:
    """Host check of the chip-wide reduction's error word (a workgroup timed out)."""
    if int(ws[2].item()):
        if not _LL_WARNED[0]:
            warnings.warn("chip-wide tridiagonalisation timed out (workgroups not co-resident); "
                          "using the one-XCD reduction")
            _LL_WARNED[0] = True
        return False
    return True


def sytrd_ll(C: torch.Tensor, vectors: bool = True, check: bool = True):
    """Tridiagonalise the symmetric fp64 GPU matrix ``C`` (n <= 1024) with the chip-wide
    kernel: returns (d, e, Vt, tau) -- Vt row k = v_k, tau_k as :func:`back_transform` takes
    them (None when ``vectors`` is False) -- or None when the kernel is not applicable or a
    workgroup timed out (not all of them co-resident). ``check=False``: no host sync; returns
    (d, e, Vt, tau, ws) and the caller checks ``ws`` with :func:`_ll_ok` after queueing
    the work that follows (so its launches overlap the reduction; the outputs of a timed-out
    call are finite: zero-initialised and partly written)."""
    n = C.shape[0]
    if not ll_usable(n):
        return None
    dev = C.device
    k = _lib.kernels()
    A = C.contiguous()
    ws = torch.zeros(int(k.harp_eig_ws_ints()), dtype=torch.int32, device=dev)
    gran = torch.zeros(int(k.harp_sytrd_ll_gran_words()), dtype=torch.int64, device=dev)
    d = torch.zeros(n, dtype=torch.float64, device=dev)
    e = torch.zeros(max(n, 1), dtype=torch.float64, device=dev)
    Vt = torch.zeros((n, n), dtype=torch.float64, device=dev) if vectors else None
    tau = torch.zeros(n, dtype=torch.float64, device=dev) if vectors else None
    st = k.harp_sytrd_ll(A.data_ptr(), n, n, d.data_ptr(), e.data_ptr(), _lib.ptr(Vt), n, _lib.ptr(tau),
                         ws.data_ptr(), gran.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(st, "sytrd_ll")
    if not check:
        return d, e, Vt, tau, ws
    if not _ll_ok(ws):
        return None
    return d, e, Vt, tau


# ------------------------------------------------------------------ eigenvectors
_TREES: dict = {}


def _tree(n: int, device: torch.device):
    """Cached D&C tree of size n: (merges int32 device [3 m], level offsets, level max
    block sizes (ctypes int arrays), split points int64 device, per-level "covers all n
    rows" flags (ctypes int array))."""
    key = (n, str(device))
    t = _TREES.get(key)
    if t is None:
        import ctypes

        from .tridiag_dc import tree_levels

        levels = tree_levels(n)
        flat, off, smax, full = [], [0], [], []
        for lev in levels:
            lev = sorted(lev)
            for m in lev:
                flat += list(m)
            off.append(off[-1] + len(lev))
            smax.append(max(hi - lo for lo, _, hi in lev))
            full.append(int(sum(hi - lo for lo, _, hi in lev) == n))  # buffers swap, no copy-back
        merges = torch.tensor(flat if flat else [0, 0, 0], dtype=torch.int32, device=device)
        mids = torch.tensor([m[1] for lev in levels for m in lev], dtype=torch.int64, device=device)
        t = (merges, (ctypes.c_int * len(off))(*off), (ctypes.c_int * max(1, len(smax)))(*smax), len(levels), mids,
             (ctypes.c_int * max(1, len(full)))(*full))
        _TREES[key] = t
    return t


def eigh_tridiag(d: torch.Tensor, e: torch.Tensor):
    """Eigenvalues (ascending) and eigenvectors of the symmetric tridiagonal (d, e) (fp64
    on a GPU: the D&C kernels; otherwise the host reference)."""
    n = d.numel()
    if not (d.device.type == "cuda" and d.dtype == torch.float64 and _lib.use_native(d)
            and 0 < n <= int(_lib.kernels().harp_dc_max_n())):
        from .tridiag_dc import eigh_tridiag as ref

        w, V = ref(d.detach().cpu().numpy(), e.detach().cpu().numpy())
        return torch.from_numpy(w).to(d), torch.from_numpy(V).to(d)
    dev = d.device
    k = _lib.kernels()
    merges, off, smax, nlev, _, full = _tree(n, dev)
    ec = e.contiguous() if e.numel() else torch.zeros(1, dtype=torch.float64, device=dev)
    # dmod (d with |e| taken off both sides of every split), Q = I and the zeroed workspace
    # in one launch (csrc/tridiag_dc.hip dc_setup_kernel; the tree splits every position)
    dmod = torch.empty(n, dtype=torch.float64, device=dev)
    Qt = torch.empty((n, n), dtype=torch.float64, device=dev)  # column-major Q == row-major Q^T
    ws = torch.empty(int(k.harp_dc_ws_doubles(n)), dtype=torch.float64, device=dev)
    perm = torch.empty(n, dtype=torch.int64, device=dev)  # identity here, the sort order below
    _lib.check(k.harp_dc_setup(d.contiguous().data_ptr(), ec.data_ptr(), n, dmod.data_ptr(), Qt.data_ptr(),
                               ws.data_ptr(), perm.data_ptr(), _lib.stream_ptr(dev)), "dc_setup")
    st = k.harp_dc_tridiag(dmod.data_ptr(), ec.data_ptr(), n, Qt.data_ptr(), merges.data_ptr(), off, smax, full, nlev,
                           ws.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(st, "dc_tridiag")
    w = torch.empty(n, dtype=torch.float64, device=dev)
    _lib.check(k.harp_dc_order(dmod.data_ptr(), n, w.data_ptr(), perm.data_ptr(), _lib.stream_ptr(dev)), "dc_order")
    return w, Qt.index_select(0, perm).t()


def eigh(C: torch.Tensor, native: bool | None = None):
    """Eigenvalues (ascending) and eigenvectors (columns) of the symmetric matrix ``C``
    (fp64 on a GPU up to NATIVE_MAX_N: one-XCD reduction + D&C + WY back-transform;
    otherwise, or if the cooperative launch could not claim its workgroups,
    torch.linalg.eigh). ``native``: see :func:`usable`."""
    if not usable(C, native):
        return torch.linalg.eigh(C)
    n = C.shape[0]
    dev = C.device
    k = _lib.kernels()
    if VARIANT == "ll":
        r = sytrd_ll(C, check=False)
        if r is not None:
            d, e, Vt, tau, ws = r
            out = _dc_and_back_transform(d, e[:max(n - 1, 0)], Vt, tau)
            if _ll_ok(ws):  # one sync, after the D&C and back-transform are queued
                return out
    nb = int(k.harp_eig_workgroups(n, int(os.environ.get("HARP_EIG_NB", NB_DEFAULT))))
    if nb < 1:
        return torch.linalg.eigh(C)
    A = C.contiguous().clone()
    ws = torch.zeros(int(k.harp_eig_ws_ints()), dtype=torch.int32, device=dev)
    wsd = torch.zeros(3 * n + 4, dtype=torch.float64, device=dev)
    d = torch.empty(n, dtype=torch.float64, device=dev)
    e = torch.zeros(max(n, 1), dtype=torch.float64, device=dev)
    Vt = torch.zeros((n, n), dtype=torch.float64, device=dev)  # column-major reflectors
    tau = torch.zeros(n, dtype=torch.float64, device=dev)
    st = k.harp_sytrd_fused(A.data_ptr(), n, n, d.data_ptr(), e.data_ptr(), Vt.data_ptr(), tau.data_ptr(), nb,
                            ws.data_ptr(), wsd.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(st, "sytrd_fused")
    claims, _, err = ws[:3].tolist()
    if claims < nb or err:
        warnings.warn(f"one-XCD reduction did not run cooperatively (claims {claims}/{nb}, error {err}); "
                      "using torch.linalg.eigh")
        return torch.linalg.eigh(C)
    return _dc_and_back_transform(d, e[:max(n - 1, 0)], Vt, tau)


_SIDE: dict = {}


def _dc_and_back_transform(d, e, Vt, tau):
    """D&C eigenvectors Z of the tridiagonal, X = Q Z. The WY factor M = V T of Q depends only
    on the reflectors, so it is formed on a side stream while the D&C runs (the D&C's lower
    tree levels fill a fraction of the chip); what is left after the D&C is two GEMMs."""
    dev = d.device
    cur = torch.cuda.current_stream(dev)
    side = _SIDE.get(dev)
    if side is None:
        side = _SIDE[dev] = torch.cuda.Stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        wy = wy_factor(Vt, tau, rowmajor=True)  # V and M^T row-major for the apply below
    Vt.record_stream(side)
    tau.record_stream(side)
    lam, Z = eigh_tridiag(d, e)
    cur.wait_stream(side)
    if wy is None:
        return lam, Z
    V, Mt = wy
    Mt.record_stream(cur)
    V.record_stream(cur)
    Zt = Z.t()
    if Zt.is_contiguous():
        # X^T = Z^T - (Z^T V) M^T: row-major GEMMs in place on the fresh Z^T buffer (the
        # eigenvectors come back as the columns of a transposed view); 0.121 -> ~0.084 ms at
        # n = 1000 against apply_wy (profiles/r6_dcwave/probe_wy_apply.json)
        return lam, Zt.addmm_(Zt @ V, Mt, alpha=-1).t()
    return lam, apply_wy(V.t(), Mt, Z)


def wy_factor(Vt: torch.Tensor, tau: torch.Tensor, rowmajor: bool = False):
    """Compact-WY factor of H_0 H_1 ... H_{n-3} (``Vt`` row c = v_c): Q = I - V T V^T with
    T^-1 = diag(1/tau) + striu(V^T V); returns (V^T, M^T) with M = V T (one GEMM and one
    triangular solve), or None for n <= 2 (Q = I). A reflector with tau = 0 is the
    identity (its column of V is zeroed, no host sync). ``rowmajor``: returns (V, M^T) both
    contiguous (V n x m), the operands of the in-place row-major apply in
    :func:`_dc_and_back_transform`; V^T V is then formed from two row-major operands (rocBLAS
    picks a faster kernel for that form)."""
    n = Vt.shape[1]
    m = n - 2
    if m <= 0:
        return None
    t = tau[:m]
    live = t != 0
    Vm = Vt[:m] * live.to(Vt.dtype).unsqueeze(1)  # V^T, m x n
    V = Vm.t().contiguous() if rowmajor else None
    Tinv = torch.triu(Vm @ (V if rowmajor else Vm.t()), 1)
    Tinv.diagonal().copy_(torch.where(live, 1.0 / torch.where(live, t, torch.ones_like(t)), torch.ones_like(t)))
    # M^T = T^T V^T = Tinv^-T V^T: a lower-triangular solve with n right-hand sides
    Mt = torch.linalg.solve_triangular(Tinv.t(), Vm, upper=False)
    if rowmajor:
        return V, Mt.contiguous()
    return Vm, Mt


def apply_wy(Vm: torch.Tensor, Mt: torch.Tensor, Z: torch.Tensor) -> torch.Tensor:
    """X = Q Z = Z - M (V^T Z) for the factor of :func:`wy_factor`."""
    return torch.addmm(Z, Mt.t(), Vm @ Z, alpha=-1.0)


def back_transform(Vt: torch.Tensor, tau: torch.Tensor, Z: torch.Tensor) -> torch.Tensor:
    """X = H_0 H_1 ... H_{n-3} Z for the reflectors of :func:`eigh` (``Vt`` row c = v_c):
    compact WY, Q = I - V T V^T with T^-1 = diag(1/tau) + striu(V^T V), as two GEMMs and
    one triangular solve (rocBLAS; a reflector with tau = 0 is the identity)."""
    n = Z.shape[0]
    m = n - 2
    if m <= 0:
        return Z
    V = Vt[:m].t()  # n x m
    t = tau[:m]
    live = t != 0
    if not bool(live.all()):
        V = V * live.to(V.dtype)
    Tinv = torch.triu(V.t() @ V, 1)
    Tinv.diagonal().copy_(torch.where(live, 1.0 / torch.where(live, t, torch.ones_like(t)), torch.ones_like(t)))
    Y = torch.linalg.solve_triangular(Tinv, V.t() @ Z, upper=True)
    return Z - V @ Y
