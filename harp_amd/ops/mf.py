"""Matrix-factorisation device ops (SGD update, squared-error sum).

GPU: ``csrc/mf_sgd.hip`` (subgroup-per-stream Hogwild SGD over user-sorted ratings).
CPU: the native sequential loop in ``csrc/host/mf_cpu.cpp`` (exact reference order).
Ratings are three parallel arrays ``rows`` (local user index, int32), ``cols`` (item index
within the resident H slice, int32), ``vals`` (float32).
"""
from __future__ import annotations

import ctypes
import math
from typing import List, Optional, Tuple

import os

import torch

from . import _lib

SUPPORTED_RANKS = (16, 32, 48, 64, 128, 256)  # 16-lane stream kernels
MAX_WIDE_RANK = 4096  # wave-per-stream kernels: 256 < r <= 4096, r % 4 == 0 (BASELINE #1: rank 2000)


def supported_rank(r: int) -> bool:
    return r in SUPPORTED_RANKS or (256 < r <= MAX_WIDE_RANK and r % 4 == 0)


def kernel_rank(r: int) -> int:
    """The smallest rank >= ``r`` the GPU kernels instantiate. Factors of any rank <=
    :data:`MAX_WIDE_RANK` train EXACTLY at that rank with zero-padded columns: under the
    update rule (SGDMPTask.java:46-77) e = v - w.h ignores zero columns, and a zero column
    of w and h receives lr * (e * 0 - lam * 0) = 0, so padded columns stay zero."""
    if r <= 0:
        raise ValueError(f"rank must be positive, got {r}")
    for s in SUPPORTED_RANKS:
        if s >= r:
            return s
    if r <= MAX_WIDE_RANK:
        return (r + 3) // 4 * 4
    raise NotImplementedError(f"native MF-SGD ranks go up to {MAX_WIDE_RANK}, got {r}")


def storage_rank(r: int, device) -> int:
    """Columns a model should allocate for rank-``r`` factors on ``device`` (zero-padded
    to :func:`kernel_rank` on a GPU, so the hot loop needs no per-call padding)."""
    dev = torch.device(device)
    return kernel_rank(r) if dev.type == "cuda" else r


class _Padded:
    """Native call on factors whose rank has no kernel instantiation: zero-padded copies
    at :func:`kernel_rank`, the trained columns copied back on exit (exact, see
    :func:`kernel_rank`; costs a copy of W and H per call -- models allocate padded
    storage with :func:`storage_rank` instead)."""

    def __init__(self, W: torch.Tensor, H: torch.Tensor, write_back: bool = True):
        self.W, self.H, self.wb = W, H, write_back
        r = W.shape[1]
        rk = kernel_rank(r)
        self.Wp = torch.nn.functional.pad(W, (0, rk - r)).contiguous()
        self.Hp = torch.nn.functional.pad(H, (0, rk - r)).contiguous()

    def __enter__(self):
        return self.Wp, self.Hp

    def __exit__(self, *exc):
        if self.wb and exc[0] is None:
            r = self.W.shape[1]
            self.W.copy_(self.Wp[:, :r])
            self.H.copy_(self.Hp[:, :r])
        return False

_lib.register({
    "harp_mf_sgd": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_void_p,
                    _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_float, _lib.c_float, _lib.c_void_p],
    "harp_mf_xcds": [],
    # rows, cols, vals, off, win, r, steps, chunk, blocks_per_xcd, variant, W, ldw, H, ldh, lr, lam, chk, gen, pws,
    # stream
    "harp_mf_sgd_xcd": [_lib.c_void_p] * 5 + [_lib.c_int] * 5 + [_lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_int,
                                                                 _lib.c_float, _lib.c_float, _lib.c_void_p,
                                                                 ctypes.c_uint64, _lib.c_void_p, _lib.c_void_p],
    "harp_mf_chk_words": [],
    "harp_mf_placed_ws_ints": [],
    # rows, cols, vals, off, win, r, steps, chunk, blocks_per_xcd, W, ldw, H, ldh, lr, lam, ws, stream
    "harp_mf_sgd_xcd_flow": [_lib.c_void_p] * 5 + [_lib.c_int] * 4 + [_lib.c_void_p, _lib.c_int, _lib.c_void_p,
                                                                    _lib.c_int, _lib.c_float, _lib.c_float,
                                                                    _lib.c_void_p, _lib.c_void_p],
    "harp_mf_flow_ws_ints": [],
    "harp_mf_rmse_blocks": [],
    "harp_mf_rmse": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_int,
                     _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
})


def _rt():
    rt = _lib.runtime()
    if rt is None:
        raise _lib.NativeUnavailable("libharp_runtime.so not built (python -m harp_amd.ops.build)")
    if not getattr(rt, "_mf_bound", False):
        rt.harp_mf_sgd_cpu.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                       ctypes.c_float]
        rt.harp_mf_sgd_cpu.restype = None
        rt.harp_mf_sse_cpu.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        rt.harp_mf_sse_cpu.restype = ctypes.c_double
        rt._mf_bound = True
    return rt


# variant 1 = one persistent launch per slice pass ordered by neighbour completion flags
# (mf_sgd_xcd_flow_kernel) instead of one launch per sub-step; ranks <= 256
FLOW_VARIANT = 1
_FLOW_WS: dict = {}


def _flow_ws(device: torch.device) -> torch.Tensor:
    """Zeroed int32 workspace of the flow kernel, one per (device, stream): the launch leaves
    it zeroed again, so launches on one stream reuse it (kernels on a stream serialise)."""
    stream = torch.cuda.current_stream(device)
    key = (device.index, stream.cuda_stream)
    ws = _FLOW_WS.get(key)
    if ws is None:
        n = int(_lib.kernels().harp_mf_flow_ws_ints())
        ws = _FLOW_WS[key] = torch.zeros(n, dtype=torch.int32, device=device)
    return ws


def check_flow_errors(device: torch.device) -> None:
    """Raise if a flow launch on ``device`` gave up waiting on a neighbour (host sync)."""
    for (idx, _), ws in _FLOW_WS.items():
        code = int(ws[-1].item()) if idx == device.index else 0
        if code:
            ws[-1].zero_()
            if code == 2:
                raise RuntimeError("MF-SGD flow kernel: a block ran on another XCD than blockIdx.x mod 8 (dispatch "
                                   "mapping differs from round-robin; results of that pass are invalid)")
            raise RuntimeError("MF-SGD flow kernel: a cross-XCD wait timed out (results of that pass are invalid)")


# variant 2 = mf_sgd_xcd_placed_kernel: each block trains the cell of the XCD it runs on
# (HW_REG_XCC_ID), so one XCD per cell holds whatever the dispatcher does; the fallback
# the models switch to when the placement check of the default kernel fires
PLACED_VARIANT = 2
# harp_mf_sgd_xcd variant bits 2..3: atomic (no-lost-update) write-back of W (1) / H (2)
ATOMIC_W, ATOMIC_H = 1, 2
# hot-H write-back: H rows of the items flagged in bit 31 of their column index (hot_items)
# take L2 atomic adds, every other H row the plain store (csrc/mf_sgd.hip, ATOM bit 2)
ATOMIC_HOT = 4
HOT_BIT = 1 << 31


def hot_items(counts: torch.Tensor, streams: int, trigger: float, residual: float) -> torch.Tensor:
    """Hot-item flags of a blocked SGD pass (bool, same shape as ``counts``: ratings per
    (slice, local item)). A cell holds ~1/8 of a slice's items with ~1/8 of its ratings, so
    its item shares are p_i ~ 8 c_i / T and two of the XCD's ``streams`` concurrent streams
    meet on one H row at ~ streams * sum_i p_i^2 expected collisions per rating (each one a
    lost update under plain write-back). A slice whose collisions exceed ``trigger`` gets
    its most popular items flagged -- in popularity order, until the collisions left on
    unflagged rows are at most ``residual``; below the trigger nothing is flagged (plain
    write-back everywhere: the Netflix-shape bench, sum p^2 ~ 0.0015)."""
    c = counts.double()
    T = c.sum(1, keepdim=True).clamp_min(1.0)
    p2 = XCDS * (c / T) ** 2                      # per item: its share of the cell's sum p^2
    flags = torch.zeros_like(counts, dtype=torch.bool)
    for s in range(counts.shape[0]):
        tot = float(p2[s].sum()) * streams
        if tot <= trigger:
            continue
        order = torch.argsort(c[s], descending=True)
        left = tot - torch.cumsum(p2[s][order], 0) * streams  # collisions left after flagging the top k + 1
        k = int((left > residual).sum()) + 1
        flags[s, order[:k]] = True
    return flags
# default kernel: tag residue <-> XCC per launch, raise an error word on a mismatch
# (HARP_MF_CHECK_PLACEMENT=0 turns it off: an A/B knob for its cost)
CHECK_PLACEMENT = os.environ.get("HARP_MF_CHECK_PLACEMENT", "1") != "0"
_CHK: dict = {}


class _Chk:
    """Per (device, stream) placement-check words of the default XCD kernel plus the
    launch-generation counter (a generation is never reused on the same words) and the
    placed kernel's zeroed claim workspace."""

    def __init__(self, device: torch.device):
        lib = _lib.kernels()
        self.words = torch.zeros(int(lib.harp_mf_chk_words()), dtype=torch.int64, device=device)
        self.pws = torch.zeros(int(lib.harp_mf_placed_ws_ints()), dtype=torch.int32, device=device)
        self.gen = 1

    def next_gen(self, steps: int) -> int:
        g = self.gen
        self.gen += steps
        return g


def _chk(device: torch.device) -> _Chk:
    stream = torch.cuda.current_stream(device)
    key = (device.index, stream.cuda_stream)
    c = _CHK.get(key)
    if c is None:
        c = _CHK[key] = _Chk(device)
    return c


def placement_probe(W: torch.Tensor, H: torch.Tensor, blocks_per_xcd: int) -> None:
    """One default XCD-blocked launch over EMPTY cells (every block only tags its residue ->
    XCC and exits): the placement check runs before any rating is trained, so a dispatcher
    that spreads a residue over two XCDs is caught by :func:`check_placement` before the
    first epoch instead of after a lossy one. Ranks <= 256 (the narrow
    kernels); wide ranks keep the per-epoch check."""
    r = W.shape[1]
    if not _lib.use_native(W) or not CHECK_PLACEMENT or r > 256 or not supported_rank(r):
        return
    dev = W.device
    z = torch.zeros(1, dtype=torch.int32, device=dev)
    off = torch.zeros(XCDS * XCDS + 1, dtype=torch.int64, device=dev)
    ck = _chk(dev)
    gen = ck.next_gen(XCDS)
    st = _lib.kernels().harp_mf_sgd_xcd(z.data_ptr(), z.data_ptr(), z.data_ptr(), off.data_ptr(), None, r, XCDS, 8,
                                        blocks_per_xcd, 0, W.data_ptr(), W.stride(0), H.data_ptr(), H.stride(0), 0.0,
                                        0.0, ck.words.data_ptr(), gen, ck.pws.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(st, "mf_sgd_xcd (placement probe)")


def check_placement(device: torch.device) -> dict:
    """Read (host sync) and clear the placement words of every stream on ``device``:
    ``{"violation": bool, "drained": n}`` -- a violation means a default-kernel launch had
    blocks of one residue on two XCDs (that pass ran Hogwild across L2s: every rating was
    still trained once; two residues sharing one XCD is not checked -- it only slows that
    XCD, it shares no cell); ``drained`` counts cells the placed
    kernel trained in its last block because their XCD received no block."""
    out = {"violation": False, "drained": 0}
    for (idx, _), c in _CHK.items():
        if idx != device.index:
            continue
        if int(c.words[24].item()):
            out["violation"] = True
            c.words[24].zero_()
        out["drained"] += int(c.pws[9].item())
        c.pws[9].zero_()
    return out


def _check(rows, cols, vals, W, H):
    assert rows.dtype == torch.int32 and cols.dtype == torch.int32 and vals.dtype == torch.float32
    assert rows.is_contiguous() and cols.is_contiguous() and vals.is_contiguous()
    assert W.dtype == torch.float32 and H.dtype == torch.float32 and W.stride(1) == 1 and H.stride(1) == 1
    assert W.shape[1] == H.shape[1]


def sgd_update(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, W: torch.Tensor, H: torch.Tensor,
               lr: float, lam: float, chunk: int = 64) -> int:
    """One pass of SGD over the given ratings, updating W and H in place. Returns n."""
    _check(rows, cols, vals, W, H)
    n = rows.numel()
    if n == 0:
        return 0
    r = W.shape[1]
    chunk = chunk if chunk > 0 else 64
    if _lib.use_native(W):
        if not supported_rank(r):
            with _Padded(W, H) as (Wp, Hp):
                return sgd_update(rows, cols, vals, Wp, Hp, lr, lam, chunk)
        st = _lib.kernels().harp_mf_sgd(rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), n, r, chunk, W.data_ptr(),
                                        W.stride(0), H.data_ptr(), H.stride(0), float(lr), float(lam),
                                        _lib.stream_ptr(W.device))
        _lib.check(st, "mf_sgd")
        return n
    _rt().harp_mf_sgd_cpu(rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), n, r, W.data_ptr(), W.stride(0),
                          H.data_ptr(), H.stride(0), float(lr), float(lam))
    return n


XCDS = 8  # cells per side of the XCD-blocked layout (csrc/mf_sgd.hip)


def cell_layout(rows: torch.Tensor, cols: torch.Tensor, n_rows: int, n_cols: int, nb: int = XCDS) -> torch.Tensor:
    """Cell id (user block * nb + item block) of every rating: contiguous user / item
    ranges, so a cell's H rows are one contiguous 1/nb of the slice."""
    rb = (rows.long() * nb) // max(n_rows, 1)
    cb = (cols.long() * nb) // max(n_cols, 1)
    return rb * nb + cb


def balanced_blocks(group: torch.Tensor, idx: torch.Tensor, n_groups: int, n_idx: int, nb: int = XCDS,
                    hot: float = 0.0) -> torch.Tensor:
    """Block (0..nb-1) of every (group, idx) record: within each group, contiguous idx
    ranges holding ~equal numbers of records (so skewed item popularity still gives the 8
    XCDs equal work per sub-step). ``hot`` > 0 weighs each record of an index with c records
    by 1 + hot * log2(1 + c / mean c): updates of a popular row contend for its L2 lines."""
    flat = group.long() * n_idx + idx.long()
    cnt = torch.bincount(flat, minlength=n_groups * n_idx).view(n_groups, n_idx)
    if hot > 0:
        c = cnt.double()
        mean = c.sum(1, keepdim=True) / (c > 0).sum(1, keepdim=True).clamp_min(1)
        w = c * (1.0 + hot * torch.log2(1.0 + c / mean.clamp_min(1.0)))
    else:
        w = cnt
    excl = torch.cumsum(w, 1) - w
    tot = w.sum(1, keepdim=True).clamp_min(1)
    blk = torch.clamp((excl * nb) // tot, max=nb - 1).long()
    return blk.view(-1)[flat]


def auto_chunk(n: int, blocks_per_xcd: int) -> int:
    """Ratings per update stream for an XCD-blocked pass over ``n`` ratings. A stream's
    ratings form one dependent chain (~0.6 us each: H row from L2, dot, update), so a
    kernel lasts at least chunk x that; with the 8-GPU per-rank share (12.5M Netflix
    ratings, 16 rotation sub-steps) chunk 64 left most of each XCD's 16 x blocks_per_xcd
    stream slots idle and every launch took ~40 us for ~100K ratings. Halve from 64 until
    the average cell fills the XCD's stream slots (floor 8)."""
    cell = n / float(XCDS * XCDS)
    slots = 16 * max(1, blocks_per_xcd)
    ch = 64
    while ch > 8 and cell / ch < slots:
        ch //= 2
    return ch


def sgd_update_blocked(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, cell_off: torch.Tensor,
                       W: torch.Tensor, H: torch.Tensor, lr: float, lam: float, chunk: int = 64,
                       blocks_per_xcd: int = 256, host_off: list | None = None, variant: int = 0,
                       window: Optional[Tuple[List[int], List[int]]] = None, threads: int = 1,
                       time_budget: Optional[float] = None, atomic: int = 0) -> int:
    """One SGD pass over ratings laid out in nb x nb cells (cell-major, user-sorted inside a
    cell; ``cell_off`` = nb*nb+1 int64 offsets on W's device). Sub-step s trains the nb
    row- and column-disjoint cells (x, (x+s) mod nb): on the GPU one XCD per cell
    (csrc/mf_sgd.hip, mf_sgd_xcd_kernel); on the CPU the same cells in the same order.
    ``host_off``: the offsets as a Python list (saves a device->host copy on the CPU path).
    ``chunk``: ratings per stream (8, 16, 32, 64 or 128 on the GPU; <= 0 = :func:`auto_chunk`);
    ``variant``: 0 = one launch per sub-step (placement-checked, :func:`check_placement`);
    1 (:data:`FLOW_VARIANT`, ranks <= 256) = the whole pass in one persistent launch
    ordered by per-XCD completion flags; 2 (:data:`PLACED_VARIANT`, ranks <= 256) = one
    launch per sub-step whose blocks pick their cell by the XCD they run on. ``atomic``
    (variants 0 / 2, ranks <= 256; bit set of :data:`ATOMIC_W` / :data:`ATOMIC_H`): the
    W / H changes are ADDED with L2 atomics instead of stored, so updates of concurrent
    streams to one row are never lost (csrc/mf_sgd.hip sgd_stream_lds ATOM).
    ``window=(starts, lengths)`` (64 each): cell c trains only ``lengths[c]`` ratings from
    ``starts[c]``, wrapping around the cell (fixed-fraction mode, :func:`cell_windows`).
    CPU only: ``threads > 1`` or a ``time_budget`` (s) run the cells through the 2-D
    conflict-free :class:`~harp_amd.runtime.dymoro.BlockScheduler` (order then depends on
    timing, like the reference's Scheduler). Returns the number of ratings trained."""
    _check(rows, cols, vals, W, H)
    n = rows.numel()
    if n == 0:
        return 0
    r = W.shape[1]
    nb = XCDS
    assert cell_off.numel() == nb * nb + 1 and cell_off.dtype == torch.int64
    trained = n if window is None else int(sum(window[1]))
    if _lib.use_native(W):
        if not supported_rank(r):
            with _Padded(W, H) as (Wp, Hp):
                return sgd_update_blocked(rows, cols, vals, cell_off, Wp, Hp, lr, lam, chunk, blocks_per_xcd,
                                          host_off, variant, window, atomic=atomic)
        assert cell_off.device == W.device and cell_off.is_contiguous()
        win = None
        if window is not None:
            win = torch.tensor(list(window[0]) + list(window[1]), dtype=torch.int64).pin_memory()
            win = win.to(W.device, non_blocking=True)
        if chunk <= 0:  # wide ranks (one wave per stream) take 32 / 64 / 128 only
            chunk = auto_chunk(trained, blocks_per_xcd) if r <= 256 else max(32, auto_chunk(trained, blocks_per_xcd))
        lib = _lib.kernels()
        if variant == FLOW_VARIANT and r <= 256:
            st = lib.harp_mf_sgd_xcd_flow(rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), cell_off.data_ptr(),
                                          _lib.ptr(win), r, nb, chunk, blocks_per_xcd, W.data_ptr(), W.stride(0),
                                          H.data_ptr(), H.stride(0), float(lr), float(lam),
                                          _flow_ws(W.device).data_ptr(), _lib.stream_ptr(W.device))
            _lib.check(st, "mf_sgd_xcd_flow")
        else:
            placed = variant == PLACED_VARIANT and r <= 256
            ck = _chk(W.device)
            words = ck.words if (CHECK_PLACEMENT and not placed) else None
            gen = ck.next_gen(nb) if words is not None else 0
            kv = (PLACED_VARIANT if placed else 0) | ((int(atomic) & 7) << 2 if r <= 256 else 0)
            st = lib.harp_mf_sgd_xcd(rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), cell_off.data_ptr(),
                                     _lib.ptr(win), r, nb, chunk, blocks_per_xcd, kv,
                                     W.data_ptr(), W.stride(0), H.data_ptr(), H.stride(0), float(lr), float(lam),
                                     _lib.ptr(words), gen, ck.pws.data_ptr(), _lib.stream_ptr(W.device))
            _lib.check(st, "mf_sgd_xcd")
        if win is not None:
            win.record_stream(torch.cuda.current_stream(W.device))
        return trained
    off = host_off if host_off is not None else cell_off.tolist()
    rt = _rt()

    def seg(a, m):
        if m > 0:
            rt.harp_mf_sgd_cpu(rows[a:].data_ptr(), cols[a:].data_ptr(), vals[a:].data_ptr(), m, r,
                               W.data_ptr(), W.stride(0), H.data_ptr(), H.stride(0), float(lr), float(lam))

    def cell(c: int) -> int:
        a, b = off[c], off[c + 1]
        if window is None:
            seg(a, b - a)
            return b - a
        w0, L = int(window[0][c]), int(window[1][c])
        first = min(L, (b - a) - w0)
        seg(a + w0, first)
        seg(a, L - first)
        return L

    if threads > 1 or time_budget is not None:
        # the reference's 2-D Scheduler (MJ/dymoro/Scheduler.java:95-237): row- and
        # column-disjoint cells run concurrently on a thread pool (native calls release the
        # GIL), refilled as cells finish, until every cell ran or the time budget expired
        from ..runtime.dymoro import BlockScheduler

        res = BlockScheduler(nb, nb, lambda x, y: cell(x * nb + y), num_threads=max(1, threads)).schedule(time_budget)
        return int(res["items"])
    for s in range(nb):
        for x in range(nb):
            cell(x * nb + (x + s) % nb)
    return trained


def cell_windows(cell_off: List[int], fraction: float, epoch: int) -> Tuple[List[int], List[int]]:
    """Fixed-fraction mode: every cell trains ceil(fraction * size) ratings per visit, the
    window advancing by its length each epoch, so all ratings are trained once per
    ceil(1 / fraction) epochs (deterministic stand-in for the reference's timer-bounded
    rotation steps, whose timer is tuned to cover ``trainRatio`` % of the ratings:
    SGDCollectiveMapper.java:623-668)."""
    starts, lens = [], []
    for c in range(len(cell_off) - 1):
        m = cell_off[c + 1] - cell_off[c]
        L = min(m, math.ceil(fraction * m))
        starts.append((epoch * L) % m if m else 0)
        lens.append(L)
    return starts, lens


def sse(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, W: torch.Tensor, H: torch.Tensor):
    """Sum of squared errors (0-dim float64 tensor on W's device)."""
    _check(rows, cols, vals, W, H)
    n = rows.numel()
    if n == 0:
        return torch.zeros((), dtype=torch.float64, device=W.device)
    r = W.shape[1]
    if _lib.use_native(W):
        if not supported_rank(r):
            with _Padded(W, H, write_back=False) as (Wp, Hp):
                return sse(rows, cols, vals, Wp, Hp)
        lib = _lib.kernels()
        nb = lib.harp_mf_rmse_blocks()
        part = torch.empty(nb, dtype=torch.float64, device=W.device)
        st = lib.harp_mf_rmse(rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), n, r, W.data_ptr(), W.stride(0),
                              H.data_ptr(), H.stride(0), part.data_ptr(), _lib.stream_ptr(W.device))
        _lib.check(st, "mf_rmse")
        return part.sum()
    v = _rt().harp_mf_sse_cpu(rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), n, r, W.data_ptr(), W.stride(0),
                              H.data_ptr(), H.stride(0))
    return torch.tensor(v, dtype=torch.float64)
