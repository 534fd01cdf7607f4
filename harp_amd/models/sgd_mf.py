"""MF-SGD with model rotation (Harp's second headline workload).

Reference: ml/java/.../sgd/SGDCollectiveMapper.java:183-326 — W (user factors) is
row-partitioned and stays local (ratings are regrouped by a random row owner, :384); H
(item factors) is column-partitioned into ``P x numModelSlices`` slices (numModelSlices =
2, :120) that rotate around the workers (dymoro Rotator); per iteration, P steps x 2
slices of {compute on slice k, rotate slice k}; test RMSE every 5 iterations with an
allreduce of (SSE, count) (:670-735). Update rule SGDMPTask.java:46-77.

MI355X design: ratings on each worker are bucketed once by H slice and sorted by user;
each (user-block x resident slice) pass is one HIP kernel (``ops.mf.sgd_update``); the
two slices of a worker rotate on two private RCCL channels so slice k's transfer
overlaps the kernel on slice k+1 (:class:`~harp_amd.runtime.dymoro.DeviceRotator`);
no host synchronisation inside an epoch.
"""
from __future__ import annotations

import math
import os
import random
import sys
import time
from dataclasses import dataclass, replace
from typing import List, Optional, Tuple

import torch

from ..ops import mf as MF
from ..runtime.dymoro import (DeviceRotator, RotationSchedule, StepBudget, create_rotation_order,
                              get_rotation_sequences, ring_strides, tune_budget)
from ..runtime.mapper import CollectiveMapper, Context, KeyValReader


@dataclass
class SGDConfig:
    rank: int = 128            # r
    lam: float = 0.05          # lambda
    lr: float = 0.002          # epsilon
    epochs: int = 10
    num_slices: int = 2        # model slices per worker (numModelSlices)
    chunk: int = 0             # ratings per GPU update stream (0 = auto: ops.mf.auto_chunk)
    hot_balance: float = 1.0   # XCD item blocks weigh a row's ratings by 1 + h log2(1 + c / mean c): hot rows
                               # contend for their L2 lines (ops.mf.balanced_blocks; 6.35 -> 6.02 ms per
                               # 100M-rating epoch at skew 2, profiles/r3_sgd_hot_balance); 0 = equal counts
    xcd_blocks: bool = True    # 8 x 8 cell schedule, one XCD per cell (ops.mf.sgd_update_blocked)
    blocks_per_xcd: int = 128  # workgroups per XCD of the blocked kernel (upper bound, see conflicts_per_rating)
    conflict_mode: str = "cap"  # GPU, when a cell's expected collisions S sum p^2 exceed conflicts_per_rating:
                               # "cap" lowers blocks_per_xcd (plain Hogwild write-back: stable at any step size);
                               # "hot" keeps every block and flags the cell's most popular items for lossless
                               # (atomic) H write-back, plus atomic W, until at most hot_residual collisions per
                               # rating remain on plain rows -- the reference ML-10M gate at 128 blocks / XCD:
                               # 0.8360 vs 0.8377 capped (profiles/r6_sgd). Lossless accumulation ADDS the steps
                               # of streams that read one stale row, which diverged on an 800-item toy at lr 0.01
                               # (scripts/sgd_toy_diag.py), so it is opt-in
    hot_step_budget: float = 0.1  # "hot" mode: lossless write-back ADDS every concurrent stream's step (all
                               # computed from one stale row), so the effective step grows with the collisions:
                               # blocks_per_xcd is capped so that lr x S sum p^2 <= this (ML-10M, lr 0.002,
                               # sum p^2 0.022: 141 >= 128 blocks, no cap; an 800-item toy at lr 0.01 diverged
                               # at 0.25 and at no cap)
    hot_residual: float = 0.1  # "hot" mode: expected collisions per rating left on plain-stored H rows
                               # (ML-10M at 128 blocks/XCD: 0.5 -> test RMSE 0.8367, 0.1 -> 0.8360, all-atomic
                               # 0.8355; profiles/r6_sgd)
    conflicts_per_rating: float = 5.0  # GPU: cap the XCD's concurrent streams S (16 x blocks_per_xcd) at
                               # this / sum_i p_i^2 of a cell (expected same-item concurrent updates per rating;
                               # two streams updating one H row at once lose one update). The reference's ML-10M
                               # gate (sum p^2 = 0.021 per cell): test RMSE 0.8369 / 0.8388 / 0.8408 / 0.8450 /
                               # 0.8552 at S = 128 / 256 / 512 / 1024 / 2048 (profiles/r5_mf_gate); Netflix-shape
                               # synthetic at P = 1 (0.0015): no cap below 128 blocks; 0 = no cap
    kernel_variant: int = 0    # blocked kernel: 0 = a launch per sub-step, 1 = persistent flow kernel (ops.mf)
    atomic: int = 0            # GPU blocked kernel: add the W (1) / H (2) changes with L2 atomics (no lost updates)
    train_fraction: float = 1.0  # per rotation step each cell trains this fraction (window advances per epoch)
    random_order: bool = False  # random rotation orders (RotationUtil) vs ring
    test_every: int = 5        # rmseIteInterval
    seed: int = 0
    init_scale: float = -1.0   # <0: sqrt(mean_rating / r) (E[w.h] = mean rating)
    init: str = "mean"         # "mean": U(0, 2 init_scale); "reference": U(0, 1) / sqrt(r), the reference's
                               # SGDUtil.randomize (ml/java/.../sgd/SGDUtil.java:72-82)
    checkpoint_dir: str = ""   # .hpt checkpoints (W rows + resident H slices); resume on restart
    checkpoint_every: int = 0  # epochs between checkpoints (0: never)
    model_dir: str = ""        # final text dump: W-<worker>, H-<worker>, evaluation
    time_budget_ms: float = 0.0  # >0: time-bounded rotation steps (Scheduler timer); 0: deterministic
    budget_pieces: int = 8     # launches a step's work is cut into (budget granularity)
    tune_ratio: float = 0.0    # >0: after epoch 0 retune the budget so an epoch trains this fraction
    cpu_threads: int = 1       # CPU workers: >1 runs the 8 x 8 cells through the 2-D BlockScheduler


def load_mm(path: str) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Read ``row col value`` text (Matrix Market body, optionally .bz2), 1-based ids."""
    import bz2
    import numpy as np

    opener = bz2.open if path.endswith(".bz2") else open
    with opener(path, "rt") as f:
        lines = [ln for ln in f if ln.strip() and not ln.startswith("%")]
    arr = np.loadtxt(lines, dtype=np.float64, ndmin=2)
    return (torch.from_numpy(arr[:, 0].astype("int64") - 1), torch.from_numpy(arr[:, 1].astype("int64") - 1),
            torch.from_numpy(arr[:, 2].astype("float32")))


def synthetic_ratings(n_users: int, n_items: int, n_ratings: int, seed: int = 0, device="cpu", true_rank: int = 8,
                      skew: float = 2.0):
    """Netflix-shaped synthetic ratings: uniform users, Zipf-like item popularity (item of
    rank q drawn with density ~ q^(1/skew - 1); skew=1 is uniform), values from a hidden
    rank-``true_rank`` model + noise clipped to [1, 5]."""
    g = torch.Generator(device=device).manual_seed(seed)
    u = torch.randint(0, n_users, (n_ratings,), generator=g, device=device)
    pop = torch.rand(n_ratings, generator=g, device=device) ** skew
    perm = torch.randperm(n_items, generator=g, device=device)
    it = perm[(pop * n_items).long().clamp_max(n_items - 1)]
    Ut = torch.randn((n_users, true_rank), generator=g, device=device) / math.sqrt(true_rank)
    Vt = torch.randn((n_items, true_rank), generator=g, device=device) / math.sqrt(true_rank)
    val = torch.empty(n_ratings, device=device)
    step = 1 << 24
    for s in range(0, n_ratings, step):
        e = min(s + step, n_ratings)
        val[s:e] = (3.6 + (Ut[u[s:e]] * Vt[it[s:e]]).sum(1) + 0.3 * torch.randn(e - s, generator=g, device=device))
    return u, it, val.clamp_(1.0, 5.0)


class _SetupTrace:
    """HARP_BENCH_TRACE=1: elapsed seconds of init_model's phases on stderr."""

    def __init__(self, rank: int):
        self.on = bool(os.environ.get("HARP_BENCH_TRACE"))
        self.rank, self.t0 = rank, time.perf_counter()

    def __call__(self, what: str) -> None:
        if self.on:
            print(f"sgd setup rank {self.rank}: {what} +{time.perf_counter() - self.t0:.2f}s", file=sys.stderr,
                  flush=True)


def row_owner(users: torch.Tensor, P: int, seed: int = 0) -> torch.Tensor:
    """Random-but-shared row owner (the reference's RandomPartitioner, seeded from an
    allreduced seed): a multiplicative hash of the row id, mod P."""
    h = (users * 2654435761 + seed) % 4294967296
    return h % P


class _Buckets:
    """Ratings of this worker bucketed by global H slice, user-sorted inside a bucket.

    ``cells=(n_rows, items_per_slice)``: inside a slice the ratings are further grouped
    into the 8 x 8 (user block, item block) cells of the XCD-blocked kernel
    (``ops.mf.sgd_update_blocked``), user-sorted inside a cell; ``cell_off[s]`` holds the
    65 cell offsets of slice s (relative to the slice start)."""

    def __init__(self, rows, cols, vals, slice_of_item, local_of_item, n_slices, device, cells=None, hot=0.0,
                 hot_items=None):
        g = slice_of_item[cols]
        lc = local_of_item[cols]
        span = int(rows.max().item()) + 1 if rows.numel() else 1
        nc = MF.XCDS * MF.XCDS
        if cells is not None:
            # equal-work cells: contiguous user / item ranges holding ~1/8 of the slice's
            # ratings each (skewed item popularity would otherwise leave XCDs idle)
            rb = MF.balanced_blocks(g, rows, n_slices, cells[0])
            cb = MF.balanced_blocks(g, lc, n_slices, cells[1], hot=hot)
            cid = g * nc + rb * MF.XCDS + cb
            key = cid * span + rows
        else:
            key = g * span + rows
        order = torch.argsort(key)
        self.rows = rows[order].to(torch.int32).contiguous().to(device)
        lcs = lc[order]
        self.flagged = hot_items is not None
        if hot_items is not None:  # bit 31: the item's H row takes atomic write-back (ops.mf.hot_items)
            flag = hot_items.to(lcs.device)[g[order], lcs]
            lcs = lcs | (flag.long() << 31)
        self.cols = (lcs - ((lcs >> 31) << 32)).to(torch.int32).contiguous().to(device)
        self.vals = vals[order].to(torch.float32).contiguous().to(device)
        counts = torch.bincount(g, minlength=n_slices).cpu()
        self.offsets = [0] + torch.cumsum(counts, 0).tolist()
        self.n = rows.numel()
        self.cell_off = None
        if cells is not None:
            cc = torch.bincount(cid, minlength=n_slices * nc).cpu().view(n_slices, nc)
            off = torch.zeros((n_slices, nc + 1), dtype=torch.int64)
            off[:, 1:] = torch.cumsum(cc, 1)
            self.cell_off_host = off.tolist()
            self.cell_off = off.to(device)

    def get(self, s: int, plain: bool = False):
        a, b = self.offsets[s], self.offsets[s + 1]
        c = self.cols[a:b]
        if plain and self.flagged:
            c = c & 0x7FFFFFFF
        return self.rows[a:b], c, self.vals[a:b]

    def get_cells(self, s: int):
        """(rows, cols, vals, device cell offsets, host cell offsets) of slice s."""
        return (*self.get(s), self.cell_off[s], self.cell_off_host[s])


class SGDCollectiveMapper(CollectiveMapper):
    def __init__(self, comm=None, config: Optional[SGDConfig] = None, n_users: int = 0, n_items: int = 0,
                 train=None, test=None, metrics=None):
        super().__init__(comm, metrics)
        # a private copy: the placement fallback switches kernels on it, never on the caller's
        self.cfg = replace(config) if config is not None else SGDConfig()
        self.n_users, self.n_items = n_users, n_items
        self._train, self._test = train, test
        self.rmse_history: List[Tuple[int, float, float]] = []
        self.placement_events: list = []
        self.epoch_times: List[float] = []

    # -- partitioning -------------------------------------------------------------------
    def _owner(self, users: torch.Tensor) -> torch.Tensor:
        return row_owner(users, self.get_num_workers(), self.cfg.seed)

    def init_model(self, reader: KeyValReader) -> None:
        cfg = self.cfg
        P, me, dev = self.get_num_workers(), self.get_self_id(), self.device
        S = cfg.num_slices
        n_slices = P * S
        trace = _SetupTrace(me)
        u, i, v = self._train
        mine = self._owner(u) == me
        u, i, v = u[mine], i[mine], v[mine]
        trace("own ratings")
        # local dense user index
        self.users = torch.unique(self._all_users_of(me))
        lut = torch.full((self.n_users,), -1, dtype=torch.int64, device=u.device)
        lut[self.users.to(u.device)] = torch.arange(self.users.numel(), device=u.device)
        rows = lut[u]
        # item -> (slice, local index): seeded permutation, equal slice sizes
        g = torch.Generator().manual_seed(cfg.seed + 12345)
        perm = torch.randperm(self.n_items, generator=g)
        self.ips = math.ceil(self.n_items / n_slices)
        pos = torch.empty(self.n_items, dtype=torch.int64)
        pos[perm] = torch.arange(self.n_items)
        self.slice_of_item = (pos // self.ips).to(u.device)
        self.local_of_item = (pos % self.ips).to(u.device)
        self.item_perm = perm  # slice s holds items perm[s*ips:(s+1)*ips]
        cells = (self.users.numel(), self.ips) if cfg.xcd_blocks else None
        # concurrency cap: an XCD's 16 x blocks streams share one cell's items; a stream meets
        # another on its item with probability ~ sum_i p_i^2 (p_i: item i's share of the cell's
        # ratings), so the expected concurrent same-item updates per rating are ~ S sum p^2
        self.bpx = cfg.blocks_per_xcd
        hot = None
        self.hot_items = 0
        if cfg.conflicts_per_rating > 0 and dev.type == "cuda":
            key = self.slice_of_item[i] * self.ips + self.local_of_item[i]
            cnt = torch.bincount(key, minlength=n_slices * self.ips).view(n_slices, self.ips).double()
            if P > 1:  # every rank's ratings meet on the slice's rows when it is resident there
                self.comm.all_reduce(cnt)
            tot = cnt.sum(1).clamp_min(1.0)
            # a cell holds 1/8 of a slice's items with ~1/8 of its ratings (equal-work item
            # blocks): its sum of squared shares is ~8 x the slice's
            sp2 = float((MF.XCDS * ((cnt / tot[:, None]) ** 2).sum(1)).mean())
            self.cell_sum_p2 = sp2
            # (the per-sub-step and placed kernels take the hot flag; the persistent flow kernel
            # and the wide-rank kernels keep plain write-back)
            use_hot = (cfg.conflict_mode == "hot" and cfg.xcd_blocks and MF.storage_rank(cfg.rank, dev) <= 256
                       and cfg.kernel_variant != MF.FLOW_VARIANT)
            if use_hot:
                self.bpx = max(2, min(cfg.blocks_per_xcd, int(cfg.hot_step_budget / max(cfg.lr, 1e-12)
                                                              / max(sp2, 1e-12) / 16)))
                hot = MF.hot_items(cnt.cpu(), 16 * self.bpx, cfg.conflicts_per_rating, cfg.hot_residual)
                self.hot_items = int(hot.sum())
                if not self.hot_items:
                    hot = None
            elif cfg.conflict_mode in ("hot", "cap"):  # (kernels without the hot flag: the cap)
                self.bpx = max(2, min(cfg.blocks_per_xcd, int(cfg.conflicts_per_rating / max(sp2, 1e-12) / 16)))
        trace("user / item maps")
        self.train = _Buckets(rows, i, v, self.slice_of_item, self.local_of_item, n_slices, dev, cells=cells,
                              hot=cfg.hot_balance, hot_items=hot)
        # lossless write-back where collisions are frequent: atomic W rows + flagged H rows
        self.atomic = cfg.atomic | (MF.ATOMIC_W | MF.ATOMIC_HOT if hot is not None else 0)
        trace("rating buckets")
        if self._test is not None:
            tu, ti, tv = self._test
            m = self._owner(tu) == me
            tr = lut[tu[m]]
            ok = tr >= 0  # test users never seen in training are skipped (no W row)
            self.test = _Buckets(tr[ok], ti[m][ok], tv[m][ok], self.slice_of_item, self.local_of_item, n_slices, dev)
        else:
            self.test = None
        # model: W local, H slices of the blocks initially placed here
        r = cfg.rank
        # GPU factors carry zero columns up to the next kernel rank (exact: ops.mf.kernel_rank)
        self.rs = MF.storage_rank(r, dev)
        mean = float(v.mean().item()) if v.numel() else 3.0
        trace("local mean")
        tot = torch.tensor([mean * v.numel(), float(v.numel())], dtype=torch.float64, device=dev)
        if P > 1:
            self.comm.all_reduce(tot)
        mean = float(tot[0] / max(tot[1], 1))
        trace("mean allreduce")
        if cfg.init == "reference":
            scale = 0.5 / math.sqrt(r)
        else:
            scale = cfg.init_scale if cfg.init_scale > 0 else math.sqrt(mean / r)
        gw = torch.Generator().manual_seed(cfg.seed * 31 + 7 + me)
        self.W = self._padded(torch.rand((self.users.numel(), r), generator=gw) * 2 * scale)
        trace("W init")
        orders = get_rotation_sequences(self, cfg.epochs + 2, cfg.seed) if cfg.random_order else None
        # ring mode: slice k rotates on its own stride so the slices use different xGMI links
        # (dymoro.ring_strides); random orders are shared by all slices, as in the reference
        strides = ring_strides(P, S) if orders is None else [1] * S
        self.schedules = [RotationSchedule(P, orders, stride=st) for st in strides]
        self.schedule = self.schedules[0]
        block = self.schedule.block_at(me, 0, 0)
        slabs = []
        for k in range(S):
            gs = block * S + k
            gh = torch.Generator().manual_seed(cfg.seed * 1009 + gs)
            slabs.append(self._padded(torch.rand((self.ips, r), generator=gh) * 2 * scale))
        self.rot = DeviceRotator(self.comm, slabs, name="sgd-h", metrics=self.metrics)
        trace("H slabs + rotator")
        self.trained = 0
        # timer-bounded steps: one budget for every path (GPU pieces, CPU pieces, and the
        # threaded CPU BlockScheduler, which adds its step times so the tuner can read them)
        self.budget = StepBudget(cfg.time_budget_ms / 1e3, dev) if cfg.time_budget_ms > 0 else None
        self.budget_history = [self.budget.budget_s] if self.budget is not None else []
        self._cursor = {}
        # placement pre-flight: one launch over empty cells tags every residue's XCC, so a
        # dispatcher that splits a residue over two XCDs switches the schedule BEFORE the
        # first epoch (otherwise the first epoch would run Hogwild across L2s)
        if dev.type == "cuda" and cfg.xcd_blocks and cfg.kernel_variant == 0:
            MF.placement_probe(self.W, slabs[0], self.bpx)
            self._check_placement(-1)

    def _padded(self, M: torch.Tensor) -> torch.Tensor:
        """``M`` [n, r] on the device with zero columns up to the storage rank."""
        out = torch.zeros((M.shape[0], self.rs), dtype=torch.float32, device=self.device)
        out[:, : M.shape[1]] = M.to(self.device)
        return out

    def _all_users_of(self, me: int) -> torch.Tensor:
        allu = torch.arange(self.n_users, device=self._train[0].device)
        return allu[self._owner(allu) == me]

    # -- training -------------------------------------------------------------------------
    def train_epoch(self, epoch: int, evaluate: bool = False) -> int:
        cfg = self.cfg
        P, me = self.get_num_workers(), self.get_self_id()
        S = cfg.num_slices
        n = 0
        timer = self.metrics.timer
        for s in range(P):
            for k in range(S):
                slab = self.rot.get(k)
                gs = self.schedules[k].block_at(me, epoch, s) * S + k
                with timer.phase("compute"):
                    if cfg.xcd_blocks and self.device.type == "cpu" and cfg.cpu_threads > 1:
                        # CPU worker: the reference's threaded 2-D scheduler with its timer
                        r_, c_, v_, off, hoff = self.train.get_cells(gs)
                        budget = self.budget.budget_s if self.budget is not None else None
                        t0 = time.perf_counter()
                        n += MF.sgd_update_blocked(r_, c_, v_, off, self.W, slab, cfg.lr, cfg.lam, cfg.chunk,
                                                   host_off=hoff, threads=cfg.cpu_threads, time_budget=budget)
                        if self.budget is not None:
                            self.budget.compute_s += time.perf_counter() - t0
                    elif cfg.time_budget_ms > 0:
                        n += self._budget_step(gs, slab)
                    elif cfg.xcd_blocks:
                        r_, c_, v_, off, hoff = self.train.get_cells(gs)
                        win = MF.cell_windows(hoff, cfg.train_fraction, epoch) if cfg.train_fraction < 1.0 else None
                        n += MF.sgd_update_blocked(r_, c_, v_, off, self.W, slab, cfg.lr, cfg.lam, cfg.chunk,
                                                   self.bpx, host_off=hoff, variant=cfg.kernel_variant,
                                                   window=win, atomic=self.atomic)
                    else:
                        if cfg.train_fraction < 1.0:
                            raise ValueError("train_fraction < 1 needs the XCD-blocked layout")
                        n += MF.sgd_update(*self.train.get(gs, plain=True), self.W, slab, cfg.lr, cfg.lam, cfg.chunk)
                with timer.phase("rotate"):
                    self.rot.start(k, self.schedules[k].rotation_map(epoch, s))
        self.trained += n
        if cfg.time_budget_ms > 0 and cfg.tune_ratio > 0 and epoch == 0:
            total = torch.tensor([float(self.train.n)], dtype=torch.float64, device=self.device)
            if P > 1:
                self.comm.all_reduce(total)
            new = tune_budget(self, self.budget.compute_s, n, int(total.item()), P * S, cfg.tune_ratio, "sgd", epoch)
            self.budget.budget_s = new
            self.budget_history.append(new)
        return n

    def _budget_step(self, gs: int, slab: torch.Tensor) -> int:
        """Train slice ``gs`` for at most the step budget, in ``budget_pieces`` pieces
        that each train one window of every cell (see below)."""
        cfg = self.cfg
        if cfg.xcd_blocks:
            r_, c_, v_, off, hoff = self.train.get_cells(gs)
            sizes = [hoff[c + 1] - hoff[c] for c in range(len(hoff) - 1)]
        else:
            r_, c_, v_ = self.train.get(gs, plain=True)
            sizes = [r_.numel()]
        P = max(1, cfg.budget_pieces)
        # piece q covers [q*m/P, (q+1)*m/P) of every cell (an exact partition); the next
        # piece index persists per slice, so a cut visit resumes where it stopped
        def piece():
            q = self._cursor.get(gs, 0)
            self._cursor[gs] = (q + 1) % P
            starts = [(q * m) // P for m in sizes]
            L = [((q + 1) * m) // P - (q * m) // P for m in sizes]
            if cfg.xcd_blocks:
                return MF.sgd_update_blocked(r_, c_, v_, off, self.W, slab, cfg.lr, cfg.lam, cfg.chunk,
                                             self.bpx, host_off=hoff, variant=cfg.kernel_variant,
                                             window=(starts, L), atomic=self.atomic)
            a, m = starts[0], L[0]
            return MF.sgd_update(r_[a:a + m], c_[a:a + m], v_[a:a + m], self.W, slab, cfg.lr, cfg.lam,
                                 cfg.chunk) if m else 0

        items, _ = self.budget.run(piece for _ in range(P))
        return items

    def map_collective(self, reader: KeyValReader, context: Context) -> None:
        self.init_model(reader)
        start = self.start_iteration = self.resume()
        for ep in range(start, self.cfg.epochs):
            self.metrics.begin_iteration()
            t0 = time.perf_counter()
            n = self.train_epoch(ep)
            self.rot.wait_all()
            if torch.cuda.is_available() and self.device.type == "cuda":
                torch.cuda.synchronize()
            self.epoch_times.append(time.perf_counter() - t0)
            if self.cfg.kernel_variant == MF.FLOW_VARIANT and self.device.type == "cuda":
                MF.check_flow_errors(self.device)  # a timed-out wait / foreign XCD invalidates the epoch
            self._check_placement(ep)
            self.metrics.end_iteration("sgd", ep, trained=n, epoch_s=self.epoch_times[-1],
                                       updates_per_s=n / max(self.epoch_times[-1], 1e-12))
            if self.cfg.test_every and ((ep + 1) % self.cfg.test_every == 0 or ep == self.cfg.epochs - 1):
                self.rmse_history.append((ep + 1, *self._eval_ring(ep)))
            self.inject_fault(ep)
            if self._ckpt().due(ep):
                self.checkpoint(ep)
        if self.cfg.model_dir:
            self.save_models(self.cfg.model_dir)
        self.result = {"rmse": self.rmse_history, "epoch_s": self.epoch_times, "trained": self.trained,
                       "start_epoch": start, "placement": self.placement_events, "blocks_per_xcd": self.bpx,
                       "hot_items": self.hot_items, "atomic": self.atomic}

    def _check_placement(self, ep: int) -> None:
        """Once per epoch (the epoch is already synchronised): did a default XCD-blocked
        launch run blocks of one residue on two XCDs (csrc/mf_sgd.hip placement_check)?
        Then that epoch ran Hogwild across L2s (every rating still trained once) and the
        remaining epochs use a schedule that does not depend on the dispatcher's placement:
        the placed kernel (ranks <= 256) or the flat kernel (wide ranks; with train_fraction
        < 1 the windows need the blocked layout, so that run keeps it and only records the
        event)."""
        if self.device.type != "cuda" or not self.cfg.xcd_blocks:
            return
        got = MF.check_placement(self.device)
        if got["drained"]:
            self.placement_events.append((ep, "drained", got["drained"]))
        if not got["violation"] or self.cfg.kernel_variant == MF.PLACED_VARIANT:
            return
        import warnings

        if MF.storage_rank(self.cfg.rank, self.device) <= 256:
            self.cfg.kernel_variant = MF.PLACED_VARIANT
            what = "placed"
        elif self.cfg.train_fraction < 1.0 or self.cfg.time_budget_ms > 0:
            what = "blocked (kept: windowed training needs the XCD-blocked layout)"
        else:
            self.cfg.xcd_blocks = False
            what = "flat"
        self.placement_events.append((ep, "violation", what))
        warnings.warn(f"MF-SGD epoch {ep}: XCD placement check fired (blocks of one residue on two XCDs); "
                      f"switching to the {what} kernel")

    # -- checkpoint / resume / model output --------------------------------------------------
    def _ckpt(self):
        from ..utils.checkpoint import Checkpointer

        return Checkpointer(self.cfg.checkpoint_dir, self.comm, self.cfg.checkpoint_every)

    def _slab_items(self, gs: int) -> torch.Tensor:
        """Real item ids of the rows of global slice ``gs`` (padding rows dropped)."""
        lo = gs * self.ips
        hi = min(lo + self.ips, self.n_items)
        return self.item_perm[lo:hi] if hi > lo else self.item_perm[:0]

    def _resident(self, epoch: int):
        """(k, global slice, real item ids) of the slabs this rank holds when ``epoch`` starts."""
        S = self.cfg.num_slices
        block = self.schedule.block_at(self.get_self_id(), epoch, 0)
        return [(k, block * S + k, self._slab_items(block * S + k)) for k in range(S)]

    def checkpoint(self, ep: int) -> str:
        """After epoch ``ep``: W rows (global user ids) and the H slices resident for epoch
        ``ep + 1`` (global item ids), so any world size can resume."""
        from ..utils.checkpoint import tensor_table

        self.rot.wait_all()
        r = self.cfg.rank
        tabs = {"W": tensor_table(self.W[:, :r].contiguous(), self.users)}
        for k, gs, items in self._resident(ep + 1):
            tabs[f"H{k}"] = tensor_table(self.rot.slabs[k][: items.numel(), :r].contiguous(), items)
        extra = {"rmse": [list(x) for x in self.rmse_history], "trained": int(self.trained)}
        return self._ckpt().save(ep, tabs, extra=extra)

    def resume(self) -> int:
        got = self._ckpt().load_latest(device=self.device, rng=True)
        if got is None:
            return 0
        man, tabs = got
        ep = int(man["iteration"]) + 1
        r = self.cfg.rank

        def scatter(tab, n_rows):
            full = torch.zeros((n_rows, r), dtype=torch.float32, device=self.device)
            ids = torch.tensor(tab.ids, dtype=torch.long, device=self.device)
            full[ids] = tab.buffer.to(self.device, torch.float32)
            return full

        self.W[:, :r].copy_(scatter(tabs["W"], self.n_users)[self.users.to(self.device)])
        H = torch.zeros((self.n_items, r), dtype=torch.float32, device=self.device)
        for name, tab in tabs.items():
            if name.startswith("H") and len(tab):
                ids = torch.tensor(tab.ids, dtype=torch.long, device=self.device)
                H[ids] = tab.buffer.to(self.device, torch.float32)
        for k, gs, items in self._resident(ep):
            slab = self.rot.slabs[k]
            slab.zero_()
            slab[: items.numel(), :r] = H[items.to(self.device)]
        self.rmse_history = [tuple(x) for x in man["extra"].get("rmse", [])]
        self.trained = int(man["extra"].get("trained", 0))
        return ep

    def save_models(self, folder: str) -> None:
        """Reference saveModels (SGDCollectiveMapper.java:737-818): ``H-<worker>`` rows of
        the resident H slices, ``W-<worker>`` rows of the local users (``id : v1 .. vr``),
        ``evaluation`` (last test RMSE) from the master."""
        from ..utils.model_io import write_factor_rows, write_scalar

        self.rot.wait_all()
        me = self.get_self_id()
        ep = self.cfg.epochs
        items, rows = [], []
        for k, gs, it_ids in self._resident(ep):
            items.append(it_ids)
            rows.append(self.rot.slabs[k][: it_ids.numel(), : self.cfg.rank])
        write_factor_rows(f"{folder}/H-{me}", torch.cat(items), torch.cat(rows))
        write_factor_rows(f"{folder}/W-{me}", self.users, self.W[:, : self.cfg.rank])
        if self.is_master():
            last = self.rmse_history[-1][2] if self.rmse_history else float("nan")
            write_scalar(f"{folder}/evaluation", last)

    def _eval_ring(self, epoch: int) -> Tuple[float, float]:
        """RMSE with a ring tour (P steps, every slice visits every worker, slices end where
        they started, so the training schedule is unaffected)."""
        P, me, S = self.get_num_workers(), self.get_self_id(), self.cfg.num_slices
        dev = self.device
        acc = torch.zeros(4, dtype=torch.float64, device=dev)
        start = self.schedule.placement(epoch + 1, 0)  # placement the next epoch starts from
        ring = [(w + 1) % P for w in range(P)]
        for s in range(P):
            # block held by me after s ring steps from `start`
            holder = [(start[i] + s) % P for i in range(P)]
            block = holder.index(me)
            for k in range(S):
                slab = self.rot.get(k)
                gs = block * S + k
                tr = self.train.get(gs, plain=True)
                acc[0] += MF.sse(*tr, self.W, slab)
                acc[1] += tr[0].numel()
                if self.test is not None:
                    te = self.test.get(gs)
                    acc[2] += MF.sse(*te, self.W, slab)
                    acc[3] += te[0].numel()
                if P > 1:
                    self.rot.start(k, ring)
        self.rot.wait_all()
        if P > 1:
            self.comm.all_reduce(acc)
        a = acc.cpu().tolist()
        return math.sqrt(a[0] / max(a[1], 1)), (math.sqrt(a[2] / a[3]) if a[3] else float("nan"))


def run_sgd(comm, cfg: SGDConfig, n_users: int, n_items: int, train, test=None) -> dict:
    m = SGDCollectiveMapper(comm, cfg, n_users, n_items, train, test)
    m.run(KeyValReader([]))
    return m.result
