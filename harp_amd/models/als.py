"""Alternating least squares (implicit feedback and explicit), distributed + batch.

Reference: ml/daal/.../daal_als/ALSDaalCollectiveMapper.java:290-404 (DAAL
``implicit_als`` distributed training: step 1 each node computes the partial Y^T Y of
its item-factor block, step 2 the master sums them, steps 3/4 exchange the factor rows
each node needs (harpdaal_allgather) and solve the per-user normal equations; the item
half-step is symmetric; ``alpha`` confidence, ``lambda`` regularisation) and
daal_als_batch (single node).

Implicit model (Hu, Koren & Volinsky 2008): c_ui = 1 + alpha r_ui, p_ui = [r_ui > 0];
x_u = (Y^T Y + Y^T (C_u - I) Y + lambda I)^-1 Y^T C_u p_u.

MI355X design: ratings are regrouped once (all-to-all-v) by user owner and by item
owner; each half-step all-gathers the other side's factors (one collective, the model is
tiny next to 288 GB) and builds every owned row's f x f system at once: the Gram
term is one GEMM, the per-rating rank-1 terms are scatter-added in row blocks sized to a
memory budget, and the systems are solved by one batched Cholesky.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..parallel.comm import Communicator
from ..ops import als as OA
from ..runtime.mapper import inject_fault
from .mf_common import FactorCheckpoint, gather_factors, rmse, save_factor_models, shuffle_coo


@dataclass
class ALSConfig:
    factors: int = 10
    lam: float = 0.01
    alpha: float = 40.0
    iterations: int = 10
    implicit: bool = True
    weighted_lambda: bool = False  # lambda * n_u (ALS-WR) instead of lambda
    seed: int = 0
    block_bytes: int = 1 << 28
    wave_solve: bool = True   # fp32 GPU: build A / rhs, then the one-wave-per-system Cholesky kernel
                              # (False: the fused build + in-LDS solve kernel)
    checkpoint_dir: str = ""  # .hpt checkpoints of X / Y (global row ids: any world size resumes)
    checkpoint_every: int = 0
    model_dir: str = ""       # final text dump W-<worker> (users), H-<worker> (items)


def _sorted_rows(rows: torch.Tensor, n_rows: int):
    order = torch.argsort(rows, stable=True)
    crow = torch.zeros(n_rows + 1, dtype=torch.int64, device=rows.device)
    crow[1:] = torch.cumsum(torch.bincount(rows, minlength=n_rows), 0)
    return order, crow


def solve_rows(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n_rows: int, F: torch.Tensor,
               cfg: ALSConfig, crow: Optional[torch.Tensor] = None) -> torch.Tensor:
    """New factors for ``n_rows`` rows given ratings (rows sorted ascending) against the
    full opposite factor matrix F [n_cols, f]."""
    f = F.shape[1]
    dt = F.dtype
    dev = F.device
    if crow is None:  # rows are sorted: row starts by binary search (no histogram atomics)
        crow = torch.searchsorted(rows, torch.arange(n_rows + 1, dtype=rows.dtype, device=dev))
    eye = torch.eye(f, dtype=dt, device=dev)
    G = F.t() @ F if cfg.implicit else None
    out = torch.empty((n_rows, f), dtype=dt, device=dev)
    blk = max(1, int(cfg.block_bytes // (f * f * dt.itemsize * 2)))
    # native path: per-row normal equations in one HIP pass (csrc/als.hip), no per-rating
    # f x f outer products in HBM
    native = OA.available(F) and f <= OA.MAX_F and dt in (torch.float32, torch.float64)
    if native:
        F = F.contiguous()
        cols64 = cols.to(torch.int64).contiguous()
        vals_dt = vals.to(dt).contiguous()
        crow = crow.to(torch.int64).contiguous()
        blk = max(blk, 1 << 17)  # no per-rating intermediates: big blocks, fewer solver launches
        blk = min(blk, (2**32 - 1) // OA.THREADS)  # one workgroup per row: grid x threads < 2^32
    # torch path: the per-rating f x f outer products of a block live in memory at once, so
    # blocks are bounded by RATINGS (a row block of popular items holds millions of them);
    # at least one row per block
    per_rating = f * f * dt.itemsize
    max_ratings = max(1, int(cfg.block_bytes // per_rating))
    crow_h = crow.cpu() if not native else None
    bounds = []
    a = 0
    while a < n_rows:
        if native:
            b = min(n_rows, a + blk)
        else:
            lim = int(crow_h[a]) + max_ratings
            b = int(torch.searchsorted(crow_h, torch.tensor([lim], dtype=crow_h.dtype), right=True)[0]) - 1
            b = min(n_rows, max(b, a + 1), a + blk)
        bounds.append((a, b))
        a = b
    for a, b in bounds:
        if native:
            # build + Cholesky-solve every row's system in one kernel; rows whose system is
            # not SPD (info) send the block through rocSOLVER with the lstsq fallback
            scale = cfg.weighted_lambda or not cfg.implicit
            info = torch.empty(b - a, dtype=torch.int32, device=dev)
            if dt == torch.float32 and cfg.wave_solve:
                # build pass, then one wave per system (register Cholesky, no workgroup
                # barriers): the fused kernel's in-LDS solve was ~70 % of its time
                A = torch.empty((b - a, f, f), dtype=dt, device=dev)
                rhs = torch.empty((b - a, f), dtype=dt, device=dev)
                OA.normal_equations(crow, cols64, vals_dt, F, G, cfg.implicit, cfg.alpha, cfg.lam, scale, A, rhs, a)
                OA.chol_solve(A, rhs, out[a:b], info)
                if bool(info.any()):
                    out[a:b] = _solve(A, rhs)
                continue
            OA.normal_equations(crow, cols64, vals_dt, F, G, cfg.implicit, cfg.alpha, cfg.lam, scale, None, None, a,
                                X=out[a:b], info=info)
            if bool(info.any()):
                A = torch.empty((b - a, f, f), dtype=dt, device=dev)
                rhs = torch.empty((b - a, f), dtype=dt, device=dev)
                OA.normal_equations(crow, cols64, vals_dt, F, G, cfg.implicit, cfg.alpha, cfg.lam, scale, A, rhs, a)
                out[a:b] = _solve(A, rhs)
            continue
        s, e = int(crow[a]), int(crow[b])
        r = rows[s:e] - a
        Fc = F[cols[s:e]]
        v = vals[s:e].to(dt)
        A = torch.zeros((b - a, f, f), dtype=dt, device=dev)
        rhs = torch.zeros((b - a, f), dtype=dt, device=dev)
        if cfg.implicit:
            c = 1 + cfg.alpha * v
            w = c - 1
            A.index_add_(0, r, (w[:, None] * Fc)[:, :, None] * Fc[:, None, :])
            A += G
            rhs.index_add_(0, r, (c * (v > 0).to(dt))[:, None] * Fc)
        else:
            A.index_add_(0, r, Fc[:, :, None] * Fc[:, None, :])
            rhs.index_add_(0, r, v[:, None] * Fc)
        cnt = (crow[a + 1:b + 1] - crow[a:b]).to(dt)
        if cfg.weighted_lambda or not cfg.implicit:
            lam = cfg.lam * cnt.clamp_min(1)
        else:
            lam = torch.full((b - a,), cfg.lam, dtype=dt, device=dev)
        A += lam[:, None, None] * eye
        out[a:b] = _solve(A, rhs)
    return out


def _solve(A: torch.Tensor, rhs: torch.Tensor) -> torch.Tensor:
    L, info = torch.linalg.cholesky_ex(A)
    x = torch.cholesky_solve(rhs[:, :, None], L)[:, :, 0]
    bad = info != 0
    if bool(bad.any()):
        x[bad] = torch.linalg.lstsq(A[bad], rhs[bad][:, :, None]).solution[:, :, 0]
    return x


def implicit_loss(u, i, v, X, Y, cfg: ALSConfig) -> float:
    """Dense implicit objective (small problems / tests):
    sum_ui c_ui (p_ui - x_u.y_i)^2 + lambda (|X|^2 + |Y|^2)."""
    S = X @ Y.t()
    C = torch.ones_like(S)
    Pm = torch.zeros_like(S)
    C[u, i] = 1 + cfg.alpha * v.to(S.dtype)
    Pm[u, i] = (v > 0).to(S.dtype)
    return float((C * (Pm - S) ** 2).sum() + cfg.lam * ((X * X).sum() + (Y * Y).sum()))


def train_als(comm: Communicator, u: torch.Tensor, i: torch.Tensor, v: torch.Tensor, n_users: int, n_items: int,
              cfg: ALSConfig, test: Optional[Tuple[torch.Tensor, ...]] = None) -> Dict[str, object]:
    """``(u, i, v)``: this worker's share of the training triples (any split). Returns the
    local user / item factor blocks, their global ids, and per-iteration timings / RMSE."""
    P, me, dev = comm.world_size, comm.rank, comm.device
    dt = torch.float64 if dev.type == "cpu" else torch.float32
    uu, ui, uv = shuffle_coo(comm, u % P, u, i, v)
    iu, ii, iv = shuffle_coo(comm, i % P, u, i, v)
    my_users = torch.arange(me, n_users, P, device=dev)
    my_items = torch.arange(me, n_items, P, device=dev)
    # by-user system: local row = u // P
    ur = (uu.to(dev) // P)
    o, crow_u = _sorted_rows(ur, my_users.numel())
    ur, uc, uv = ur[o], ui.to(dev)[o], uv.to(dev)[o]
    ir = (ii.to(dev) // P)
    o, crow_i = _sorted_rows(ir, my_items.numel())
    ir, ic, iv = ir[o], iu.to(dev)[o], iv.to(dev)[o]
    g = torch.Generator().manual_seed(cfg.seed)
    Y0 = (torch.rand((n_items, cfg.factors), generator=g, dtype=torch.float64) * 0.1).to(dev, dt)
    Y = Y0[my_items]
    X = torch.zeros((my_users.numel(), cfg.factors), dtype=dt, device=dev)
    hist: List[Dict[str, float]] = []
    ck = FactorCheckpoint(comm, cfg.checkpoint_dir, cfg.checkpoint_every)
    start, hist = ck.resume({"X": (X, my_users, n_users), "Y": (Y, my_items, n_items)}, hist)
    for it in range(start, cfg.iterations):
        t0 = time.perf_counter()
        Yf = gather_factors(comm, my_items, Y, n_items)
        X = solve_rows(ur, uc, uv, my_users.numel(), Yf, cfg, crow_u)
        Xf = gather_factors(comm, my_users, X, n_users)
        Y = solve_rows(ir, ic, iv, my_items.numel(), Xf, cfg, crow_i)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        rec = {"iter": it + 1, "time_s": time.perf_counter() - t0}
        if test is not None:
            Yf = gather_factors(comm, my_items, Y, n_items)
            tu, ti, tv = test
            mine = (tu % P) == me
            pred = (Xf[tu[mine].to(dev)] * Yf[ti[mine].to(dev)]).sum(1)
            tvm = tv[mine].to(dev, dt)
            rec["test_rmse"] = rmse(comm, ((pred - tvm) ** 2).sum(), int(mine.sum()))
            if cfg.implicit:
                # the reference's implicit-ALS test error (daal_als/ComputeRMSE.java:97-104):
                # preference 1 for every test pair, weighted by the confidence 1 + alpha r
                rec["test_conf_rmse"] = rmse(comm, (((1.0 - pred) ** 2) * (1.0 + cfg.alpha * tvm)).sum(),
                                             int(mine.sum()))
        hist.append(rec)
        inject_fault(me, it)
        ck.maybe_save(it, {"X": (X, my_users), "Y": (Y, my_items)}, hist)
    if cfg.model_dir:
        save_factor_models(comm, cfg.model_dir, {"W": (X, my_users), "H": (Y, my_items)})
    return {"X": X, "Y": Y, "start_iteration": start, "user_ids": my_users, "item_ids": my_items, "history": hist}


def train_als_batch(u, i, v, n_users, n_items, cfg: ALSConfig):
    """daal_als_batch: the single-node variant (same solver, no communication)."""
    return train_als(Communicator(), u, i, v, n_users, n_items, cfg)
