"""Matrix factorisation by cyclic coordinate descent (Harp MF-CCD).

Reference: ml/java/.../ccd/CCDMPCollectiveMapper.java:226-304 and CCDMPTask.java:67-125
— ratings are kept both by row and by column; W and H are stored per latent dimension;
an iteration is a row phase (every row r, every dimension t:
``z* = sum_j (res_j + w_rt h_jt) h_jt / (lambda |row| + sum_j h_jt^2)``, residuals
updated with the change) followed by the symmetric column phase; the factor tables
rotate between workers (two dymoro Rotators); ResTask recomputes residuals;
TestRMSETask reports test RMSE (allreduce).

MI355X design: each worker owns a row block of W (ratings regrouped by row) and a column
block of H (ratings regrouped by column). Instead of rotating per-dimension slabs, a
phase all-gathers the opposite factor once (one collective; the factors are small next
to HBM), then runs the coordinate updates for ALL owned rows at once: per dimension t
one segmented reduction over the nonzeros gives every row's numerator / denominator,
and one fused update rewrites the residuals. The update order over t matches the
reference's within-row order; rows are independent inside a phase, so results are
identical for any P.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..parallel.comm import Communicator
from .mf_common import gather_factors, rmse, shuffle_coo


@dataclass
class CCDConfig:
    rank: int = 16
    lam: float = 0.1
    iterations: int = 10
    seed: int = 0
    init_scale: float = -1.0  # <= 0: uniform [0, 1/sqrt(rank)) like CCDMPCollectiveMapper.java:200-213


def _phase(rows: torch.Tensor, cols: torch.Tensor, res: torch.Tensor, n_rows: int, F_own: torch.Tensor,
           F_other: torch.Tensor, lam: float, cnt: torch.Tensor) -> None:
    """Coordinate updates of F_own (rows local) against fixed F_other; res updated in place."""
    k = F_own.shape[1]
    down0 = lam * cnt
    for t in range(k):
        h = F_other[cols, t]
        w = F_own[rows, t]
        up = torch.zeros(n_rows, dtype=res.dtype, device=res.device)
        down = down0.clone()
        up.index_add_(0, rows, (res + w * h) * h)
        down.index_add_(0, rows, h * h)
        z = torch.where(down > 0, up / down.clamp_min(1e-300), F_own[:, t])
        delta = z - F_own[:, t]
        res -= delta[rows] * h
        F_own[:, t] = z


def train_ccd(comm: Communicator, u: torch.Tensor, i: torch.Tensor, v: torch.Tensor, n_users: int, n_items: int,
              cfg: CCDConfig, test: Optional[Tuple[torch.Tensor, ...]] = None) -> Dict[str, object]:
    P, me, dev = comm.world_size, comm.rank, comm.device
    dt = torch.float64 if dev.type == "cpu" else torch.float32
    uu, ui, uv = shuffle_coo(comm, u % P, u, i, v)
    iu, ii, iv = shuffle_coo(comm, i % P, u, i, v)
    my_users = torch.arange(me, n_users, P, device=dev)
    my_items = torch.arange(me, n_items, P, device=dev)
    ur, uc, uval = uu.to(dev) // P, ui.to(dev), uv.to(dev, dt)
    ir, ic, ival = ii.to(dev) // P, iu.to(dev), iv.to(dev, dt)
    cnt_u = torch.bincount(ur, minlength=my_users.numel()).to(dt)
    cnt_i = torch.bincount(ir, minlength=my_items.numel()).to(dt)
    g = torch.Generator().manual_seed(cfg.seed)
    sc = cfg.init_scale if cfg.init_scale > 0 else cfg.rank ** -0.5
    W0 = (torch.rand((n_users, cfg.rank), generator=g, dtype=torch.float64) * sc).to(dev, dt)
    H0 = (torch.rand((n_items, cfg.rank), generator=g, dtype=torch.float64) * sc).to(dev, dt)
    W = W0[my_users].clone()
    H = H0[my_items].clone()
    del W0, H0
    hist: List[Dict[str, float]] = []
    for it in range(cfg.iterations):
        t0 = time.perf_counter()
        Hf = gather_factors(comm, my_items, H, n_items)
        res = uval - (W[ur] * Hf[uc]).sum(1)  # ResTask
        _phase(ur, uc, res, my_users.numel(), W, Hf, cfg.lam, cnt_u)
        Wf = gather_factors(comm, my_users, W, n_users)
        res = ival - (H[ir] * Wf[ic]).sum(1)
        _phase(ir, ic, res, my_items.numel(), H, Wf, cfg.lam, cnt_i)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        rec = {"iter": it + 1, "time_s": time.perf_counter() - t0,
               "train_rmse": rmse(comm, (res * res).sum(), res.numel())}
        if test is not None:
            Hf = gather_factors(comm, my_items, H, n_items)
            tu, ti, tv = test
            mine = (tu % P) == me
            pred = (Wf[tu[mine].to(dev)] * Hf[ti[mine].to(dev)]).sum(1)
            rec["test_rmse"] = rmse(comm, ((pred - tv[mine].to(dev, dt)) ** 2).sum(), int(mine.sum()))
        hist.append(rec)
    return {"W": W, "H": H, "user_ids": my_users, "item_ids": my_items, "history": hist}
