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
from ..ops import ccd as C
from ..runtime.mapper import inject_fault
from .mf_common import FactorCheckpoint, gather_factors, rmse, save_factor_models, shuffle_coo


@dataclass
class CCDConfig:
    rank: int = 16
    lam: float = 0.1
    iterations: int = 10
    seed: int = 0
    init_scale: float = -1.0  # <= 0: uniform [0, 1/sqrt(rank)) like CCDMPCollectiveMapper.java:200-213
    checkpoint_dir: str = ""  # .hpt checkpoints of W / H (global row ids: any world size resumes)
    checkpoint_every: int = 0
    model_dir: str = ""       # final text dump W-<worker>, H-<worker> (``id : v1 .. vr``)
    mode: str = "allgather"   # "allgather": gather the opposite factor per phase; "rotation":
                              # rotate latent-dimension slices (memory O((m + n) r / P) per rank)
    slices_per_rank: int = 2  # rotation mode: dimension slices per rank (2 = transfer / compute overlap)
    residual_resync: int = 10  # allgather mode, one worker: a phase's exact residuals are carried to the
                               # other order by a fixed permutation; ResTask recomputes them every N
                               # iterations (1 = before every phase, the reference's schedule)


def train_ccd(comm: Communicator, u: torch.Tensor, i: torch.Tensor, v: torch.Tensor, n_users: int, n_items: int,
              cfg: CCDConfig, test: Optional[Tuple[torch.Tensor, ...]] = None) -> Dict[str, object]:
    if cfg.mode == "rotation":
        return train_ccd_rotation(comm, u, i, v, n_users, n_items, cfg, test)
    if cfg.mode != "allgather":
        raise ValueError(f"unknown CCD mode {cfg.mode}")
    P, me, dev = comm.world_size, comm.rank, comm.device
    dt = torch.float64 if dev.type == "cpu" else torch.float32
    uu, ui, uv = shuffle_coo(comm, u % P, u, i, v)
    iu, ii, iv = shuffle_coo(comm, i % P, u, i, v)
    my_users = torch.arange(me, n_users, P, device=dev)
    my_items = torch.arange(me, n_items, P, device=dev)

    def csr(rows_local, cols_global, vals, n_rows):
        o = torch.argsort(rows_local, stable=True)
        r = rows_local[o].to(torch.int32).contiguous()
        return r, C.row_ptr_of(r, n_rows), cols_global[o].to(torch.int32).contiguous(), vals[o].to(dt).contiguous(), o

    ur, uptr, uc, uval, ou = csr(uu.to(dev) // P, ui.to(dev), uv.to(dev), my_users.numel())
    ir, iptr, ic, ival, oi = csr(ii.to(dev) // P, iu.to(dev), iv.to(dev), my_items.numel())
    # One worker holds the same ratings in both orders: a phase leaves exact residuals
    # (every coordinate update rewrites them), so the other order is a gather through a
    # fixed permutation instead of a recompute over all nonzeros (ResTask: a 120-dim dot
    # product per rating, ~20 ms at 1e8 ratings). With P > 1 the row and column blocks of a
    # worker hold different ratings, so every phase recomputes (the reference's schedule).
    carry = P == 1 and cfg.residual_resync > 1
    if carry:
        inv = torch.empty_like(ou)
        inv[ou] = torch.arange(ou.numel(), device=ou.device)
        idx_t = torch.int32 if ou.numel() < 2**31 else torch.int64  # int32: half the index bytes per gather
        i2u = inv[oi].to(idx_t).contiguous()   # item-order position k holds user-order element i2u[k]
        inv[oi] = torch.arange(oi.numel(), device=oi.device)
        u2i = inv[ou].to(idx_t).contiguous()
        del inv
    del ou, oi
    g = torch.Generator().manual_seed(cfg.seed)
    sc = cfg.init_scale if cfg.init_scale > 0 else cfg.rank ** -0.5
    W0 = (torch.rand((n_users, cfg.rank), generator=g, dtype=torch.float64) * sc).to(dev, dt)
    H0 = (torch.rand((n_items, cfg.rank), generator=g, dtype=torch.float64) * sc).to(dev, dt)
    W = W0[my_users].contiguous()
    H = H0[my_items].contiguous()
    del W0, H0
    ulong, ilong = C.long_rows_of(uptr), C.long_rows_of(iptr)
    res_u = torch.empty_like(uval)
    res_i = torch.empty_like(ival)
    hist: List[Dict[str, float]] = []
    ck = FactorCheckpoint(comm, cfg.checkpoint_dir, cfg.checkpoint_every)
    start, hist = ck.resume({"W": (W, my_users, n_users), "H": (H, my_items, n_items)}, hist)
    for it in range(start, cfg.iterations):
        t0 = time.perf_counter()
        Hf = gather_factors(comm, my_items, H, n_items).contiguous()
        resync = not carry or it == start or (it - start) % cfg.residual_resync == 0
        if resync:
            C.residual(ur, uc, uval, W, Hf, res_u)  # ResTask
        else:
            torch.index_select(res_i, 0, u2i, out=res_u)
        C.phase(ur, uptr, uc, res_u, W, Hf, cfg.lam, ulong)
        Wf = gather_factors(comm, my_users, W, n_users).contiguous()
        if carry:
            torch.index_select(res_u, 0, i2u, out=res_i)
        else:
            C.residual(ir, ic, ival, H, Wf, res_i)
        C.phase(ir, iptr, ic, res_i, H, Wf, cfg.lam, ilong)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        rec = {"iter": it + 1, "time_s": time.perf_counter() - t0,
               "train_rmse": rmse(comm, (res_i.double() ** 2).sum(), res_i.numel())}
        if test is not None:
            Hf = gather_factors(comm, my_items, H, n_items)
            tu, ti, tv = test
            mine = (tu % P) == me
            pred = (Wf[tu[mine].to(dev)] * Hf[ti[mine].to(dev)]).sum(1)
            rec["test_rmse"] = rmse(comm, ((pred.double() - tv[mine].to(dev, torch.float64)) ** 2).sum(),
                                    int(mine.sum()))
        hist.append(rec)
        inject_fault(me, it)
        ck.maybe_save(it, {"W": (W, my_users), "H": (H, my_items)}, hist)
    if cfg.model_dir:
        save_factor_models(comm, cfg.model_dir, {"W": (W, my_users), "H": (H, my_items)})
    return {"W": W, "H": H, "start_iteration": start, "user_ids": my_users, "item_ids": my_items, "history": hist}


def train_ccd_rotation(comm: Communicator, u: torch.Tensor, i: torch.Tensor, v: torch.Tensor, n_users: int,
                       n_items: int, cfg: CCDConfig, test: Optional[Tuple[torch.Tensor, ...]] = None
                       ) -> Dict[str, object]:
    """Memory-scalable CCD: the reference's two Rotators (CCDMPCollectiveMapper.java:
    226-304, W and H tables split by latent dimension, rotated with
    ``RotationUtil`` orders of length 4 per iteration).

    The r latent dimensions are cut into S*P slices; a slice is a pair of dimension-slabs
    W_s [m, r/(SP)] and H_s [n, r/(SP)] over ALL users / items (owner-major row order, so
    a rank's own rows are one contiguous block). Ratings stay with their owner (row CSR by
    user, column CSR by item, residuals in both orders). An iteration is four ring tours of
    P steps x S slices: residual (res = v - sum_s W_s H_s^T, accumulated slice by slice),
    row phase (every owned row runs CD over the resident slice's dimensions), residual of
    the column copy, column phase. Slice k+1's transfer overlaps the kernels on slice k
    (two RCCL channels). A rank never holds more than S slices: (m + n) * r / P floats,
    instead of the allgather mode's full opposite factor."""
    from ..runtime.dymoro import DeviceRotator

    P, me, dev = comm.world_size, comm.rank, comm.device
    dt = torch.float64 if dev.type == "cpu" else torch.float32
    S = max(1, cfg.slices_per_rank)
    ns = S * P
    rs = -(-cfg.rank // ns)  # dims per slice (padded dims stay exactly zero)
    bu, bi = -(-n_users // P), -(-n_items // P)
    uu, ui, uv = shuffle_coo(comm, u % P, u, i, v)
    iu, ii, iv = shuffle_coo(comm, i % P, u, i, v)
    upos = lambda x: (x % P) * bu + x // P  # noqa: E731  owner-major row positions
    ipos = lambda x: (x % P) * bi + x // P  # noqa: E731
    n_mu = len(range(me, n_users, P))
    n_mi = len(range(me, n_items, P))

    def csr(rows_local, cols_pos, vals, n_rows):
        o = torch.argsort(rows_local, stable=True)
        r = rows_local[o].to(torch.int32).contiguous()
        return (r, C.row_ptr_of(r, n_rows), cols_pos[o].to(torch.int32).contiguous(),
                vals[o].to(dt).contiguous())

    ur, uptr, uc, uval = csr(uu.to(dev) // P, ipos(ui.to(dev)), uv.to(dev), n_mu)
    ir, iptr, ic, ival = csr(ii.to(dev) // P, upos(iu.to(dev)), iv.to(dev), n_mi)
    ulong, ilong = C.long_rows_of(uptr), C.long_rows_of(iptr)
    # initial factors: the allgather mode's draw (same generator order), split by dimension
    g = torch.Generator().manual_seed(cfg.seed)
    sc = cfg.init_scale if cfg.init_scale > 0 else cfg.rank ** -0.5
    W0 = torch.rand((n_users, cfg.rank), generator=g, dtype=torch.float64) * sc
    H0 = torch.rand((n_items, cfg.rank), generator=g, dtype=torch.float64) * sc
    slabs = []
    for k in range(S):
        gsl = me * S + k  # global slice initially resident here
        dims = list(range(gsl * rs, min((gsl + 1) * rs, cfg.rank)))
        Ws = torch.zeros((P * bu, rs), dtype=dt)
        Hs = torch.zeros((P * bi, rs), dtype=dt)
        if dims:
            Ws[upos(torch.arange(n_users))[:, None], torch.arange(len(dims))[None, :]] = W0[:, dims].to(dt)
            Hs[ipos(torch.arange(n_items))[:, None], torch.arange(len(dims))[None, :]] = H0[:, dims].to(dt)
        slabs += [Ws.to(dev), Hs.to(dev)]
    del W0, H0
    rot = DeviceRotator(comm, slabs, name="ccd-wh")
    ring = [(r + 1) % P for r in range(P)]
    res_u = torch.empty_like(uval)
    res_i = torch.empty_like(ival)
    mine_u = slice(me * bu, me * bu + n_mu)
    mine_i = slice(me * bi, me * bi + n_mi)

    def tour(fn):
        """P ring steps over the S resident slices (every slice visits every rank once and
        returns home)."""
        for step in range(P):
            for k in range(S):
                Ws, Hs = rot.get(2 * k), rot.get(2 * k + 1)
                fn(Ws, Hs)
                if P > 1:
                    rot.start(2 * k, ring)
                    rot.start(2 * k + 1, ring)
        rot.wait_all()

    hist: List[Dict[str, float]] = []
    # checkpoint: each rank's home slices (after every tour the slices are back home)
    from ..utils.checkpoint import Checkpointer, tensor_table

    ck = Checkpointer(cfg.checkpoint_dir, comm, cfg.checkpoint_every)
    start = 0
    got = ck.load_latest(device=dev, rng=True)
    if got is not None:
        man, tabs = got
        if man["world"] != P:
            raise ValueError(f"CCD rotation-mode resume needs the checkpoint's world size {man['world']}, got {P}")
        for k in range(S):
            rot.slabs[2 * k].copy_(tabs[f"W{k}"].buffer.to(dev))
            rot.slabs[2 * k + 1].copy_(tabs[f"H{k}"].buffer.to(dev))
        hist = list(man["extra"].get("history", []))
        start = int(man["iteration"]) + 1
    for it in range(start, cfg.iterations):
        t0 = time.perf_counter()
        res_u.copy_(uval)
        tour(lambda Ws, Hs: C.residual(ur, uc, res_u, Ws[mine_u], Hs, res_u))
        tour(lambda Ws, Hs: C.phase(ur, uptr, uc, res_u, Ws[mine_u], Hs, cfg.lam, ulong))
        res_i.copy_(ival)
        tour(lambda Ws, Hs: C.residual(ir, ic, res_i, Hs[mine_i], Ws, res_i))
        tour(lambda Ws, Hs: C.phase(ir, iptr, ic, res_i, Hs[mine_i], Ws, cfg.lam, ilong))
        if dev.type == "cuda":
            torch.cuda.synchronize()
        rec = {"iter": it + 1, "time_s": time.perf_counter() - t0,
               "train_rmse": rmse(comm, (res_i.double() ** 2).sum(), res_i.numel())}
        hist.append(rec)
        inject_fault(me, it)
        if ck.due(it):
            tabs = {}
            for k in range(S):
                tabs[f"W{k}"] = tensor_table(rot.slabs[2 * k])
                tabs[f"H{k}"] = tensor_table(rot.slabs[2 * k + 1])
            ck.save(it, tabs, extra={"history": list(hist), "mode": "rotation"})
    # assemble this rank's owned rows of the full factors (one tour; for the result only)
    W = torch.zeros((n_mu, ns * rs), dtype=dt, device=dev)
    H = torch.zeros((n_mi, ns * rs), dtype=dt, device=dev)
    for step in range(P):
        for k in range(S):
            gsl = ((me - step) % P) * S + k
            Ws, Hs = rot.get(2 * k), rot.get(2 * k + 1)
            W[:, gsl * rs:(gsl + 1) * rs] = Ws[mine_u]
            H[:, gsl * rs:(gsl + 1) * rs] = Hs[mine_i]
            if P > 1:
                rot.start(2 * k, ring)
                rot.start(2 * k + 1, ring)
    rot.wait_all()
    W, H = W[:, :cfg.rank].contiguous(), H[:, :cfg.rank].contiguous()
    my_users = torch.arange(me, n_users, P, device=dev)
    my_items = torch.arange(me, n_items, P, device=dev)
    if test is not None:
        Wf = gather_factors(comm, my_users, W, n_users)
        Hf = gather_factors(comm, my_items, H, n_items)
        tu, ti, tv = test
        mine = (tu % P) == me
        pred = (Wf[tu[mine].to(dev)] * Hf[ti[mine].to(dev)]).sum(1)
        hist[-1]["test_rmse"] = rmse(comm, ((pred.double() - tv[mine].to(dev, torch.float64)) ** 2).sum(),
                                     int(mine.sum()))
    if cfg.model_dir:
        save_factor_models(comm, cfg.model_dir, {"W": (W, my_users), "H": (H, my_items)})
    return {"W": W, "H": H, "start_iteration": start, "user_ids": my_users, "item_ids": my_items, "history": hist,
            "slab_floats_per_rank": sum(x.numel() for x in slabs)}
