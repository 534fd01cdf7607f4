"""WDA-MDS: weighted deterministic-annealing SMACOF (Harp wdamds).

Reference: ml/java/.../wdamds/WDAMDSMapper.java:150-330 — distances (stored as
``short`` / Short.MAX_VALUE), weights and the V matrix are row-partitioned; X (n x d)
is allgathered. Annealing: T_max = max(delta) / sqrt(2d), T_min = min(0.01 T_max, 0.01),
T = alpha T_max, and while T > T_min: repeat SMACOF steps until the stress decrease falls
below ``threshold`` (max MAX_ITER=10000), then T *= alpha; finally a T = 0 stage.
Each SMACOF step: B(Z) (BCCalcTask.java:97-170: b_ij = -w_ij (delta_ij - sqrt(2d) T) /
d_ij(Z) when d_ij >= 1e-10 and delta_ij > sqrt(2d) T, b_ii = -sum_j b_ij), BC = B(Z) X,
then conjugate gradient on V X = BC (WDAMDSMapper.java:585-700: allgather p per CG
step, allreduce inner products, stop after ``cg_iter`` steps or when the X norm
changes by < 1e-2). Stress (StressCalcTask.java:72-96): sum_ij w_ij (delta_ij - diff -
d_ij)^2 over pairs with delta_ij >= diff, divided by sum w delta^2, allreduced.

MI355X design: every per-row-block kernel is GEMM-shaped — pairwise distances of the
local row block against all of X are one GEMM with the norm epilogue, B(Z) X is one
GEMM, V p is one GEMM (V = diag(W 1) - W built on the fly from the resident weight
block; no V file needed); X / p all-gathers and scalar allreduces are the only
communication, exactly the reference's pattern but with bulk collectives. On a HIP
device B(Z) X and the stress are single fused passes over the fp64 row blocks
(``csrc/mds.hip``: the embedding dimension is 2..4, so distances come straight from the
coordinates and B is never materialised).
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ..parallel.comm import Communicator
from .common import gather_rows, reduce_partials


@dataclass
class MDSConfig:
    d: int = 3
    alpha: float = 0.95
    threshold: float = 1e-6
    cg_iter: int = 20
    max_iter: int = 10000
    seed: int = 0
    checkpoint_dir: str = ""   # .hpt checkpoint after every ``checkpoint_every`` annealing stages
    checkpoint_every: int = 1
    model_dir: str = ""        # X written as <model_dir>/X (XFileUtil.storeXOnMaster format)


def _dist_block(Xr: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    G = Xr @ X.t()
    return ((Xr * Xr).sum(1)[:, None] + (X * X).sum(1)[None, :] - 2 * G).clamp_min(0).sqrt()


class _Rows:
    def __init__(self, comm, delta_rows, w_rows, row0):
        self.comm = comm
        self.D, self.W, self.row0 = delta_rows, w_rows, row0
        self.n_r, self.n = delta_rows.shape
        self.diag = torch.arange(self.n_r, device=delta_rows.device) + row0
        self.vdiag = w_rows.sum(1) - w_rows[torch.arange(self.n_r), self.diag]

    def gather(self, Xr):
        return gather_rows(self.comm, Xr) if self.comm.world_size > 1 else Xr

    def allsum(self, v: torch.Tensor) -> torch.Tensor:
        if self.comm.world_size == 1:
            return v
        return reduce_partials(self.comm, {"v": v.reshape(-1)})["v"].reshape(v.shape).to(v.dtype)

    def _native(self, X) -> bool:
        if self.D.device.type != "cuda":
            return False
        from ..ops import mds as mds_ops

        return X.shape[1] <= mds_ops.MAX_DIM and self.D.stride() == self.W.stride() and self.D.stride(1) == 1

    def stress(self, X, T, d):
        diff = math.sqrt(2.0 * d) * T if T > 1e-9 else 0.0
        if self._native(X):  # one fused pass (csrc/mds.hip)
            from ..ops import mds as mds_ops

            return mds_ops.stress_rows(self.D, self.W, self.row0, X, diff).sum()
        Dz = _dist_block(X[self.row0:self.row0 + self.n_r], X)
        Dz[torch.arange(self.n_r), self.diag] = 0
        m = (self.W != 0) & (self.D >= diff)
        dd = self.D - diff - Dz
        return (self.W * dd * dd * m).sum()

    def bc(self, X, T, d):
        diff = math.sqrt(2.0 * d) * T if T > 1e-9 else 0.0
        if self._native(X):  # B(Z) X without materialising B (csrc/mds.hip)
            from ..ops import mds as mds_ops

            return mds_ops.bc_rows(self.D, self.W, self.row0, X, diff)
        Dz = _dist_block(X[self.row0:self.row0 + self.n_r], X)
        ok = (self.W != 0) & (Dz >= 1e-10) & (self.D > diff)
        B = torch.where(ok, -self.W * (self.D - diff) / Dz.clamp_min(1e-10), torch.zeros_like(Dz))
        ar = torch.arange(self.n_r)
        B[ar, self.diag] = 0
        B[ar, self.diag] = -B.sum(1)
        return B @ X

    def vmul(self, Y):
        """(V Y) for the local rows: V = diag(sum_j w_ij, j != i) - W (off-diagonal)."""
        WY = self.W @ Y - self.W[torch.arange(self.n_r), self.diag][:, None] * Y[self.row0:self.row0 + self.n_r]
        return self.vdiag[:, None] * Y[self.row0:self.row0 + self.n_r] - WY


def _cg(rows: _Rows, X: torch.Tensor, BC: torch.Tensor, cg_iter: int) -> torch.Tensor:
    """CG on V X = BC starting from the current X (WDAMDSMapper.conjugateGradient)."""
    r0, n_r = rows.row0, rows.n_r
    R = BC - rows.vmul(X)
    Pl = R.clone()
    rtr = rows.allsum((R * R).sum().reshape(1))[0]
    for _ in range(cg_iter):
        Pf = rows.gather(Pl)
        AP = rows.vmul(Pf)
        ip = rows.allsum((AP * Pl).sum().reshape(1))[0]
        if float(ip) == 0:
            break
        a = rtr / ip
        s1 = float(X.norm())
        X = X + a * Pf
        s2 = float(X.norm())
        if abs(s2 - s1) < 1e-2:
            break
        R = R - a * AP
        rtr_new = rows.allsum((R * R).sum().reshape(1))[0]
        Pl = R + (rtr_new / rtr) * Pl
        rtr = rtr_new
    return X


def wda_mds(comm: Communicator, delta_rows: torch.Tensor, weight_rows: torch.Tensor, row0: int, n: int,
            cfg: MDSConfig, X0: Optional[torch.Tensor] = None) -> Dict[str, object]:
    """delta_rows / weight_rows: this worker's contiguous row block [n_r, n] starting at
    global row ``row0``. Returns the embedding X [n, d] (identical on all workers)."""
    dev = comm.device
    dt = torch.float64
    D, Wt = delta_rows.to(dev, dt), weight_rows.to(dev, dt)
    rows = _Rows(comm, D, Wt, row0)
    sums = reduce_partials(comm, {"s": (Wt * D * D).sum().reshape(1)})
    mx = reduce_partials(comm, {"m": D.max().reshape(1)}, op=_max())
    sum_sq, max_d = float(sums["s"][0]), float(mx["m"][0])
    if X0 is None:
        g = torch.Generator().manual_seed(cfg.seed)
        X = torch.rand((n, cfg.d), generator=g, dtype=dt).to(dev)
    else:
        X = X0.to(dev, dt).clone()
    t_max = max_d / math.sqrt(2.0 * cfg.d)
    t_min = min(0.01 * t_max, 0.01)
    T = cfg.alpha * t_max
    hist: List[Dict[str, float]] = []
    t0 = time.perf_counter()
    smacof = 0
    # checkpoint unit = one annealing stage: X is replicated (bit-identical on every
    # worker), so it is saved once and a restart may use any number of workers
    from ..runtime.mapper import inject_fault
    from ..utils.checkpoint import Checkpointer, tensor_table

    ck = Checkpointer(cfg.checkpoint_dir, comm, cfg.checkpoint_every)
    stage_no, start_stage = 0, 0
    got = ck.load_latest(device=dev)
    if got is not None:
        man, tabs = got
        ex = man["extra"]
        X = tabs["X"].buffer.to(dev, dt).reshape(n, cfg.d).clone()
        T, smacof, hist = float(ex["T"]), int(ex["smacof"]), list(ex["history"])
        stage_no = start_stage = int(man["iteration"]) + 1

    def stress(X, T):
        return float(rows.allsum(rows.stress(X, T, cfg.d).reshape(1))[0]) / sum_sq

    def stage(X, T):
        nonlocal smacof
        pre = stress(X, T)
        it = 0
        while True:
            BC = rows.bc(X, T, cfg.d)
            X = _cg(rows, X, BC, cfg.cg_iter)
            # keep every worker's copy of X bit-identical: rebuild from owned rows
            X = rows.gather(X[row0:row0 + rows.n_r])
            s = stress(X, T)
            it += 1
            smacof += 1
            if pre - s < cfg.threshold or it >= cfg.max_iter:
                return X, s
            pre = s

    def after_stage(X, T_next):
        nonlocal stage_no
        inject_fault(comm.rank, stage_no)
        if ck.due(stage_no):
            ck.save(stage_no, {"X": tensor_table(X)}, extra={"T": T_next, "smacof": smacof, "history": hist},
                    replicated=("X",))
        stage_no += 1

    s = hist[-1]["stress"] if hist else float("nan")
    while T > t_min:
        X, s = stage(X, T)
        hist.append({"T": T, "stress": s})
        T *= cfg.alpha
        after_stage(X, T)
    if not (hist and hist[-1]["T"] == 0.0):
        X, s = stage(X, 0.0)
        hist.append({"T": 0.0, "stress": s})
    if cfg.model_dir and comm.rank == 0:
        from ..utils.model_io import write_mds_points

        write_mds_points(os.path.join(cfg.model_dir, "X"), X)
    return {"X": X, "stress": s, "history": hist, "smacof_iters": smacof, "time_s": time.perf_counter() - t0,
            "start_stage": start_stage}


def _max():
    from ..core.combiner import Operation

    return Operation.MAX


def read_ids(path: str) -> List[Dict[str, int]]:
    """A wdamds ids file (tutorial/mds_data/ids/*_ids): per row block ``id height width
    id row_offset`` (tab separated; MDSDataSplit / DataFileUtil layout)."""
    out = []
    with open(path) as f:
        for ln in f:
            t = ln.split()
            if len(t) >= 5:
                out.append({"id": int(t[0]), "height": int(t[1]), "width": int(t[2]), "row0": int(t[4])})
    return out


def load_row_block(data_dir: str, kind: str, block: Dict[str, int]) -> torch.Tensor:
    """One row block of the reference's binary matrices (DataFileUtil.java:150-200:
    big-endian Java shorts, row-major ``height x width``): ``kind`` "distance" ->
    delta / Short.MAX_VALUE (fp64), "weight" -> the short value as fp64."""
    import numpy as np

    path = os.path.join(data_dir, f"{kind}_{block['id']}")
    a = np.fromfile(path, dtype=">i2")
    if a.size != block["height"] * block["width"]:
        raise ValueError(f"{path}: {a.size} shorts, expected {block['height']} x {block['width']}")
    a = a.reshape(block["height"], block["width"]).astype(np.float64)
    if kind == "distance":
        a /= 32767.0
    return torch.from_numpy(a)


def load_rows(data_dir: str, ids_dir: str, blocks: List[int]):
    """(delta rows, weight rows, first row) of the consecutive row blocks ``blocks``."""
    dist_ids = {b["id"]: b for b in read_ids(os.path.join(ids_dir, "distance_ids"))}
    w_ids = {b["id"]: b for b in read_ids(os.path.join(ids_dir, "weight_ids"))}
    D = torch.cat([load_row_block(data_dir, "distance", dist_ids[b]) for b in blocks])
    W = torch.cat([load_row_block(data_dir, "weight", w_ids[b]) for b in blocks])
    return D, W, dist_ids[blocks[0]]["row0"]


def quantize_distances(D: torch.Tensor) -> torch.Tensor:
    """The reference's storage format: short(delta / max * Short.MAX_VALUE), back to
    [0, 1] doubles."""
    q = torch.round(D / D.max() * 32767).to(torch.int16)
    return q.double() / 32767.0
