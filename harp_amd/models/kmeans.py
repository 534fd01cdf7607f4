"""K-means with Harp's four interchangeable model-synchronisation strategies.

Reference workloads:
  * ml/java kmeans/regroupallgather (headline): per iteration threads compute local
    sums (CenCalcTask), merge them (CenMergeTask), then ``regroup`` -> average at the
    owner -> ``allgather`` (KMeansCollectiveMapper.java:107-211);
  * contrib kmeans {allreduce, regroup-allgather, broadcast-reduce, push-pull}
    (contrib/.../kmeans/common/KmeansMapCollective.java:30-270) and the DAAL variant's
    same four strategies (ml/daal/.../daal_kmeans/regroupallgather/
    KMeansDaalCollectiveMapper.java:435-530);
  * kmeans/rotation: centroid partitions rotate through the ring while each worker
    keeps its points (ml/java/.../kmeans/rotation/KMeansCollectiveMapper.java:106-228);
    here a true model-parallel variant: no worker ever holds all K centroids — the
    E-step keeps a running argmin over the resident block (kernel min-distance output),
    the M-step rotates partial-sum slabs back to each block's owner.

MI355X design: points live in HBM as padded bf16 rows (device-generated), one fused
MFMA kernel does E-step + argmin + accumulation (``ops.kmeans.assign``), the centroid
partial-sum table is a :class:`PackedTable` whose rows are the partitions, so each
strategy's collectives are single RCCL calls: allreduce -> ncclAllReduce; regroup ->
ncclReduceScatter (block partitioner = owner-contiguous slab), allgather ->
ncclAllGather; reduce + broadcast -> ncclReduce + ncclBroadcast; push/pull -> owner
all-to-all-v. Per-iteration phase times mirror the reference's Compute/Merge/Aggregate
log (KMeansCollectiveMapper.java:191-193).
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict, dataclass, field
from typing import List, Optional

import torch

from ..core.combiner import ArrCombiner, Operation
from ..core.partition import Partitioner
from ..core.table import PackedTable, Table
from ..ops import kmeans as K
from ..runtime.mapper import CollectiveMapper, Context, KeyValReader

STRATEGIES = ("allreduce", "regroup_allgather", "bcast_reduce", "push_pull", "rotation")


@dataclass
class KMeansConfig:
    num_points: int = 1000            # points on THIS worker (weak split is the caller's choice)
    num_centroids: int = 10
    dim: int = 100
    iterations: int = 10
    strategy: str = "regroup_allgather"
    seed: int = 1
    data_lo: float = 0.0
    data_hi: float = 1000.0
    variant: int = K.DEFAULT_VARIANT   # HIP kernel tiling variant
    objective_every: int = 1           # compute the objective every k iterations (0: never)
    checkpoint_dir: str = ""           # .hpt checkpoints of the centroid table (resume on restart)
    checkpoint_every: int = 0          # iterations between checkpoints (0: never)
    graph: bool = False                # replay the iteration's local kernels from HIP graphs


class BlockPartitioner(Partitioner):
    """Owner of row id = id // ceil(n/P): contiguous owner slabs, so a regroup of the
    packed centroid table is a reduce-scatter with no permutation."""

    def __init__(self, num_workers: int, n: int):
        super().__init__(num_workers)
        self.block = max(1, math.ceil(n / num_workers))

    def get_worker_id(self, partition_id: int) -> int:
        return min(int(partition_id) // self.block, self.num_workers - 1)


class KMeansCollectiveMapper(CollectiveMapper):
    """One K-means job on this worker. ``map_collective`` reads points from the input
    split (text rows ``x1 .. xd``, like contrib Utils.generateData) or generates them on
    the device when the split is empty."""

    def __init__(self, comm=None, config: Optional[KMeansConfig] = None, points: Optional[torch.Tensor] = None,
                 init_centroids: Optional[torch.Tensor] = None, metrics=None):
        super().__init__(comm, metrics)
        self.cfg = config or KMeansConfig()
        self._points_in = points
        self._init_c = init_centroids
        self.history: List[dict] = []

    # -- data -----------------------------------------------------------------------------
    def load_points(self, reader: KeyValReader) -> torch.Tensor:
        cfg = self.cfg
        if self._points_in is not None:
            return K.pack_points(self._points_in.float(), self.device)
        files = [v for _, v in reader]
        if files:
            rows = []
            for f in files:
                with open(f) as fh:
                    for line in fh:
                        vals = line.split()
                        if vals:
                            rows.append([float(v) for v in vals])
            return K.pack_points(torch.tensor(rows, dtype=torch.float32), self.device)
        return K.generate_points(cfg.num_points, cfg.dim, cfg.data_lo, cfg.data_hi,
                                 seed=cfg.seed * 7919 + 17, device=self.device,
                                 row0=self.get_self_id() * cfg.num_points)

    def initial_centroids(self) -> torch.Tensor:
        cfg = self.cfg
        if self._init_c is not None:
            return self._init_c.float().to(self.device)
        g = torch.Generator().manual_seed(cfg.seed)
        return (torch.rand((cfg.num_centroids, cfg.dim), generator=g) * (cfg.data_hi - cfg.data_lo)
                + cfg.data_lo).to(self.device)

    # -- main ------------------------------------------------------------------------------
    def map_collective(self, reader: KeyValReader, context: Context) -> None:
        cfg = self.cfg
        self.init_model(reader)
        start = self.start_iteration = self.resume() if cfg.checkpoint_dir else 0
        for it in range(start, cfg.iterations):
            self.step(it)
            self.inject_fault(it)
            if cfg.checkpoint_dir and cfg.checkpoint_every and (it + 1) % cfg.checkpoint_every == 0:
                self.checkpoint(it)
        self.finish()

    # -- checkpoint / resume ------------------------------------------
    def _ckpt(self):
        from ..utils.checkpoint import Checkpointer

        return Checkpointer(self.cfg.checkpoint_dir, self.comm, self.cfg.checkpoint_every)

    def checkpoint(self, it: int) -> str:
        """Write the model after iteration ``it`` as ``<dir>/it-<it>/`` + ``LATEST``.

        Replicated strategies save the [Kp, d] centroid table once (rank 0, replicated);
        the model-parallel rotation strategy saves each rank's resident centroid block
        (after P steps every block is back home) under its global centroid ids."""
        extra = {"objective": list(self.objective), "strategy": self.cfg.strategy}
        if self.cfg.strategy == "rotation":
            blk = self.c_rot.get(0)
            lo = self.get_self_id() * self.Kb
            t = PackedTable(list(range(lo, lo + self.Kb)), blk, table_id=0, combiner=self.sumop)
            return self._ckpt().save(it, {"centroids": t}, extra=extra)
        t = PackedTable(self.ids, self.c, table_id=0, combiner=self.sumop)
        return self._ckpt().save(it, {"centroids": t}, extra=extra, replicated=("centroids",))

    def resume(self) -> int:
        """Load the latest checkpoint if one exists (any world size); returns the first
        iteration to run."""
        got = self._ckpt().load_latest(device=self.device, rng=True)
        if got is None:
            return 0
        man, tabs = got
        c = tabs["centroids"]
        ids = c.ids if isinstance(c, PackedTable) else c.sorted_ids()
        buf = c.buffer if isinstance(c, PackedTable) else torch.stack([c[i] for i in ids])
        keep = [j for j, i in enumerate(ids) if i < self.cfg.num_centroids]  # padding rows carry nothing
        full = torch.zeros_like(self.c)
        full[torch.tensor([ids[j] for j in keep], dtype=torch.long, device=self.device)] = \
            buf[torch.tensor(keep, dtype=torch.long, device=buf.device)].to(self.device, torch.float32)
        self.c = full.contiguous()
        self.op = K.prepare(self.c[: self.cfg.num_centroids].contiguous(), self.dp, self.op)
        if self.cfg.strategy == "rotation":
            for a in ("c_rot", "s_rot"):
                if hasattr(self, a):
                    delattr(self, a)  # rebuilt from self.c (block me = rows [me*Kb, (me+1)*Kb))
        self.objective = list(man["extra"].get("objective", []))
        return int(man["iteration"]) + 1

    def init_model(self, reader: KeyValReader) -> None:
        """Load/generate points, create + broadcast the initial centroids."""
        cfg = self.cfg
        if cfg.strategy not in STRATEGIES:
            raise ValueError(f"unknown strategy {cfg.strategy}")
        dev = self.device
        self.X = self.load_points(reader)
        d, k = cfg.dim, cfg.num_centroids
        self.dp = self.X.shape[1]
        Kp = K.padded_k(k)
        self.ids = list(range(Kp))
        self.sumop = ArrCombiner(Operation.SUM)
        # centroid table [Kp, d] fp32: master creates it, chain-broadcast to all
        # (KMeansCollectiveMapper.java:295-313 broadcast("main","broadcast-centroids"))
        if self.is_master():
            c0 = torch.zeros((Kp, d), dtype=torch.float32, device=dev)
            c0[:k] = self.initial_centroids()
            cen = PackedTable(self.ids, c0, table_id=0, combiner=self.sumop)
        else:
            cen = PackedTable([], torch.zeros((0, d), dtype=torch.float32, device=dev), table_id=0,
                              combiner=self.sumop)
        if not self.broadcast("main", "broadcast-centroids", cen, 0, False):
            raise IOError("Fail to bcast")
        self.c = cen.buffer  # [Kp, d]
        if cfg.strategy == "rotation":  # room for every rank's padded block (resume / gather)
            kb = K.padded_k(math.ceil(k / self.get_num_workers()))
            if kb * self.get_num_workers() > Kp:
                self.c = torch.cat([self.c, self.c.new_zeros((kb * self.get_num_workers() - Kp, d))])
        self.op = K.prepare(self.c[:k].contiguous(), self.dp)
        self.sums = torch.zeros((Kp, self.dp), dtype=torch.float32, device=dev)
        self.part = BlockPartitioner(self.get_num_workers(), Kp)
        self.lab = torch.empty(self.X.shape[0], dtype=torch.int32, device=dev)
        self.objective = []

    def step(self, it: int) -> None:
        """One Lloyd iteration: fused assign+accumulate, model sync, operand prepare."""
        cfg = self.cfg
        if cfg.strategy == "rotation":
            return self._rotation_step(it)
        want_obj = cfg.objective_every > 0 and (it % cfg.objective_every == 0 or it == cfg.iterations - 1)
        if cfg.graph and not want_obj and cfg.strategy == "allreduce" and self.device.type == "cuda":
            return self._graph_step(it)
        timer = self.metrics.timer
        self.metrics.begin_iteration()
        t_it = time.perf_counter()
        with timer.phase("compute"):
            self.sums.zero_()
            _, obj = K.assign(self.X, self.op, sums=self.sums, labels=self.lab, want_objective=want_obj,
                              variant=cfg.variant)
        with timer.phase("sync"):
            self.c = self._sync(it, self.sums, self.c, self.part, self.ids, self.sumop, cfg.dim, cfg.num_centroids)
        with timer.phase("prepare"):
            self.op = K.prepare(self.c[:cfg.num_centroids], self.dp, self.op)
        if obj is not None:
            ot = obj.reshape(1).to(torch.float64)
            if self.get_num_workers() > 1:
                self.comm.all_reduce(ot)
            self.objective.append(float(ot.item()))
        self.history.append({"iter": it, "s": time.perf_counter() - t_it})
        self.metrics.end_iteration("kmeans", it, strategy=cfg.strategy, flops=self._iter_flops(),
                                   objective=self.objective[-1] if obj is not None else None)

    def _iter_flops(self) -> float:
        """Useful distance FLOPs of one iteration on this rank: 2 n K d (the GEMM's
        padding columns and rows excluded)."""
        return 2.0 * self.X.shape[0] * self.cfg.num_centroids * self.cfg.dim if getattr(self, "X", None) is not None else 0.0

    def _sum_table(self, sums: torch.Tensor) -> PackedTable:
        """The partial-sum table of the allreduce strategy, built once over the persistent
        ``sums`` buffer: its layout is verified across ranks on the first call only
        (``static_layout``), later calls are a single RCCL all-reduce."""
        t = getattr(self, "_sums_pt", None)
        if t is None or t.buffer is not sums:
            t = PackedTable(self.ids, sums, combiner=self.sumop)
            t.static_layout = True
            self._sums_pt = t
        return t

    # -- HIP-graph iteration ------------------------------------------------------------
    def _graph_step(self, it: int) -> None:
        """The allreduce iteration with its device work replayed from two HIP graphs:
        [zero sums, fused assign, label bucketing, row gather-sum] and [normalize, operand
        prepare]; only the RCCL all-reduce between them is issued eagerly. Every launch in
        the graphs writes fixed buffers (sums, labels, centroids, the kernel operand), so the
        captured pointers stay valid; the one workspace (bucketing) is allocated by a warm-up
        run before capture."""
        if getattr(self, "_graphs", None) is None:
            self._capture_graphs()
        timer = self.metrics.timer
        self.metrics.begin_iteration()
        t_it = time.perf_counter()
        with timer.phase("compute"):
            self._graphs[0].replay()
        with timer.phase("sync"):
            if not self.allreduce("main", f"allreduce-{it}", self._sum_table(self.sums)):
                raise IOError("allreduce failed")
        with timer.phase("prepare"):
            self._graphs[1].replay()
        self.history.append({"iter": it, "s": time.perf_counter() - t_it})
        self.metrics.end_iteration("kmeans", it, strategy="allreduce", hip_graph=True, flops=self._iter_flops())

    def _capture_graphs(self) -> None:
        cfg = self.cfg
        d, k = cfg.dim, cfg.num_centroids

        def local():
            self.sums.zero_()
            K.assign(self.X, self.op, sums=self.sums, labels=self.lab, want_objective=False, variant=cfg.variant)

        def post():
            K.normalize(self.sums, self.c, d)
            K.prepare(self.c[:k], self.dp, self.op)

        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            local()  # warm-up: allocates the bucketing workspace outside the graph
        torch.cuda.current_stream(self.device).wait_stream(side)
        graphs = []
        for fn in (local, post):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            graphs.append(g)
        self._graphs = graphs

    def finish(self) -> None:
        k = self.cfg.num_centroids
        if self.cfg.strategy == "rotation" and hasattr(self, "c_rot"):
            self.c = self._rotation_gather()
        self.centroids = self.c[:k].clone()
        self.labels = self.lab
        self.result = {"objective": self.objective, "centroids": self.centroids.cpu() if self.is_master() else None}

    # -- model synchronisation strategies ----------------------------------------------
    def _sync(self, it, sums, c, part, ids, sumop, d, k):
        s = self.cfg.strategy
        Kp = sums.shape[0]
        if s == "allreduce":
            t = self._sum_table(sums)
            if not self.allreduce("main", f"allreduce-{it}", t):
                raise IOError("allreduce failed")
            return K.normalize(t.buffer, c, d)
        if s == "regroup_allgather":
            t = PackedTable(ids, sums, combiner=sumop)
            t.static_layout = True
            if not self.regroup("main", f"regroup-{it}", t, part):
                raise IOError("regroup failed")
            mine = t.ids
            lo = mine[0] if mine else 0
            cs = c[lo:lo + len(mine)]
            K.normalize(t.buffer, cs, d)  # average at the owner (KMeansCollectiveMapper.java:170-183)
            ct = PackedTable(mine, cs.clone(), combiner=sumop)
            if not self.allgather("main", f"allgather-{it}", ct):
                raise IOError("allgather failed")
            return ct.buffer
        if s == "bcast_reduce":
            t = PackedTable(ids, sums, combiner=sumop)
            t.static_layout = True
            if not self.reduce("main", f"reduce-{it}", t, 0):
                raise IOError("reduce failed")
            if self.is_master():
                K.normalize(t.buffer, c, d)
                ct = PackedTable(ids, c, combiner=sumop)
            else:
                ct = PackedTable([], c[:0], combiner=sumop)
            if not self.broadcast("main", f"bcast-{it}", ct, 0, True):
                raise IOError("broadcast failed")
            return ct.buffer
        if s == "push_pull":
            # parameter-server sync (KMeansDaalCollectiveMapper.java:504-530): push the partial
            # sums to the owners of a distributed global table, average there, pull every
            # centroid back. Packed tables + cached comm plans: push = one all-to-all-v into
            # the owner slabs, pull = one all-gather (every worker wants every id).
            st = self._pp_tables(sums, c, part, ids)
            st["glob"].buffer.zero_()
            if not self.push("main", f"push-{it}", st["local"], st["glob"], part):
                raise IOError("push failed")
            K.normalize(st["glob"].buffer, st["cglob"].buffer, d)  # average at the owner
            st["pulled"].buffer.zero_()  # pull combines into the local rows (callers zero them)
            if not self.pull("main", f"pull-{it}", st["pulled"], st["cglob"], True):
                raise IOError("pull failed")
            c.copy_(st["pulled"].buffer)
            return c
        raise ValueError(s)

    def _pp_tables(self, sums, c, part, ids) -> dict:
        """Persistent packed tables of the push_pull strategy (static layouts)."""
        st = getattr(self, "_pp", None)
        if st is not None and st["sums"] is sums and st["c"] is c:
            return st
        me = self.get_self_id()
        mine = [i for i in ids if part.get_worker_id(i) == me]
        lo = mine[0] if mine else 0
        st = {"sums": sums, "c": c,
              "local": PackedTable(ids, sums, combiner=self.sumop),
              "glob": PackedTable(mine, torch.zeros((len(mine), sums.shape[1]), dtype=sums.dtype, device=sums.device),
                                  combiner=self.sumop),
              "cglob": PackedTable(mine, c[lo:lo + len(mine)], combiner=self.sumop),
              "pulled": PackedTable(ids, torch.zeros_like(c), combiner=self.sumop)}
        for t in ("local", "glob", "cglob", "pulled"):
            st[t].static_layout = True
        self._pp = st
        return st

    # -- model rotation (ml/java kmeans/rotation) ------------------------------------------
    def _rotation_init(self) -> None:
        """Worker r keeps centroid block r ([Kb, d], Kb a multiple of the kernel's 128-row
        tile) and never holds the whole model; the block and a partial-sum slab rotate on
        private channels (DeviceRotator) — the model-parallel K-means of
        kmeans/rotation/KMeansCollectiveMapper.java:106-228 (ExpTask E-step over the
        resident block with a running argmin, MaxTask M-step accumulation, rotate)."""
        from ..runtime.dymoro import DeviceRotator

        cfg = self.cfg
        P, me = self.get_num_workers(), self.get_self_id()
        self.Kb = K.padded_k(math.ceil(cfg.num_centroids / P))
        lo = me * self.Kb
        real = max(0, min(cfg.num_centroids - lo, self.Kb))
        blk = torch.zeros((self.Kb, cfg.dim), dtype=torch.float32, device=self.device)
        blk[:real] = self.c[lo:lo + real]
        self.c_rot = DeviceRotator(self.comm, [blk], name="km-c", metrics=self.metrics)
        self.s_rot = DeviceRotator(self.comm, [torch.zeros((self.Kb, self.dp), dtype=torch.float32,
                                                           device=self.device)], name="km-s", metrics=self.metrics)
        self.best_d = torch.empty(self.X.shape[0], dtype=torch.float32, device=self.device)
        self.md = torch.empty_like(self.best_d)
        self.best_l = torch.empty(self.X.shape[0], dtype=torch.int64, device=self.device)
        self.full_sums = torch.zeros((self.Kb * P, self.dp), dtype=torch.float32, device=self.device)

    def _rotation_step(self, it: int) -> None:
        cfg = self.cfg
        P, me = self.get_num_workers(), self.get_self_id()
        if not hasattr(self, "c_rot"):
            self._rotation_init()
        ring = [(r + 1) % P for r in range(P)]
        t_it = time.perf_counter()
        timer = self.metrics.timer
        self.metrics.begin_iteration()
        with timer.phase("compute"):
            self.best_d.fill_(float("inf"))
            self.best_l.fill_(0)
            for s in range(P):
                b = (me - s) % P  # block resident at step s (ring)
                real = max(0, min(cfg.num_centroids - b * self.Kb, self.Kb))
                cb = self.c_rot.get(0)
                if real:
                    op = K.prepare(cb[:real].contiguous(), self.dp)
                    K.assign(self.X, op, labels=self.lab, want_objective=False, variant=cfg.variant, min_dist=self.md)
                    better = self.md < self.best_d
                    self.best_d = torch.where(better, self.md, self.best_d)
                    self.best_l = torch.where(better, self.lab.long() + b * self.Kb, self.best_l)
                self.c_rot.start(0, ring)  # after P steps every block is home again
            from ..ops import segment

            self.full_sums.zero_()
            perm, start = segment.bucket_labels(self.best_l.to(torch.int32), self.full_sums.shape[0])
            segment.bucket_rowsum(self.X, perm, start, self.full_sums)
        with timer.phase("sync"):
            for s in range(P):
                b = (me - s) % P
                slab = self.s_rot.get(0)
                if s == 0:
                    slab.zero_()
                slab += self.full_sums[b * self.Kb:(b + 1) * self.Kb]
                self.s_rot.start(0, ring)
            slab = self.s_rot.get(0)  # block ``me``'s complete sums
            cb = self.c_rot.get(0)
            K.normalize(slab, cb, cfg.dim)
        want_obj = cfg.objective_every > 0 and (it % cfg.objective_every == 0 or it == cfg.iterations - 1)
        if want_obj:
            ot = self.best_d.double().clamp_min(0).sum().reshape(1)
            if P > 1:
                self.comm.all_reduce(ot)
            self.objective.append(float(ot.item()))
        self.history.append({"iter": it, "s": time.perf_counter() - t_it})
        self.metrics.end_iteration("kmeans", it, strategy="rotation", flops=self._iter_flops(),
                                   objective=self.objective[-1] if want_obj else None)

    def _rotation_gather(self) -> torch.Tensor:
        from .common import gather_rows

        cb = self.c_rot.get(0)
        return gather_rows(self.comm, cb)[: self.cfg.num_centroids]


def run_kmeans(comm, cfg: KMeansConfig, points=None, init_centroids=None) -> dict:
    """Launcher target: run one K-means job on this rank, return objective history."""
    m = KMeansCollectiveMapper(comm, cfg, points, init_centroids)
    m.run(KeyValReader([]))
    return {"objective": m.objective, "centroids": m.centroids.cpu(), "phases": m.metrics.timer.flush(),
            "start_iteration": m.start_iteration}
