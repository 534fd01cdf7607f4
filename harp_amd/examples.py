"""Collective examples with ``--verify`` and the collective micro-benchmark.

Reference: ml/java/.../examples/{ExamplesMain.java:59-166, AllReduce.java, AllGather.java,
BCast.java, Reduce.java, Rotate.java} (each mapper builds ``-partitions`` partitions of
``-elements`` values, repeats the op ``-iterations`` times with unique op names and, with
``-verify``, checks the result after every call; data types int/double/...), and
ml/java/.../benchmark/BenchmarkMapper.java:64-152 (allreduce / allgather loops over
``numPartitions`` partitions of ``bytesPerPartition`` bytes, total time logged).

Run (one process per GPU, RCCL):
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m harp_amd.examples \
        --op allreduce --elements 1000000 --partitions 4 --iterations 20 --verify
On CPU: ``--backend gloo`` (or ``python -m harp_amd.examples --spawn 2 ...``).

The benchmark reports algorithm bandwidth (bytes of the table / time) and the RCCL
"bus bandwidth" convention (allreduce x 2(P-1)/P, allgather x (P-1)/P) so numbers
compare with the xGMI link model in ``utils.metrics``.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from typing import Dict, List, Optional

import torch

from .core.combiner import ArrCombiner, Operation
from .core.table import PackedTable, Table
from .runtime.mapper import CollectiveMapper, Context, KeyValReader

_DTYPES = {"int": torch.int32, "long": torch.int64, "float": torch.float32, "double": torch.float64,
           "short": torch.int16, "byte": torch.int8}
OPS = ("allreduce", "allgather", "reduce", "bcast", "rotate", "regroup", "push_pull")


class ExampleMapper(CollectiveMapper):
    """One collective example; conf keys: op, elements, partitions, iterations, data_type,
    verify, packed (True: one device buffer per table -> single RCCL calls)."""

    def map_collective(self, reader: KeyValReader, context: Context) -> None:
        c = context.conf
        op = c.get("op", "allreduce")
        n, parts, iters = int(c.get("elements", 1000)), int(c.get("partitions", 1)), int(c.get("iterations", 10))
        dt = _DTYPES[c.get("data_type", "double")]
        verify = bool(c.get("verify", False))
        packed = bool(c.get("packed", True))
        P, me, dev = self.get_num_workers(), self.get_self_id(), self.device
        checks = 0
        t0 = time.perf_counter()
        times: List[float] = []
        if op == "allreduce":
            t = self._table(list(range(parts)), torch.ones((parts, n), dtype=dt, device=dev), packed)
            expected = float(P)
            for i in range(iters):
                s = time.perf_counter()
                assert self.allreduce("main", f"all-reduce-{i}", t)
                self._sync()
                times.append(time.perf_counter() - s)
                if verify:
                    checks += self._check(t, lambda pid: expected)
                    expected *= P
                    if dt.is_floating_point is False and expected > 2 ** 30:
                        t = self._table(list(range(parts)), torch.ones((parts, n), dtype=dt, device=dev), packed)
                        expected = float(P)
        elif op == "allgather":
            for i in range(iters):
                ids = [me + P * j for j in range(parts)]
                t = self._table(ids, self._fill(ids, n, dt, i), packed)
                s = time.perf_counter()
                assert self.allgather("main", f"all-gather-{i}", t)
                self._sync()
                times.append(time.perf_counter() - s)
                if verify:
                    if sorted(t.get_partition_ids()) != list(range(P * parts)):
                        raise RuntimeError(f"allgather: wrong ids {sorted(t.get_partition_ids())}")
                    checks += self._check(t, lambda pid: float(pid + i))
        elif op in ("reduce", "bcast"):
            root = 0
            for i in range(iters):
                if op == "reduce":
                    t = self._table(list(range(parts)), torch.full((parts, n), me + 1, dtype=dt, device=dev), packed)
                    s = time.perf_counter()
                    assert self.reduce("main", f"reduce-{i}", t, root)
                else:
                    ids = list(range(parts)) if me == root else []
                    t = self._table(ids, self._fill(ids, n, dt, i), packed)
                    s = time.perf_counter()
                    assert self.broadcast("main", f"bcast-{i}", t, root, bool(c.get("use_mst", False)))
                self._sync()
                times.append(time.perf_counter() - s)
                if verify:
                    if op == "reduce":
                        if me == root:
                            checks += self._check(t, lambda pid: float(P * (P + 1) // 2))
                        elif len(t) != 0:
                            raise RuntimeError("reduce: non-root table must be released")
                    else:
                        checks += self._check(t, lambda pid: float(pid + i))
        elif op == "rotate":
            ids = [me * parts + j for j in range(parts)]
            t = self._table(ids, self._fill(ids, n, dt, 0), packed)
            for i in range(iters):
                s = time.perf_counter()
                assert self.rotate("main", f"rotate-{i}", t, None)
                self._sync()
                times.append(time.perf_counter() - s)
                if verify:
                    owner = (me - (i + 1)) % P  # after i+1 ring steps we hold this worker's block
                    want = [owner * parts + j for j in range(parts)]
                    if sorted(t.get_partition_ids()) != want:
                        raise RuntimeError(f"rotate: got {sorted(t.get_partition_ids())} want {want}")
                    checks += self._check(t, lambda pid: float(pid))
        elif op == "regroup":
            for i in range(iters):
                ids = list(range(parts * P))
                t = self._table(ids, torch.ones((len(ids), n), dtype=dt, device=dev), packed)
                s = time.perf_counter()
                assert self.regroup("main", f"regroup-{i}", t, None)
                self._sync()
                times.append(time.perf_counter() - s)
                if verify:
                    if any(pid % P != me for pid in t.get_partition_ids()):
                        raise RuntimeError("regroup: partition at wrong owner")
                    checks += self._check(t, lambda pid: float(P))
        elif op == "push_pull":
            for i in range(iters):
                glob = Table(1, ArrCombiner(Operation.SUM))
                for pid in range(parts * P):
                    if pid % P == me:
                        glob.add(pid, torch.zeros(n, dtype=dt, device=dev))
                local = Table(2, ArrCombiner(Operation.SUM))
                for pid in range(parts * P):
                    local.add(pid, torch.ones(n, dtype=dt, device=dev))
                s = time.perf_counter()
                assert self.push("main", f"push-{i}", local, glob, None)
                back = Table(3, ArrCombiner(Operation.SUM))
                for pid in range(parts * P):
                    back.add(pid, torch.zeros(n, dtype=dt, device=dev))
                assert self.pull("main", f"pull-{i}", back, glob, True)
                self._sync()
                times.append(time.perf_counter() - s)
                if verify:
                    checks += self._check(back, lambda pid: float(P))
        else:
            raise ValueError(op)
        total = time.perf_counter() - t0
        nbytes = parts * n * torch.empty((), dtype=dt).element_size()
        steady = sorted(times[1:] or times)[len(times[1:] or times) // 2]
        bus = {"allreduce": 2 * (P - 1) / P, "allgather": (P - 1) / P * P}.get(op, 1.0)
        self.result = {"op": op, "workers": P, "elements": n, "partitions": parts, "iterations": iters,
                       "total_s": total, "median_s": steady, "bytes": nbytes,
                       "algbw_GBps": nbytes / steady / 1e9 if steady > 0 else None,
                       "busbw_GBps": nbytes * bus / steady / 1e9 if steady > 0 else None,
                       "verified_partitions": checks, "verify": verify}

    # -- helpers ------------------------------------------------------------------------
    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize()

    def _table(self, ids, rows: torch.Tensor, packed: bool) -> Table:
        comb = ArrCombiner(Operation.SUM)
        if packed:
            return PackedTable(ids, rows.contiguous(), combiner=comb)
        t = Table(0, comb)
        for k, pid in enumerate(ids):
            t.add(pid, rows[k].clone())
        return t

    def _fill(self, ids, n, dt, i):
        return torch.tensor([float(pid + i) for pid in ids], dtype=torch.float64).to(self.device, dt)[:, None] \
            .expand(len(ids), n).contiguous() if ids else torch.zeros((0, n), dtype=dt, device=self.device)

    def _check(self, t: Table, want) -> int:
        for p in t.get_partitions():
            v = p.get()
            e = want(p.id())
            if not bool((v.double() == e).all()):
                raise RuntimeError(f"verification failed on partition {p.id()}: want {e}, "
                                   f"got {v.double().unique()[:5].tolist()}")
        return len(t)


def run_example(comm, conf: Dict) -> Dict:
    from .runtime.launcher import run_mapper

    return run_mapper(comm, ExampleMapper, [], conf)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="Harp collective examples / micro-benchmark (ExamplesMain)")
    ap.add_argument("--op", "-op", default="allreduce", choices=OPS)
    ap.add_argument("--elements", "-elements", type=int, default=1000)
    ap.add_argument("--partitions", "-partitions", type=int, default=1)
    ap.add_argument("--iterations", "-iterations", type=int, default=100)
    ap.add_argument("--data-type", "-data", default="double", choices=sorted(_DTYPES))
    ap.add_argument("--verify", "-verify", action="store_true")
    ap.add_argument("--generic", action="store_true", help="per-partition tables (generic codec path)")
    ap.add_argument("--backend", default=None)
    ap.add_argument("--spawn", type=int, default=0, help="spawn N local workers instead of torchrun")
    a = ap.parse_args(argv)
    conf = {"op": a.op, "elements": a.elements, "partitions": a.partitions, "iterations": a.iterations,
            "data_type": a.data_type, "verify": a.verify, "packed": not a.generic}
    if a.spawn:
        from .runtime.launcher import launch

        res = launch(run_example, a.spawn, args=(conf,), backend=a.backend or "gloo")
        print(json.dumps(res[0]))
        return 0
    from .runtime.launcher import init_distributed, shutdown

    comm = init_distributed(a.backend)
    res = run_example(comm, conf)
    if comm.rank == 0:
        print(json.dumps(res))
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
