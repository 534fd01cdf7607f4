"""CollectiveMapper: the worker runtime API (Harp L4).

Reference: org/apache/hadoop/mapred/CollectiveMapper.java — users subclass it and
override ``setup`` / ``mapCollective(reader, ctx)`` / ``cleanup`` (:719-741); identity
accessors ``getSelfID/getMasterID/isMaster/getNumWorkers/getMinID/getMaxID``
(:317-364); the collectives ``barrier/broadcast/reduce/allgather/allreduce/regroup/
pull/push/rotate`` named by (contextName, operationName) (:374-606); events
``getEvent/waitEvent/sendEvent`` (:623-663); ``freeMemory/freeConn/logMemUsage/
logGCTime`` (:670-714); bootstrap = barrier("start-worker", "handshake") then
setup -> mapCollective -> cleanup (:751-790).

The (ctx, op) names are kept for API compatibility and label per-collective metrics;
RCCL's per-communicator issue order does the matching the reference's mailboxes did.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Any, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import torch

from ..core.partition import PartitionFunction, Partitioner
from ..core.table import Table
from ..parallel import collectives as C
from ..parallel.comm import Communicator
from ..parallel.events import Event, EventChannel, EventType
from ..utils.metrics import Metrics, table_nbytes

log = logging.getLogger("harp_amd.mapper")


class KeyValReader:
    """Yields (key, value) records of this worker's input split (value = file path),
    like MultiFileRecordReader (harp-daal-interface fileformat/MultiFileRecordReader.java)."""

    def __init__(self, records: Iterable[Tuple[Any, Any]] = ()):
        self._records = list(records)
        self._i = -1

    def next_key_value(self) -> bool:
        self._i += 1
        return self._i < len(self._records)

    def get_current_key(self):
        return self._records[self._i][0]

    def get_current_value(self):
        return self._records[self._i][1]

    def __iter__(self) -> Iterator[Tuple[Any, Any]]:
        return iter(self._records)

    def __len__(self) -> int:
        return len(self._records)


class Context:
    """Job context: configuration dict + progress hook (Hadoop Context analog)."""

    def __init__(self, conf: Optional[Dict[str, Any]] = None):
        self.conf = dict(conf or {})
        self.counters: Dict[str, float] = {}
        self.last_progress = time.monotonic()

    def get_configuration(self) -> Dict[str, Any]:
        return self.conf

    def progress(self) -> None:
        self.last_progress = time.monotonic()

    def get(self, key: str, default=None):
        return self.conf.get(key, default)

    def increment(self, name: str, v: float = 1) -> None:
        self.counters[name] = self.counters.get(name, 0) + v


class CollectiveMapper:
    """Base class of every application mapper."""

    def __init__(self, comm: Optional[Communicator] = None, metrics: Optional[Metrics] = None):
        self.comm = comm or Communicator()
        self.metrics = metrics or Metrics(rank=self.comm.rank, world=self.comm.world_size)
        self.metrics.world = self.comm.world_size
        if self.comm.device.type != "cuda":
            self.metrics.timer.use_events = False  # a CPU worker on a GPU host: wall-clock phases
        self.events = EventChannel(self.comm.rank, self.comm.world_size)
        self.result: Any = None

    # -- to override ------------------------------------------------------------------
    def setup(self, context: Context) -> None:
        pass

    def map_collective(self, reader: KeyValReader, context: Context) -> None:  # pragma: no cover
        raise NotImplementedError

    def cleanup(self, context: Context) -> None:
        pass

    # -- lifecycle (CollectiveMapper.run) ----------------------------------------------
    def run(self, reader: KeyValReader, context: Optional[Context] = None) -> Any:
        context = context or Context()
        t0 = time.perf_counter()
        if not self.barrier("start-worker", "handshake"):
            raise RuntimeError("Fail to do master barrier.")
        self.metrics.record("init", time.perf_counter() - t0)
        self.setup(context)
        try:
            self.map_collective(reader, context)
        finally:
            self.cleanup(context)
        return self.result

    # -- identity -----------------------------------------------------------------------
    def get_self_id(self) -> int:
        return self.comm.rank

    def get_master_id(self) -> int:
        return 0

    def is_master(self) -> bool:
        return self.comm.rank == 0

    def get_num_workers(self) -> int:
        return self.comm.world_size

    def get_min_id(self) -> int:
        return 0

    def get_max_id(self) -> int:
        return self.comm.world_size - 1

    @property
    def device(self) -> torch.device:
        return self.comm.device

    # -- collectives ------------------------------------------------------------------------
    def _timed(self, ctx: str, op: str, kind: str, fn, *a, **kw):
        """Run one collective, recording its bytes (this rank's table payload before the
        call; 0 on a 1-worker job, where nothing moves) and its stream time (HIP events
        around it on the current stream)."""
        nbytes = table_nbytes(a[0]) if a and isinstance(a[0], Table) and self.comm.world_size > 1 else 0
        with self.metrics.time_collective(kind, ctx, op, nbytes, self.comm.device):
            ok = fn(self.comm, *a, **kw)
        return ok

    def barrier(self, ctx: str, op: str) -> bool:
        return self._timed(ctx, op, "barrier", C.barrier)

    def broadcast(self, ctx: str, op: str, table: Table, root: int = 0, use_mst: bool = False) -> bool:
        return self._timed(ctx, op, "broadcast", C.broadcast, table, root, use_mst)

    def reduce(self, ctx: str, op: str, table: Table, root: int = 0) -> bool:
        return self._timed(ctx, op, "reduce", C.reduce, table, root)

    def allgather(self, ctx: str, op: str, table: Table) -> bool:
        return self._timed(ctx, op, "allgather", C.allgather, table)

    def allreduce(self, ctx: str, op: str, table: Table) -> bool:
        return self._timed(ctx, op, "allreduce", C.allreduce, table)

    def regroup(self, ctx: str, op: str, table: Table, partitioner: Optional[Partitioner] = None) -> bool:
        return self._timed(ctx, op, "regroup", C.regroup, table, partitioner)

    def regroup_aggregate(self, ctx: str, op: str, table: Table, partitioner, function: PartitionFunction) -> bool:
        return self._timed(ctx, op, "regroup_aggregate", C.regroup_aggregate, table, partitioner, function)

    def aggregate(self, ctx: str, op: str, table: Table, partitioner, function: PartitionFunction) -> bool:
        return self._timed(ctx, op, "aggregate", C.aggregate, table, partitioner, function)

    def pull(self, ctx: str, op: str, local: Table, global_table: Table, use_bcast: bool = True,
             sparse: bool = False, overwrite: bool = False) -> bool:
        if sparse:
            return self._timed(ctx, op, "pull", C.pull, local, global_table, use_bcast, sparse=True)
        if overwrite:
            return self._timed(ctx, op, "pull", C.pull, local, global_table, use_bcast, overwrite=True)
        return self._timed(ctx, op, "pull", C.pull, local, global_table, use_bcast)

    def push(self, ctx: str, op: str, local: Table, global_table: Table,
             partitioner: Optional[Partitioner] = None, sparse: bool = False) -> bool:
        if sparse:
            return self._timed(ctx, op, "push", C.push, local, global_table, partitioner, sparse=True)
        return self._timed(ctx, op, "push", C.push, local, global_table, partitioner)

    def rotate(self, ctx: str, op: str, table: Table, rotate_map=None) -> bool:
        return self._timed(ctx, op, "rotate", C.rotate, table, rotate_map)

    def join(self, ctx: str, op: str, dynamic: Table, partitioner, static: Table) -> bool:
        return self._timed(ctx, op, "join", C.join, dynamic, partitioner, static)

    # -- events -----------------------------------------------------------------------------
    def get_event(self) -> Optional[Event]:
        return self.events.get_event()

    def wait_event(self, timeout: Optional[float] = None) -> Optional[Event]:
        return self.events.wait_event(timeout)

    def send_event(self, event: Event) -> bool:
        return self.events.send_event(event)

    def send_message(self, ctx: str, target: int, body: Any) -> bool:
        return self.send_event(Event(EventType.MESSAGE, ctx, self.get_self_id(), target, body))

    # -- fault injection (tests) --------------------------------------------------
    def inject_fault(self, iteration: int) -> None:
        inject_fault(self.get_self_id(), iteration)

    # -- memory / logging ------------------------------------------------------------------
    def free_memory(self) -> None:
        from ..core.pool import ResourcePool

        ResourcePool.get().arrays.clean()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()

    def free_conn(self) -> None:
        """No pooled sockets exist (RCCL owns the links); kept for API compatibility."""

    def log_mem_usage(self) -> Dict[str, float]:
        info = self.metrics.memory()
        log.info("mem %s", info)
        return info

    def log_gc_time(self) -> None:
        import gc

        log.info("gc counts %s", gc.get_count())


def inject_fault(rank: int, iteration: int) -> None:
    """``HARP_FAULT="rank=R,iter=I,kind=exit|hang|raise[,attempt=A][,seconds=S]"`` makes
    rank R fail after iteration I of job attempt A (default 0, see ``launch(retries)``):
    ``exit`` kills the process (a dead peer), ``hang`` stops it for S seconds (a stuck
    peer: the others' collective watchdog fires), ``raise`` fails the mapper."""
    spec = os.environ.get("HARP_FAULT")
    if not spec:
        return
    kv = dict(x.split("=", 1) for x in spec.split(",") if "=" in x)
    if int(kv.get("rank", -1)) != rank or int(kv.get("iter", -1)) != iteration:
        return
    if int(kv.get("attempt", 0)) != int(os.environ.get("HARP_ATTEMPT", "0")):
        return
    kind = kv.get("kind", "exit")
    log.error("injected fault %s on rank %d at iteration %d", kind, rank, iteration)
    if kind == "exit":
        os._exit(17)
    if kind == "hang":
        time.sleep(float(kv.get("seconds", 3600)))
        return
    raise RuntimeError(f"injected fault at iteration {iteration}")
