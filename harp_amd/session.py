"""Python session API over numpy arrays (what the reference's py4j stub aimed at).

Reference: python/harp_session.py (``HarpSession(name)``, ``.com``), python/collectives/
collectives.py (``Collectives.barrier(ctx, op)``, ``broadcast(ctx, op, data: ndarray,
data_type: Type, partition_mode: PartitioningMode, bcast_worker_id, use_mst_bcast)``),
python/harp_constants.py (``Type`` BYTE..DOUBLE, ``PartitioningMode`` HETEROGENEOUS /
HOMOGENEOUS), python/context/{harp_context,data_reader}.py (``self_id``, ``name``,
``reader``, ``com``) and core/harp-boot (the py4j gateway). There the Java side was a
stub (``broadcast`` printed and returned False).

Here the session is native: it joins (or starts) the torch.distributed group directly —
no JVM, no gateway — and every collective takes / returns numpy arrays:

* HOMOGENEOUS: the array's first axis indexes partitions of equal shape -> a
  :class:`PackedTable` -> ONE RCCL (GPU) or gloo (CPU) call;
* HETEROGENEOUS: ``data`` is a dict {partition id: ndarray} of any shapes -> a generic
  :class:`Table` through the variable-length codec path.
"""
from __future__ import annotations

import enum
from typing import Dict, Iterator, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from .core.combiner import ArrCombiner, Operation
from .core.partition import Partitioner
from .core.table import PackedTable, Table
from .parallel import collectives as CL
from .parallel.comm import Communicator


class Type(enum.Enum):
    BYTE = 1
    SHORT = 2
    INT = 3
    FLOAT = 4
    LONG = 5
    DOUBLE = 6


class PartitioningMode(enum.Enum):
    HETEROGENEOUS = 1
    HOMOGENEOUS = 2


_NP = {Type.BYTE: np.int8, Type.SHORT: np.int16, Type.INT: np.int32, Type.FLOAT: np.float32, Type.LONG: np.int64,
       Type.DOUBLE: np.float64}

Data = Union[np.ndarray, Dict[int, np.ndarray]]


class DataReader:
    """(key, value) records of this worker's input split (python/context/data_reader.py)."""

    def __init__(self, records: Sequence[Tuple[object, object]] = ()):
        self._r = list(records)
        self._i = -1

    def next_key_val(self) -> bool:
        self._i += 1
        return self._i < len(self._r)

    @property
    def current_key(self):
        return self._r[self._i][0]

    @property
    def current_val(self):
        return self._r[self._i][1]

    def __iter__(self) -> Iterator[Tuple[object, object]]:
        return iter(self._r)


class Collectives:
    """numpy-facing collectives of one session (python/collectives/collectives.py)."""

    def __init__(self, comm: Communicator):
        self.comm = comm

    # -- conversions ----------------------------------------------------------------
    def _table(self, data: Data, dtype: Type, mode: PartitioningMode, op: Operation = Operation.SUM) -> Table:
        dev = self.comm.device
        comb = ArrCombiner(op)
        if mode == PartitioningMode.HOMOGENEOUS:
            arr = np.ascontiguousarray(np.asarray(data, dtype=_NP[dtype]))
            shape = arr.shape
            if arr.ndim == 1:
                arr = arr[None, :]
            t = PackedTable(list(range(arr.shape[0])), torch.from_numpy(arr).to(dev), combiner=comb)
            t.user_shape = shape
            return t
        t = Table(0, comb)
        for pid, a in (data or {}).items():
            t.add(int(pid), torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=_NP[dtype]))).to(dev))
        return t

    @staticmethod
    def _out(t: Table, mode: PartitioningMode) -> Data:
        if mode == PartitioningMode.HOMOGENEOUS and isinstance(t, PackedTable):
            out = t.buffer.detach().cpu().numpy()
            shape = getattr(t, "user_shape", None)
            return out.reshape(shape) if shape is not None and out.size == int(np.prod(shape)) else out
        return {p.id(): p.get().detach().cpu().numpy() for p in t.get_partitions()}

    # -- collectives ----------------------------------------------------------------
    def barrier(self, ctx_name: str = "main", op_name: str = "barrier") -> bool:
        return CL.barrier(self.comm)

    def broadcast(self, ctx_name: str, op_name: str, data: Optional[Data], data_type: Type = Type.DOUBLE,
                  partition_mode: PartitioningMode = PartitioningMode.HOMOGENEOUS, bcast_worker_id: int = 0,
                  use_mst_bcast: bool = False) -> Data:
        if partition_mode == PartitioningMode.HOMOGENEOUS:
            # non-roots need the shape: send it first (tiny)
            shp = self.comm.all_gather_ints(list(np.shape(data)) + [0] * (8 - np.ndim(data))
                                            if self.comm.rank == bcast_worker_id else [0] * 8)
            shape = [int(x) for x in shp[bcast_worker_id].tolist() if x]
            if self.comm.rank != bcast_worker_id:
                data = np.zeros(shape, dtype=_NP[data_type])
            t = self._table(data, data_type, partition_mode)
            if self.comm.world_size > 1:
                self.comm.broadcast(t.buffer, bcast_worker_id)
            return self._out(t, partition_mode)
        t = self._table(data if self.comm.rank == bcast_worker_id else {}, data_type, partition_mode)
        if not CL.broadcast(self.comm, t, bcast_worker_id, use_mst_bcast):
            raise IOError("broadcast failed")
        return self._out(t, partition_mode)

    def allreduce(self, ctx_name: str, op_name: str, data: Data, data_type: Type = Type.DOUBLE,
                  partition_mode: PartitioningMode = PartitioningMode.HOMOGENEOUS,
                  op: Operation = Operation.SUM) -> Data:
        t = self._table(data, data_type, partition_mode, op)
        if not CL.allreduce(self.comm, t):
            raise IOError("allreduce failed")
        return self._out(t, partition_mode)

    def reduce(self, ctx_name: str, op_name: str, data: Data, data_type: Type = Type.DOUBLE,
               partition_mode: PartitioningMode = PartitioningMode.HOMOGENEOUS, root: int = 0,
               op: Operation = Operation.SUM) -> Optional[Data]:
        t = self._table(data, data_type, partition_mode, op)
        if not CL.reduce(self.comm, t, root):
            raise IOError("reduce failed")
        return self._out(t, partition_mode) if self.comm.rank == root else None

    def allgather(self, ctx_name: str, op_name: str, data: Dict[int, np.ndarray],
                  data_type: Type = Type.DOUBLE) -> Dict[int, np.ndarray]:
        """Partitions of every worker (ids must be distinct or they are combined)."""
        t = self._table(data, data_type, PartitioningMode.HETEROGENEOUS)
        if not CL.allgather(self.comm, t):
            raise IOError("allgather failed")
        return self._out(t, PartitioningMode.HETEROGENEOUS)

    def regroup(self, ctx_name: str, op_name: str, data: Dict[int, np.ndarray], data_type: Type = Type.DOUBLE,
                partitioner: Optional[Partitioner] = None) -> Dict[int, np.ndarray]:
        t = self._table(data, data_type, PartitioningMode.HETEROGENEOUS)
        if not CL.regroup(self.comm, t, partitioner):
            raise IOError("regroup failed")
        return self._out(t, PartitioningMode.HETEROGENEOUS)

    def rotate(self, ctx_name: str, op_name: str, data: Dict[int, np.ndarray], data_type: Type = Type.DOUBLE,
               rotate_map=None) -> Dict[int, np.ndarray]:
        t = self._table(data, data_type, PartitioningMode.HETEROGENEOUS)
        if not CL.rotate(self.comm, t, rotate_map):
            raise IOError("rotate failed")
        return self._out(t, PartitioningMode.HETEROGENEOUS)


class HarpSession:
    """``HarpSession(name)``: joins the job's process group (torchrun env) or runs as a
    single worker; ``.com`` is the :class:`Collectives`, ``.ctx`` identity accessors."""

    def __init__(self, name: str = "harp", comm: Optional[Communicator] = None,
                 records: Sequence[Tuple[object, object]] = ()):
        import os

        if comm is None:
            if "WORLD_SIZE" in os.environ and not torch.distributed.is_initialized():
                from .runtime.launcher import init_distributed

                comm = init_distributed()
            else:
                comm = Communicator()
        self._name = name
        self.comm = comm
        self.collective_com = Collectives(comm)
        self._reader = DataReader(records)

    @property
    def name(self) -> str:
        return self._name

    @property
    def self_id(self) -> int:
        return self.comm.rank

    @property
    def num_workers(self) -> int:
        return self.comm.world_size

    @property
    def reader(self) -> DataReader:
        return self._reader

    @property
    def com(self) -> Collectives:
        return self.collective_com

    @property
    def ctx(self) -> "HarpSession":
        return self
