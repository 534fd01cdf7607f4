"""Key-addressed partition tables (Harp ``Table``) and the packed dense fast path.

Reference semantics (partition/Table.java:28-193):
  * ``Table(tableID, combiner)``;
  * ``addPartition(p)`` inserts when the id is absent, otherwise
    ``combiner.combine(existing, p)`` **in place** and ``p`` is not inserted (:116-128);
  * ``insertPartition`` / ``getPartition`` / ``removePartition`` / ``release`` / ``free``.

MI355X design: a generic :class:`Table` holds ``Partition`` objects whose payloads are
torch tensors (HBM or host), typed :class:`~harp_amd.core.arrays.Array` views, Writables
or KV maps. Every headline workload uses *same-shaped dense numeric partitions*
(centroid blocks, H slices, cross-products), so :class:`PackedTable` stores them as ONE
contiguous device buffer ``[num_partitions, *part_shape]`` plus an id index; each Harp
collective on a packed table becomes a single RCCL call whose reduction op is the
combiner (SURVEY §7.2 rule 1).
"""
from __future__ import annotations

import itertools
import math
from typing import Any, Dict, Iterable, Iterator, List, Optional, Sequence

import torch

from .combiner import ArrCombiner, Operation, PartitionCombiner, PartitionStatus
from .partition import Partition

_table_ids = itertools.count()


class Table:
    def __init__(self, table_id: int | None = None, combiner: PartitionCombiner | None = None):
        self.table_id = next(_table_ids) if table_id is None else int(table_id)
        self.combiner = combiner if combiner is not None else ArrCombiner(Operation.SUM)
        self._parts: Dict[int, Partition] = {}

    # -- Harp API -------------------------------------------------------------
    def get_table_id(self) -> int:
        return self.table_id

    def get_combiner(self) -> PartitionCombiner:
        return self.combiner

    def get_num_partitions(self) -> int:
        return len(self._parts)

    def get_partition_ids(self) -> List[int]:
        return list(self._parts.keys())

    def get_partitions(self) -> List[Partition]:
        return list(self._parts.values())

    def add_partition(self, partition: Partition | None) -> PartitionStatus:
        if partition is None:
            return PartitionStatus.ADD_FAILED
        cur = self._parts.get(partition.id())
        if cur is None:
            return self.insert_partition(partition)
        return self.combiner.combine(cur.get(), partition.get())

    def insert_partition(self, partition: Partition) -> PartitionStatus:
        self._parts[partition.id()] = partition
        return PartitionStatus.ADDED

    def get_partition(self, partition_id: int) -> Optional[Partition]:
        return self._parts.get(int(partition_id))

    def remove_partition(self, partition_id: int) -> Optional[Partition]:
        return self._parts.pop(int(partition_id), None)

    def is_empty(self) -> bool:
        return not self._parts

    def release(self) -> None:
        for p in self._parts.values():
            p.release()
        self._parts.clear()

    def free(self) -> None:
        for p in self._parts.values():
            p.free()
        self._parts.clear()

    # -- pythonic helpers -----------------------------------------------------------
    def add(self, partition_id: int, data: Any) -> PartitionStatus:
        return self.add_partition(Partition(partition_id, data))

    def __len__(self) -> int:
        return len(self._parts)

    def __contains__(self, pid: int) -> bool:
        return int(pid) in self._parts

    def __iter__(self) -> Iterator[Partition]:
        return iter(list(self._parts.values()))

    def __getitem__(self, pid: int) -> Any:
        return self._parts[int(pid)].get()

    def items(self):
        return [(p.id(), p.get()) for p in self._parts.values()]

    def sorted_ids(self) -> List[int]:
        return sorted(self._parts)

    def is_packed(self) -> bool:
        return False

    def empty_like(self) -> "Table":
        return Table(self.table_id, self.combiner)

    def __repr__(self) -> str:
        return f"{type(self).__name__}(id={self.table_id}, partitions={len(self._parts)}, combiner={self.combiner})"


class PackedTable(Table):
    """Dense table: ``buffer[i]`` is the payload of partition ``ids[i]``.

    Partitions returned by :meth:`get_partition` are views into the buffer, so in-place
    updates by the application are seen by the collectives with no packing step.
    Adding a partition whose id is absent appends (re-allocates the slab); adding an
    existing id combines in place exactly like :class:`Table`.
    """

    def __init__(self, ids: Sequence[int] | torch.Tensor, buffer: torch.Tensor,
                 table_id: int | None = None, combiner: PartitionCombiner | None = None):
        super().__init__(table_id, combiner)
        ids_l = [int(i) for i in (ids.tolist() if isinstance(ids, torch.Tensor) else ids)]
        if buffer.shape[0] != len(ids_l):
            raise ValueError("buffer rows must equal number of ids")
        if len(set(ids_l)) != len(ids_l):
            raise ValueError("duplicate partition ids")
        self.buffer = buffer
        self._ids = ids_l
        self._row = {pid: i for i, pid in enumerate(ids_l)}
        self.version = 0  # bumped on every id-layout change (cached comm plans key on it)
        self._ids_hash = None
        self._rebuild_parts()

    # construction helpers
    @classmethod
    def zeros(cls, ids: Sequence[int], part_shape: Sequence[int] | int, dtype=torch.float32,
              device="cpu", combiner: PartitionCombiner | None = None, table_id: int | None = None):
        shape = (part_shape,) if isinstance(part_shape, int) else tuple(part_shape)
        buf = torch.zeros((len(ids),) + shape, dtype=dtype, device=device)
        return cls(list(ids), buf, table_id=table_id, combiner=combiner)

    @classmethod
    def from_table(cls, table: Table) -> "PackedTable":
        ids = table.sorted_ids()
        parts = [table[i] for i in ids]
        if not parts:
            raise ValueError("cannot pack an empty table without a part shape")
        buf = torch.stack([p if isinstance(p, torch.Tensor) else p.tensor for p in parts])
        return cls(ids, buf, table.table_id, table.combiner)

    # Partition views are created lazily: the dense collectives move ``buffer`` as one
    # RCCL call and never touch per-partition objects (building 10^4 tensor views per call
    # cost ~15 ms of host time per K-means iteration at K = 1e4).
    @property
    def _parts(self) -> Dict[int, Partition]:
        if self._parts_cache is None:
            self._parts_cache = {pid: Partition(pid, self.buffer[i]) for i, pid in enumerate(self._ids)}
        return self._parts_cache

    @_parts.setter
    def _parts(self, value) -> None:
        self._parts_cache = value

    def _rebuild_parts(self) -> None:
        self._parts_cache = None
        self.version = getattr(self, "version", 0) + 1
        self._ids_hash = None

    def ids_hash(self) -> int:
        """crc32 of the id list (int64 little-endian), cached per layout version."""
        if self._ids_hash is None:
            import zlib

            import numpy as np

            self._ids_hash = zlib.crc32(np.asarray(self._ids, dtype=np.int64).tobytes()) & 0x7FFFFFFF
        return self._ids_hash

    def __len__(self) -> int:
        return len(self._ids)

    def get_num_partitions(self) -> int:
        return len(self._ids)

    def get_partition_ids(self) -> List[int]:
        return list(self._ids)

    def __contains__(self, pid) -> bool:
        return int(pid) in self._row

    def is_empty(self) -> bool:
        return not self._ids

    def sorted_ids(self) -> List[int]:
        return sorted(self._ids)

    @property
    def ids(self) -> List[int]:
        return list(self._ids)

    @property
    def part_shape(self):
        return tuple(self.buffer.shape[1:])

    def row_of(self, pid: int) -> int:
        return self._row[int(pid)]

    def is_packed(self) -> bool:
        return True

    def insert_partition(self, partition: Partition) -> PartitionStatus:
        data = partition.get()
        t = data if isinstance(data, torch.Tensor) else getattr(data, "tensor", None)
        if t is None or t.numel() != math.prod(self.part_shape):
            return PartitionStatus.ADD_FAILED
        t = t.reshape(self.part_shape).to(device=self.buffer.device, dtype=self.buffer.dtype)
        self.buffer = torch.cat([self.buffer, t.unsqueeze(0)], 0)
        self._ids.append(partition.id())
        self._row[partition.id()] = len(self._ids) - 1
        self._rebuild_parts()
        return PartitionStatus.ADDED

    def remove_partition(self, partition_id: int) -> Optional[Partition]:
        pid = int(partition_id)
        if pid not in self._row:
            return None
        i = self._row[pid]
        p = Partition(pid, self.buffer[i].clone())
        keep = [j for j in range(len(self._ids)) if j != i]
        self.buffer = self.buffer[keep] if keep else self.buffer[:0]
        self._ids = [self._ids[j] for j in keep]
        self._row = {q: j for j, q in enumerate(self._ids)}
        self._rebuild_parts()
        return p

    def set_contents(self, ids: Sequence[int], buffer: torch.Tensor) -> None:
        ids_l = [int(i) for i in ids]
        if buffer.shape[0] != len(ids_l):
            raise ValueError("buffer rows must equal number of ids")
        self.buffer = buffer
        self._ids = ids_l
        self._row = {pid: i for i, pid in enumerate(ids_l)}
        self._rebuild_parts()

    def release(self) -> None:
        self.set_contents([], self.buffer[:0])

    def free(self) -> None:
        self.release()

    def layout_signature(self) -> tuple:
        return (tuple(self._ids), self.part_shape, str(self.buffer.dtype))

    def empty_like(self) -> "PackedTable":
        return PackedTable([], self.buffer[:0].clone(), self.table_id, self.combiner)

    def to_table(self) -> Table:
        t = Table(self.table_id, self.combiner)
        for i, pid in enumerate(self._ids):
            t.insert_partition(Partition(pid, self.buffer[i].clone()))
        return t
