"""Key-value tables (Harp ``keyval`` package).

Reference (core/harp-collective/.../keyval/): tables whose partitions are hash maps.
``Int2IntKVTable`` maps key -> partition id = key (Int2IntKVTable.java:207-209 style),
``Long2DoubleKVTable`` uses ``(int) key`` (:155), ``Key2ValKVTable`` uses ``hashCode()``
(:219-221); ``addKeyVal`` creates the partition on demand and combines values with a
``Type{Int,Long,Double}Combiner`` / ``ValCombiner``; ``getVal`` returns the partition
map's default (``Integer.MIN_VALUE`` for int maps) when absent
(Int2IntKVPartition.java:31-166; test/.../keyval/*KVPartitionTest.java). Partition-level
combine merges the maps entry by entry.

Two representations:
  * dict-backed partitions (Writable, wire-encodable) for irregular host data such as
    word counts and graph messages — the reference's model;
  * :class:`TensorKVPartition` — sorted int64 keys + a value tensor on the device,
    combined with ``torch.unique`` + ``scatter_reduce`` (no per-key host work), for
    GPU-resident sparse models (LDA word-topic counts, graph vertex values).
"""
from __future__ import annotations

import enum
from typing import Any, Callable, Dict, Iterable, Optional, Tuple

import torch

from .combiner import Operation, PartitionCombiner, PartitionStatus
from .partition import Partition
from .table import Table
from .writable import DataInput, DataOutput, Writable, class_name, writable_class

INT_MIN = -(2 ** 31)
LONG_MIN = -(2 ** 63)


class ValStatus(enum.Enum):
    ADDED = 0
    ADD_FAILED = 1
    COMBINED = 2
    COMBINE_FAILED = 3


def _apply(op: Operation, a, b):
    if op is Operation.SUM:
        return a + b
    if op is Operation.MINUS:
        return a - b
    if op is Operation.MULTIPLY:
        return a * b
    if op is Operation.MAX:
        return a if a >= b else b
    if op is Operation.MIN:
        return a if a <= b else b
    raise ValueError(op)


class TypeIntCombiner:
    """Combines primitive values (keyval/TypeIntCombiner.java etc.)."""

    def __init__(self, op: Operation = Operation.SUM):
        self.op = Operation(op)

    def combine(self, cur, new):
        return _apply(self.op, cur, new)


TypeLongCombiner = TypeIntCombiner
TypeDoubleCombiner = TypeIntCombiner


class ValCombiner:
    """Combines object values (keyval/ValCombiner.java): ``combine(cur, new) -> ValStatus``
    mutating ``cur`` in place, or return a new value via :meth:`merge`."""

    def combine(self, cur, new) -> ValStatus:  # pragma: no cover - abstract
        raise NotImplementedError


_KT = {"i": ("write_int", "read_int"), "l": ("write_long", "read_long"), "d": ("write_double", "read_double")}


class KVPartition(Writable):
    """A hash-map partition. ``key_type``/``val_type``: 'i' int32, 'l' int64, 'd' double,
    'o' object (Writable)."""

    key_type = "i"
    val_type = "i"
    default = INT_MIN

    def __init__(self):
        self.kv: Dict[Any, Any] = {}

    def initialize(self) -> None:
        self.kv = {}

    def put_key_val(self, key, val, combiner) -> ValStatus:
        cur = self.kv.get(key)
        if cur is None:
            self.kv[key] = val
            return ValStatus.ADDED
        if isinstance(combiner, ValCombiner):
            res = combiner.combine(cur, val)
            return res if isinstance(res, ValStatus) else ValStatus.COMBINED
        self.kv[key] = combiner.combine(cur, val)
        return ValStatus.COMBINED

    def get_val(self, key):
        return self.kv.get(key, self.default)

    def get_kv_map(self) -> Dict[Any, Any]:
        return self.kv

    def size(self) -> int:
        return len(self.kv)

    def is_empty(self) -> bool:
        return not self.kv

    def clear(self) -> None:
        self.kv.clear()

    # -- wire format ------------------------------------------------------------------
    def _wk(self, out: DataOutput, t: str, v) -> None:
        if t == "o":
            out.write_utf(class_name(v))
            v.write(out)
        else:
            getattr(out, _KT[t][0])(v)

    def _rk(self, inp: DataInput, t: str):
        if t == "o":
            obj = writable_class(inp.read_utf())()
            obj.read(inp)
            return obj
        return getattr(inp, _KT[t][1])()

    def write(self, out: DataOutput) -> None:
        out.write_int(len(self.kv))
        for k, v in self.kv.items():
            self._wk(out, self.key_type, k)
            self._wk(out, self.val_type, v)

    def read(self, inp: DataInput) -> None:
        self.kv = {}
        for _ in range(inp.read_int()):
            k = self._rk(inp, self.key_type)
            self.kv[k] = self._rk(inp, self.val_type)


class Int2IntKVPartition(KVPartition):
    key_type, val_type, default = "i", "i", INT_MIN


class Int2LongKVPartition(KVPartition):
    key_type, val_type, default = "i", "l", LONG_MIN


class Long2DoubleKVPartition(KVPartition):
    key_type, val_type, default = "l", "d", float("-inf")


class Long2IntKVPartition(KVPartition):
    key_type, val_type, default = "l", "i", INT_MIN


class Int2ValKVPartition(KVPartition):
    key_type, val_type, default = "i", "o", None


class Key2ValKVPartition(KVPartition):
    key_type, val_type, default = "o", "o", None


class _KVPartitionCombiner(PartitionCombiner):
    def __init__(self, val_combiner):
        self.val_combiner = val_combiner

    def combine(self, cur: KVPartition, new: KVPartition) -> PartitionStatus:
        for k, v in new.kv.items():
            cur.put_key_val(k, v, self.val_combiner)
        return PartitionStatus.COMBINED


class KVTable(Table):
    """Table of KV partitions; subclasses fix the partition class and the key -> id map."""

    partition_cls = Int2IntKVPartition

    def __init__(self, table_id: int = 0, combiner=None):
        self.val_combiner = combiner if combiner is not None else TypeIntCombiner(Operation.SUM)
        super().__init__(table_id, _KVPartitionCombiner(self.val_combiner))

    def get_kv_partition_id(self, key) -> int:
        return int(key)

    def _get_or_create(self, key) -> KVPartition:
        pid = self.get_kv_partition_id(key)
        p = self.get_partition(pid)
        if p is None:
            kvp = self.partition_cls()
            kvp.initialize()
            p = Partition(pid, kvp)
            self.insert_partition(p)
        return p.get()

    def add_key_val(self, key, val) -> ValStatus:
        return self._get_or_create(key).put_key_val(key, val, self.val_combiner)

    def get_val(self, key):
        p = self.get_partition(self.get_kv_partition_id(key))
        if p is None:
            return self.partition_cls.default
        return p.get().get_val(key)

    def items(self):
        for p in self.get_partitions():
            yield from p.get().kv.items()

    def to_dict(self) -> dict:
        return dict(self.items())


class Int2IntKVTable(KVTable):
    partition_cls = Int2IntKVPartition


class Int2LongKVTable(KVTable):
    partition_cls = Int2LongKVPartition


class Long2DoubleKVTable(KVTable):
    partition_cls = Long2DoubleKVPartition

    def get_kv_partition_id(self, key) -> int:
        k = int(key) & 0xFFFFFFFF  # Java (int) cast
        return k - (1 << 32) if k >= (1 << 31) else k


class Long2IntKVTable(Long2DoubleKVTable):
    partition_cls = Long2IntKVPartition


class Int2ValKVTable(KVTable):
    partition_cls = Int2ValKVPartition


class Key2ValKVTable(KVTable):
    """Object keys; partition id = the key's stable hash (``hash_code()`` if the key
    defines it, else a CRC of its wire bytes), so every worker agrees."""

    partition_cls = Key2ValKVPartition

    def __init__(self, table_id: int = 0, combiner=None, num_partitions: Optional[int] = None):
        super().__init__(table_id, combiner)
        self.num_partitions = num_partitions

    def get_kv_partition_id(self, key) -> int:
        hc = getattr(key, "hash_code", None)
        if hc is not None:
            h = hc()
        else:
            import zlib

            h = zlib.crc32(key.to_bytes())
        return h % self.num_partitions if self.num_partitions else h


# ---------------------------------------------------------------- device KV partitions
def _reduce_by_key(keys: torch.Tensor, vals: torch.Tensor, op: Operation):
    """Sort keys, merge duplicates with ``op`` (sum/max/min/prod) on the tensor's device."""
    keys = keys.to(torch.int64)
    if keys.numel() == 0:
        return keys, vals
    uk, inv = torch.unique(keys, sorted=True, return_inverse=True)
    red = {Operation.SUM: "sum", Operation.MAX: "amax", Operation.MIN: "amin", Operation.MULTIPLY: "prod"}.get(op)
    if red is None:
        raise ValueError(f"{op} is not a commutative key reduction")
    shape = (uk.numel(),) + tuple(vals.shape[1:])
    idx = inv.view(-1, *([1] * (vals.dim() - 1))).expand_as(vals)
    out = torch.zeros(shape, dtype=vals.dtype, device=vals.device)
    return uk, out.scatter_reduce(0, idx, vals, red, include_self=False)


class TensorKVPartition(Writable):
    """Sorted unique int64 ``keys`` [n] and ``vals`` [n, ...] on any device."""

    def __init__(self, keys: Optional[torch.Tensor] = None, vals: Optional[torch.Tensor] = None,
                 op: Operation = Operation.SUM, presorted: bool = False):
        self.op = Operation(op)
        if keys is None:
            self.keys, self.vals = torch.empty(0, dtype=torch.int64), torch.empty(0)
            return
        if not presorted:
            keys, vals = _reduce_by_key(keys, vals, self.op)
        self.keys, self.vals = keys, vals

    def lookup(self, q: torch.Tensor, default=0) -> torch.Tensor:
        out = torch.full((q.numel(),) + tuple(self.vals.shape[1:]), default, dtype=self.vals.dtype,
                         device=self.vals.device)
        if self.keys.numel():
            pos = torch.searchsorted(self.keys, q.to(self.keys.device)).clamp_max(self.keys.numel() - 1)
            m = self.keys[pos] == q
            out[m] = self.vals[pos[m]]
        return out

    def write(self, out: DataOutput) -> None:
        k = self.keys.cpu().contiguous()
        v = self.vals.cpu().contiguous()
        out.write_int(list(Operation).index(self.op))
        out.write_utf(str(v.dtype).replace("torch.", ""))
        out.write_int(v.dim())
        for s in v.shape:
            out.write_long(s)
        out.write_bytes(k.numpy().tobytes())
        out.write_bytes(v.reshape(-1).view(torch.uint8).numpy().tobytes())

    def read(self, inp: DataInput) -> None:
        import math

        import numpy as np

        self.op = list(Operation)[inp.read_int()]
        dt = getattr(torch, inp.read_utf())
        shape = tuple(inp.read_long() for _ in range(inp.read_int()))
        n = shape[0] if shape else 0
        self.keys = torch.from_numpy(np.frombuffer(inp.read_bytes(8 * n), dtype=np.int64).copy())
        nbytes = math.prod(shape) * torch.tensor([], dtype=dt).element_size()
        raw = inp.read_bytes(nbytes)
        self.vals = (torch.frombuffer(bytearray(raw), dtype=torch.uint8).view(dt).reshape(shape) if nbytes
                     else torch.empty(shape, dtype=dt))


class TensorKVCombiner(PartitionCombiner):
    """Merges two TensorKVPartitions (concat + reduce-by-key on the device)."""

    def combine(self, cur: TensorKVPartition, new: TensorKVPartition) -> PartitionStatus:
        k = torch.cat([cur.keys, new.keys.to(cur.keys.device)])
        v = torch.cat([cur.vals, new.vals.to(cur.vals.device, cur.vals.dtype)])
        cur.keys, cur.vals = _reduce_by_key(k, v, cur.op)
        return PartitionStatus.COMBINED
