"""Example payloads, combiners and tables (Harp ``example`` package).

Reference: core/harp-collective/.../example/ — ``StringKey`` (UTF key, hashCode),
``IntCount`` (val, count) + ``IntCountPlus``, ``IntVal`` + ``IntPlus``, ``EdgeVal``
(growable (src, val, dest) arrays) + ``EdgeValCombiner``, the word-count / vertex /
edge / message tables, and ``WordAvgFunction`` (val /= count after a regroup); these are
what the groupByKey / graph demos (collective/GroupByKeyCollective.java,
GraphCollective.java) operate on.
"""
from __future__ import annotations

from typing import List

import torch

from .keyval import Int2ValKVTable, Key2ValKVTable, ValCombiner, ValStatus
from .partition import PartitionFunction
from .writable import DataInput, DataOutput, Writable


def java_string_hash(s: str) -> int:
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


class Key(Writable):
    """Base of object keys (keyval/Key.java): must define equality and a stable hash."""

    def hash_code(self) -> int:  # pragma: no cover - abstract
        raise NotImplementedError


class StringKey(Key):
    def __init__(self, s: str = ""):
        self.str = s

    def get_string_key(self) -> str:
        return self.str

    def hash_code(self) -> int:
        return java_string_hash(self.str)

    def __eq__(self, other) -> bool:
        return isinstance(other, StringKey) and other.str == self.str

    def __hash__(self) -> int:
        return hash(self.str)

    def write(self, out: DataOutput) -> None:
        out.write_utf(self.str)

    def read(self, inp: DataInput) -> None:
        self.str = inp.read_utf()

    def __repr__(self) -> str:
        return f"StringKey({self.str!r})"


class IntCount(Writable):
    def __init__(self, val: int = 0, count: int = 0):
        self.val, self.count = val, count

    def write(self, out: DataOutput) -> None:
        out.write_int(self.val)
        out.write_int(self.count)

    def read(self, inp: DataInput) -> None:
        self.val = inp.read_int()
        self.count = inp.read_int()

    def num_write_bytes(self) -> int:
        return 8

    def __repr__(self) -> str:
        return f"IntCount({self.val}, {self.count})"


class IntCountPlus(ValCombiner):
    def combine(self, cur: IntCount, new: IntCount) -> ValStatus:
        cur.val += new.val
        cur.count += new.count
        return ValStatus.COMBINED


class IntVal(Writable):
    def __init__(self, val: int = 0):
        self.val = val

    def write(self, out: DataOutput) -> None:
        out.write_int(self.val)

    def read(self, inp: DataInput) -> None:
        self.val = inp.read_int()


class IntPlus(ValCombiner):
    def combine(self, cur: IntVal, new: IntVal) -> ValStatus:
        cur.val += new.val
        return ValStatus.COMBINED


class EdgeVal(Writable):
    """Edges (src, val, dest) kept as growable int arrays (example/EdgeVal.java)."""

    def __init__(self):
        self.src: List[int] = []
        self.val: List[int] = []
        self.dest: List[int] = []

    def add_edge(self, s: int, v: int, d: int) -> None:
        self.src.append(s)
        self.val.append(v)
        self.dest.append(d)

    def add_edge_val(self, other: "EdgeVal") -> None:
        self.src += other.src
        self.val += other.val
        self.dest += other.dest

    def get_num_edges(self) -> int:
        return len(self.src)

    def as_tensor(self) -> torch.Tensor:
        return torch.tensor([self.src, self.val, self.dest], dtype=torch.int32)

    def write(self, out: DataOutput) -> None:
        out.write_int(len(self.src))
        for a, b, c in zip(self.src, self.val, self.dest):
            out.write_int(a)
            out.write_int(b)
            out.write_int(c)

    def read(self, inp: DataInput) -> None:
        n = inp.read_int()
        self.src, self.val, self.dest = [], [], []
        for _ in range(n):
            self.add_edge(inp.read_int(), inp.read_int(), inp.read_int())

    def clear(self) -> None:
        self.src, self.val, self.dest = [], [], []


class EdgeValCombiner(ValCombiner):
    def combine(self, cur: EdgeVal, new: EdgeVal) -> ValStatus:
        cur.add_edge_val(new)
        return ValStatus.COMBINED


class WordCountTable(Key2ValKVTable):
    """StringKey -> IntCount, combined with IntCountPlus (example/WordCountTable.java)."""

    def __init__(self, table_id: int = 0, num_partitions: int | None = None):
        super().__init__(table_id, IntCountPlus(), num_partitions)

    def add_word(self, word: str, val: int = 1, count: int = 1):
        return self.add_key_val(StringKey(word), IntCount(val, count))


class EdgeTable(Int2ValKVTable):
    """vertex id -> EdgeVal (example/EdgeTable.java)."""

    def __init__(self, table_id: int = 0):
        super().__init__(table_id, EdgeValCombiner())


class VertexTable(Int2ValKVTable):
    """vertex id -> IntVal summed (example/VertexTable.java)."""

    def __init__(self, table_id: int = 0):
        super().__init__(table_id, IntPlus())


class MessageTable(Int2ValKVTable):
    """vertex id -> IntVal messages summed (example/MessageTable.java)."""

    def __init__(self, table_id: int = 0):
        super().__init__(table_id, IntPlus())


class WordAvgFunction(PartitionFunction):
    """After a word-count regroup: val := val / count for every word (integer division,
    example/WordAvgFunction.java)."""

    def apply(self, partition):
        for v in partition.kv.values():
            if v.count:
                v.val = v.val // v.count
                v.count = 1
        return partition
