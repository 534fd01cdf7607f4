"""KV tables (keyval/*KVPartitionTest.java behaviours), example payloads, the Harp wire
format (io/DataTest, SerializerTest, DataUtilTest) and the .hpt checkpoint."""
import os

import pytest
import torch

from harp_amd.core import DoubleArray, IntArray, Operation, PackedTable, Partition, Table, ArrCombiner
from harp_amd.core.arrays import PARTITION_LIST, SIMPLE_LIST, UNKNOWN_DATA_TYPE
from harp_amd.core.examples import (EdgeTable, EdgeVal, IntCount, StringKey, VertexTable, WordAvgFunction,
                                    WordCountTable, java_string_hash, IntVal)
from harp_amd.core.keyval import (INT_MIN, Int2IntKVPartition, Int2IntKVTable, Int2LongKVTable, Long2DoubleKVTable,
                                  TensorKVCombiner, TensorKVPartition, TypeIntCombiner, ValStatus)
from harp_amd.core.serialize import Data, decode_partition_list, encode_partition_list
from harp_amd.core.writable import DataInput, DataOutput
from harp_amd.utils.checkpoint import load_checkpoint, load_table, save_checkpoint, save_table


def test_int2int_partition_semantics():
    p = Int2IntKVPartition()
    p.initialize()
    comb = TypeIntCombiner(Operation.SUM)
    assert p.put_key_val(1, 5, comb) is ValStatus.ADDED
    assert p.put_key_val(1, 7, comb) is ValStatus.COMBINED
    assert p.get_val(1) == 12 and p.size() == 1 and not p.is_empty()
    assert p.get_val(99) == INT_MIN  # default return value
    p.clear()
    assert p.is_empty()


def test_kv_tables_and_wire_roundtrip():
    t = Int2IntKVTable(3, TypeIntCombiner(Operation.MAX))
    for k, v in [(1, 3), (2, 9), (1, 8), (1, 2)]:
        t.add_key_val(k, v)
    assert t.get_val(1) == 8 and t.get_val(2) == 9 and t.get_val(5) == INT_MIN
    assert sorted(t.get_partition_ids()) == [1, 2]  # partition id = key
    lt = Long2DoubleKVTable(0, TypeIntCombiner(Operation.SUM))
    lt.add_key_val(2 ** 33 + 5, 1.5)
    lt.add_key_val(2 ** 33 + 5, 2.0)
    assert lt.get_val(2 ** 33 + 5) == 3.5 and lt.get_partition_ids() == [5]  # (int) cast
    part = t.get_partition(1).get()
    q = Int2IntKVPartition.from_bytes(part.to_bytes())
    assert q.kv == part.kv


def test_wordcount_and_avg():
    t = WordCountTable(0)
    for w in ["a", "b", "a", "c", "a"]:
        t.add_word(w, val=len(w) * 10)
    assert t.get_val(StringKey("a")).count == 3 and t.get_val(StringKey("a")).val == 30
    assert StringKey("hello").hash_code() == java_string_hash("hello") == 99162322  # Java "hello".hashCode()
    f = WordAvgFunction()
    for p in t.get_partitions():
        f.apply(p.get())
    assert t.get_val(StringKey("a")).val == 10


def test_edge_vertex_tables():
    e = EdgeTable()
    ev = EdgeVal()
    ev.add_edge(1, 2, 3)
    e.add_key_val(7, ev)
    ev2 = EdgeVal()
    ev2.add_edge(4, 5, 6)
    e.add_key_val(7, ev2)
    assert e.get_val(7).get_num_edges() == 2
    v = VertexTable()
    v.add_key_val(1, IntVal(2))
    v.add_key_val(1, IntVal(3))
    assert v.get_val(1).val == 5


def test_tensor_kv_partition():
    p = TensorKVPartition(torch.tensor([5, 1, 5, 3]), torch.tensor([1.0, 2.0, 3.0, 4.0]))
    assert p.keys.tolist() == [1, 3, 5] and p.vals.tolist() == [2.0, 4.0, 4.0]
    q = TensorKVPartition(torch.tensor([3, 9]), torch.tensor([10.0, 1.0]))
    TensorKVCombiner().combine(p, q)
    assert p.keys.tolist() == [1, 3, 5, 9] and p.vals.tolist() == [2.0, 14.0, 4.0, 1.0]
    assert p.lookup(torch.tensor([9, 2, 1])).tolist() == [1.0, 0.0, 2.0]
    r = TensorKVPartition.from_bytes(p.to_bytes())
    assert torch.equal(r.keys, p.keys) and torch.equal(r.vals, p.vals)


def test_harp_wire_partition_list():
    parts = [Partition(3, DoubleArray.wrap([1.5, -2.0])), Partition(-7, IntArray.wrap([1, 2, 3])),
             Partition(4, IntCount(5, 6))]
    raw = encode_partition_list(parts)
    assert raw[0] == 6 and raw[1:5] == (2).to_bytes(4, "big")  # [DOUBLE_ARRAY][size BE]
    back = decode_partition_list(raw, 3)
    assert [p.id() for p in back] == [3, -7, 4]
    assert back[0].get().tensor.tolist() == [1.5, -2.0] and back[1].get().tensor.tolist() == [1, 2, 3]
    assert (back[2].get().val, back[2].get().count) == (5, 6)
    assert encode_partition_list([]) == bytes([UNKNOWN_DATA_TYPE])
    d = Data(PARTITION_LIST, "ctx", 2, parts, "op", None)
    e = Data.decode(d.encode())
    assert e.is_operation_data() and e.is_partition_data() and e.partition_id == 3 and e.worker_id == 2
    assert e.context_name == "ctx" and e.operation_name == "op" and len(e.body) == 3
    s = Data.decode(Data(SIMPLE_LIST, "c", 0, [IntArray.wrap([9])]).encode())
    assert not s.is_operation_data() and s.body[0].tensor.tolist() == [9]


def test_checkpoint_roundtrip(tmp_path):
    t = Table(5, ArrCombiner(Operation.MAX))
    t.add(1, torch.arange(6, dtype=torch.float32).reshape(2, 3))
    t.add(9, IntCount(4, 2))
    t.add(-3, torch.tensor([], dtype=torch.int64))
    path = str(tmp_path / "t.hpt")
    save_table(t, path, rank=0, world=1)
    u = load_table(path)
    assert u.table_id == 5 and u.combiner.operation is Operation.MAX
    assert torch.equal(u[1], t[1]) and u[9].val == 4 and u[-3].numel() == 0
    pk = PackedTable([4, 2], torch.randn(2, 5, dtype=torch.float64))
    save_table(pk, path)
    v = load_table(path)
    assert isinstance(v, PackedTable) and v.ids == [4, 2] and torch.equal(v.buffer, pk.buffer)
    # corruption is detected
    raw = bytearray(open(path, "rb").read())
    raw[260] ^= 0xFF  # inside the first 256-B-aligned payload
    open(path, "wb").write(bytes(raw))
    with pytest.raises(IOError):
        load_table(path)


def test_checkpoint_manifest_reshard(tmp_path):
    d = str(tmp_path / "ck")
    for r in range(2):
        t = Table(0)
        t.add(r, torch.full((2,), float(r)))
        save_checkpoint(d, {"model": t}, rank=r, world=2, iteration=7, extra={"lr": 0.1})
    man, tabs = load_checkpoint(d, rank=1, world=2)
    assert man["iteration"] == 7 and man["extra"]["lr"] == 0.1 and tabs["model"].get_partition_ids() == [1]
    man, tabs = load_checkpoint(d, rank=0, world=1)  # world changed: all shards returned
    assert sorted(tabs["model"].get_partition_ids()) == [0, 1]
