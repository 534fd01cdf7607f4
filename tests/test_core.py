"""L2 data model: behaviours of the reference's JUnit suite (core/harp-collective/src/test:
combiner/*Test, example/*PlusTest, partition/TableTest/PartitionTest/PartitionerTest,
resource/*PoolTest/*ArrayTest, io/SerializerTest)."""
import pytest
import torch

from harp_amd.core import (ArrCombiner, ArrayPool, DataInput, DataOutput, DoubleArray, DoubleArrPlus, IntArray,
                           IntArrPlus, LongArrPlus, Operation, PackedTable, Partition, Partitioner,
                           PartitionStatus, ResourcePool, Table, Writable)
from harp_amd.core.pool import adjusted_size

DTYPES = [torch.float64, torch.float32, torch.int32, torch.int64, torch.int16, torch.int8]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("op,expect", [(Operation.SUM, 3), (Operation.MULTIPLY, 2), (Operation.MIN, 1),
                                        (Operation.MAX, 2), (Operation.MINUS, -1)])
def test_arr_combiner(dtype, op, expect):
    a = torch.full((128,), 1, dtype=dtype)
    b = torch.full((128,), 2, dtype=dtype)
    assert ArrCombiner(op).combine(a, b) is PartitionStatus.COMBINED
    assert bool((a == expect).all())


def test_combiner_size_mismatch_fails():
    a, b = torch.ones(4), torch.ones(5)
    assert ArrCombiner(Operation.SUM).combine(a, b) is PartitionStatus.COMBINE_FAILED
    assert bool((a == 1).all())


@pytest.mark.parametrize("cls,dt", [(DoubleArrPlus, torch.float64), (IntArrPlus, torch.int32),
                                    (LongArrPlus, torch.int64)])
def test_example_plus(cls, dt):
    a, b = torch.arange(10, dtype=dt), torch.arange(10, dtype=dt)
    cls().combine(a, b)
    assert a.tolist() == [2 * i for i in range(10)]


def test_table_add_combines_in_place():
    t = Table(7, DoubleArrPlus())
    assert t.get_table_id() == 7
    p1 = Partition(3, torch.ones(4, dtype=torch.float64))
    assert t.add_partition(p1) is PartitionStatus.ADDED
    p2 = Partition(3, torch.full((4,), 2.0, dtype=torch.float64))
    assert t.add_partition(p2) is PartitionStatus.COMBINED
    assert t.get_partition(3) is p1  # p2 not inserted
    assert t[3].tolist() == [3.0] * 4
    assert t.add_partition(None) is PartitionStatus.ADD_FAILED
    assert t.get_num_partitions() == 1 and not t.is_empty()
    assert t.remove_partition(3) is p1 and t.is_empty()


def test_table_typed_array_payload():
    t = Table(0, ArrCombiner(Operation.MAX))
    t.add(1, IntArray.wrap([1, 5, 2]))
    t.add(1, IntArray.wrap([4, 0, 9]))
    assert t[1].tensor.tolist() == [4, 5, 9]


def test_partitioner_default():
    p = Partitioner(3)
    assert [p.get_worker_id(i) for i in range(7)] == [0, 1, 2, 0, 1, 2, 0]
    assert p.get_worker_id(-4) == 1  # abs(id % P) semantics for negative ids


def test_packed_table_views_and_combine():
    buf = torch.zeros(3, 4)
    t = PackedTable([10, 11, 12], buf, combiner=ArrCombiner(Operation.SUM))
    t.add(11, torch.ones(4))
    assert buf[1].tolist() == [1.0] * 4  # combine wrote through the view
    t.add(13, torch.full((4,), 5.0))
    assert t.ids == [10, 11, 12, 13] and t.buffer.shape == (4, 4)
    p = t.remove_partition(10)
    assert p.id() == 10 and t.ids == [11, 12, 13]
    assert t.get_partition(13).get().tolist() == [5.0] * 4
    gen = t.to_table()
    assert sorted(gen.get_partition_ids()) == [11, 12, 13]


def test_pool_sizes_and_reuse():
    assert adjusted_size(100, True) == 128
    assert adjusted_size(100, False) == 100
    assert adjusted_size(128, True) == 128
    pool = ArrayPool()
    a = pool.get_array(torch.float64, 100, True)
    assert a.numel() == 128
    assert pool.release_array(a)
    b = pool.get_array(torch.float64, 120, True)
    assert b is a  # reuse identity after release
    c = pool.get_array(torch.float64, 100, False)
    assert c.numel() == 100 and c is not a
    assert not pool.release_array(torch.empty(3))


def test_array_create_release():
    arr = DoubleArray.create(100)
    assert arr.size == 100 and arr.get().numel() == 128
    arr.tensor.fill_(1.5)
    arr.release()
    arr2 = DoubleArray.create(100)
    assert arr2.get() is arr.get()
    arr2.release()
    v = DoubleArray(torch.arange(10, dtype=torch.float64), start=2, size=3)
    assert v.tensor.tolist() == [2.0, 3.0, 4.0] and v.num_encode_bytes() == 5 + 24
    with pytest.raises(TypeError):
        DoubleArray(torch.arange(3, dtype=torch.float32))


def test_serializer_roundtrip():
    out = DataOutput()
    out.write_byte(-3)
    out.write_int(-123456)
    out.write_long(2**40 + 5)
    out.write_double(3.25)
    out.write_float(-1.5)
    out.write_utf("héllo")
    out.write_boolean(True)
    raw = out.getvalue()
    assert raw[1:5] == (-123456).to_bytes(4, "big", signed=True)  # big-endian like Harp
    inp = DataInput(raw)
    assert inp.read_byte() == -3
    assert inp.read_int() == -123456
    assert inp.read_long() == 2**40 + 5
    assert inp.read_double() == 3.25
    assert inp.read_float() == -1.5
    assert inp.read_utf() == "héllo"
    assert inp.read_boolean() is True
    assert inp.remaining() == 0
    with pytest.raises(EOFError):
        inp.read_int()


class Pt(Writable):
    def __init__(self, x=0, y=0.0):
        self.x, self.y = x, y

    def write(self, out):
        out.write_int(self.x)
        out.write_double(self.y)

    def read(self, inp):
        self.x = inp.read_int()
        self.y = inp.read_double()

    def clear(self):
        self.x, self.y = 0, 0.0


def test_writable_roundtrip_and_pool():
    p = Pt(7, 2.5)
    q = Pt.from_bytes(p.to_bytes())
    assert (q.x, q.y) == (7, 2.5)
    assert p.num_write_bytes() == 12
    w = Pt.create()
    w.x = 9
    w.release()
    w2 = Pt.create()
    assert w2 is w and w2.x == 0  # cleared on release


def test_resource_pool_singleton():
    assert ResourcePool.get() is ResourcePool.get()
    assert "ArrayPool" in ResourcePool.get().log()
