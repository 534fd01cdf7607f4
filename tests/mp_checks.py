"""Worker-side check batteries run under harp_amd.runtime.launch (gloo, 127.0.0.1).

Each function returns a dict name -> bool (or a detail string on failure) so the
pytest side can report exactly which semantic broke on which rank."""
import torch

from harp_amd.core import (ArrCombiner, Operation, PackedTable, Partition, Partitioner, Table, Writable)
from harp_amd.core.combiner import WritableCombiner
from harp_amd.parallel import collectives as C
from harp_amd.parallel.events import Event, EventType
from harp_amd.runtime.mapper import CollectiveMapper


class Msg(Writable):
    def __init__(self, text="", n=0):
        self.text, self.n = text, n

    def write(self, out):
        out.write_utf(self.text)
        out.write_int(self.n)

    def read(self, inp):
        self.text = inp.read_utf()
        self.n = inp.read_int()

    def combine(self, other):
        self.text += other.text
        self.n += other.n


def _eq(a, b):
    return torch.allclose(torch.as_tensor(a).double(), torch.as_tensor(b).double())


def collective_battery(comm):
    P, r = comm.world_size, comm.rank
    res = {}
    SUM = ArrCombiner(Operation.SUM)

    res["barrier"] = C.barrier(comm)

    # allreduce: packed fast path
    t = PackedTable(range(4), torch.full((4, 3), float(r + 1)), combiner=SUM)
    ok = C.allreduce(comm, t)
    res["allreduce_packed"] = ok and _eq(t.buffer, torch.full((4, 3), P * (P + 1) / 2))

    # allreduce: MAX via RCCL op
    t = PackedTable([0, 1], torch.tensor([[float(r)], [float(-r)]]), combiner=ArrCombiner(Operation.MAX))
    C.allreduce(comm, t)
    res["allreduce_max"] = _eq(t.buffer, torch.tensor([[P - 1.0], [0.0]]))

    # allreduce: generic heterogeneous ids
    t = Table(0, SUM)
    t.add(r, torch.full((2,), float(r + 1)))
    t.add(r + 1, torch.full((2,), float(r + 1)))
    C.allreduce(comm, t)
    exp = {}
    for q in range(P):
        for i in (q, q + 1):
            exp[i] = exp.get(i, 0) + q + 1
    res["allreduce_generic"] = sorted(t.get_partition_ids()) == sorted(exp) and all(
        _eq(t[i], torch.full((2,), float(v))) for i, v in exp.items())

    # allreduce: MINUS combiner -> rank-ordered generic combine, identical on all ranks
    t = Table(0, ArrCombiner(Operation.MINUS))
    t.add(0, torch.tensor([float(10 ** r)]))
    C.allreduce(comm, t)
    res["allreduce_minus_rank_order"] = _eq(t[0], torch.tensor([1.0 - sum(10.0 ** q for q in range(1, P))]))

    # allgather: packed, equal counts
    t = PackedTable([2 * r, 2 * r + 1], torch.full((2, 2), float(r)), combiner=SUM)
    C.allgather(comm, t)
    res["allgather_packed"] = t.ids == list(range(2 * P)) and all(
        _eq(t[i], torch.full((2,), float(i // 2))) for i in range(2 * P))

    # allgather: generic with a clashing id
    t = Table(0, SUM)
    t.add(0, torch.ones(3))
    t.add(100 + r, torch.full((3,), float(r)))
    C.allgather(comm, t)
    res["allgather_generic"] = _eq(t[0], torch.full((3,), float(P))) and all(
        _eq(t[100 + q], torch.full((3,), float(q))) for q in range(P)) and len(t) == P + 1

    # broadcast: packed into empty tables
    root = P - 1
    if r == root:
        t = PackedTable([5, 6], torch.tensor([[1.0, 2.0], [3.0, 4.0]]), combiner=SUM)
    else:
        t = PackedTable([], torch.zeros((0, 2)), combiner=SUM)
    C.broadcast(comm, t, root)
    res["broadcast_packed"] = t.ids == [5, 6] and _eq(t.buffer, torch.tensor([[1.0, 2.0], [3.0, 4.0]]))

    # broadcast: generic Writable payload combining into an existing local partition
    t = Table(0, WritableCombiner())
    t.add(1, Msg("r%d" % r, r))
    if r == 0:
        t.add(2, Msg("only-root", 42))
    C.broadcast(comm, t, 0, use_mst=True)
    if r == 0:
        res["broadcast_generic"] = t[1].text == "r0" and len(t) == 2
    else:
        res["broadcast_generic"] = t[1].text == "r%dr0" % r and t[1].n == r and t[2].text == "only-root"

    # reduce: packed
    t = PackedTable([0, 1, 2], torch.full((3, 2), float(r + 1)), combiner=SUM)
    C.reduce(comm, t, 0)
    res["reduce_packed"] = (_eq(t.buffer, torch.full((3, 2), P * (P + 1) / 2)) if r == 0
                            else (len(t) == 0 or P == 1))

    # reduce: generic, rank-ordered MINUS
    t = Table(0, ArrCombiner(Operation.MINUS))
    t.add(7, torch.tensor([float(r + 1)]))
    C.reduce(comm, t, 0)
    res["reduce_generic"] = (_eq(t[7], torch.tensor([1.0 - sum(q + 1.0 for q in range(1, P))])) if r == 0
                             else (t.is_empty() or P == 1))

    # regroup: packed with the default (strided) partitioner -> permuted reduce-scatter
    t = PackedTable(range(2 * P), torch.full((2 * P, 2), float(r + 1)), combiner=SUM)
    C.regroup(comm, t, Partitioner(P))
    res["regroup_packed"] = sorted(t.ids) == sorted([r, r + P]) and _eq(t.buffer, torch.full((2, 2), P * (P + 1) / 2))

    # regroup: generic — ids r*10+j go to (r*10+j) % P, sent ones removed locally
    t = Table(0, SUM)
    for j in range(3):
        t.add(r * 10 + j, torch.tensor([1.0]))
    t.add(-1, torch.tensor([5.0]))  # abs(-1 % P) owner
    C.regroup(comm, t, Partitioner(P))
    exp = {}
    for q in range(P):
        for j in range(3):
            i = q * 10 + j
            if i % P == r:
                exp[i] = exp.get(i, 0) + 1
        if 1 % P == r:
            exp[-1] = exp.get(-1, 0) + 5
    res["regroup_generic"] = sorted(t.get_partition_ids()) == sorted(exp) and all(
        _eq(t[i], torch.tensor([float(v)])) for i, v in exp.items())

    # aggregate: regroup -> double -> allgather
    t = Table(0, SUM)
    for i in range(P):
        t.add(i, torch.tensor([1.0]))
    C.aggregate(comm, t, Partitioner(P), lambda x: x * 2)
    res["aggregate"] = sorted(t.get_partition_ids()) == list(range(P)) and all(
        _eq(t[i], torch.tensor([2.0 * P])) for i in range(P))

    # push / pull (parameter server)
    glob = Table(1, SUM)
    glob.add(r, torch.zeros(2))
    local = Table(2, SUM)
    for i in range(P):
        local.add(i, torch.full((2,), float(r + 1)))
    local.add(1000 + r, torch.full((2,), float(r + 1)))
    C.push(comm, local, glob, Partitioner(P))
    ok = _eq(glob[r], torch.full((2,), P * (P + 1) / 2)) and _eq(local[0], torch.full((2,), float(r + 1)))
    for q in range(P):
        if (1000 + q) % P == r:
            ok = ok and _eq(glob[1000 + q], torch.full((2,), float(q + 1)))
    res["push"] = ok
    pulled = Table(3, SUM)
    for i in range(P):
        pulled.add(i, torch.zeros(2))
    pulled.add(5000, torch.zeros(2))  # not in any global table -> untouched
    C.pull(comm, pulled, glob, True)
    res["pull"] = all(_eq(pulled[i], torch.full((2,), P * (P + 1) / 2)) for i in range(P)) and _eq(
        pulled[5000], torch.zeros(2)) and _eq(glob[r], torch.full((2,), P * (P + 1) / 2))

    # rotate: generic, default ring
    t = Table(0, SUM)
    t.add(r, torch.tensor([float(r)]))
    t.add(50 + r, Msg("m%d" % r, r)) if False else None
    C.rotate(comm, t)
    src = (r - 1) % P
    res["rotate_generic"] = t.get_partition_ids() == [src] and _eq(t[src], torch.tensor([float(src)]))

    # rotate: packed with an explicit permutation (reverse), async handle
    t = PackedTable([r * 3, r * 3 + 1], torch.full((2, 4), float(r)), combiner=SUM)
    rmap = [P - 1 - q for q in range(P)]
    h = C.rotate(comm, t, rmap, async_op=True)
    if hasattr(h, "wait"):
        h.wait()
    s = rmap.index(r)
    res["rotate_packed"] = t.ids == [s * 3, s * 3 + 1] and _eq(t.buffer, torch.full((2, 4), float(s)))

    # join: static ids {r, r+1}; dynamic id r
    static = Table(0, SUM)
    static.add(r, torch.zeros(1))
    static.add((r + 1) % P, torch.zeros(1))
    dyn = Table(1, SUM)
    dyn.add(r, torch.tensor([float(r + 1)]))
    dyn.add(900 + r, torch.tensor([1.0]))  # no static holder, no partitioner -> stays local
    C.join(comm, dyn, None, static)
    exp = {r: r + 1.0, (r + 1) % P: (r + 1) % P + 1.0, 900 + r: 1.0}
    res["join"] = sorted(dyn.get_partition_ids()) == sorted(exp) and all(
        _eq(dyn[i], torch.tensor([v])) for i, v in exp.items())

    # events: MESSAGE to the next worker, COLLECTIVE from the master, LOCAL to self
    m = CollectiveMapper(comm)
    m.send_event(Event(EventType.MESSAGE, "ev", r, (r + 1) % P, torch.tensor([float(r)])))
    if r == 0:
        m.send_event(Event(EventType.COLLECTIVE, "ev", 0, -1, Msg("hello", 1)))
    m.send_event(Event(EventType.LOCAL, "ev", r, r, None))
    want = 2 + (1 if (r != 0 and P > 1) else 0)
    got = []
    while len(got) < want:
        ev = m.wait_event(timeout=60)
        if ev is None:
            break
        got.append(ev)
    kinds = sorted(e.event_type.name for e in got)
    ok = len(got) == want and "LOCAL" in kinds
    msg = [e for e in got if e.event_type is EventType.MESSAGE]
    ok = ok and len(msg) == 1 and msg[0].source_id == (r - 1) % P and _eq(msg[0].body, [float((r - 1) % P)])
    if r != 0 and P > 1:
        col = [e for e in got if e.event_type is EventType.COLLECTIVE]
        ok = ok and len(col) == 1 and col[0].body.text == "hello"
    res["events"] = ok
    C.barrier(comm)

    # failure contract: a collective whose transport raises returns False
    def boom(op):
        raise TimeoutError("injected")

    comm.fault_hook = boom
    res["fault_returns_false"] = C.barrier(comm) is False
    comm.fault_hook = None
    res["barrier_after_fault"] = C.barrier(comm)
    return res


def runtime_battery(comm):
    """KV/groupByKey, partition utilities, object comm, table-level Rotator, checkpoint."""
    import os
    import tempfile

    from harp_amd.core.examples import IntCount, StringKey, WordAvgFunction, WordCountTable
    from harp_amd.core.keyval import TensorKVCombiner, TensorKVPartition
    from harp_amd.parallel import partition_util as PU
    from harp_amd.runtime.dymoro import Rotator
    from harp_amd.utils.checkpoint import load_checkpoint, save_checkpoint

    P, r = comm.world_size, comm.rank
    res = {}
    # word count: every worker counts its words, groupByKey at owners, average, allgather
    words = ["apple", "banana", "cherry", "apple", "durian"][: 3 + r % 3]
    wc = WordCountTable(0, num_partitions=7)
    for w in words:
        wc.add_word(w, val=10)
    C.aggregate(comm, wc, Partitioner(P), WordAvgFunction())
    total = {}
    for q in range(P):
        for w in ["apple", "banana", "cherry", "apple", "durian"][: 3 + q % 3]:
            total[w] = total.get(w, 0) + 1
    got = {k.str: (v.val, v.count) for k, v in wc.items()}
    res["wordcount_aggregate"] = set(got) == set(total) and all(got[w] == (10, 1) for w in total)
    wc2 = WordCountTable(0, num_partitions=5)
    for w in words:
        wc2.add_word(w)
    C.group_by_key(comm, wc2, Partitioner(P))
    mine = {k.str: v.count for k, v in wc2.items()}
    allm = PU.allgather_objects(comm, [IntCount(sum(mine.values()), len(mine))])
    res["group_by_key"] = sum(x.val for x in allm) == sum(total.values()) and sum(x.count for x in allm) == len(total)
    # device KV allreduce (generic path, combine = reduce-by-key)
    t = Table(0, TensorKVCombiner())
    t.add(0, TensorKVPartition(torch.tensor([r, 100]), torch.tensor([1.0, float(r)])))
    C.allreduce(comm, t)
    kv = t[0]
    res["tensor_kv_allreduce"] = kv.keys.tolist() == list(range(P)) + [100] and kv.vals.tolist() == [1.0] * P + [
        float(sum(range(P)))]
    # partition utilities
    tab = Table(0)
    for i in range(r + 1):
        tab.add(i, torch.zeros(1))
    cnt = PU.regroup_partition_count(comm, tab, Partitioner(P))
    res["regroup_partition_count"] = int(cnt.sum()) == sum(q + 1 for q in range(P)) and int(cnt[r].sum()) == r + 1
    sets = PU.allgather_partition_set(comm, tab)
    res["allgather_partition_set"] = [s.par_set for s in sets] == [list(range(q + 1)) for q in range(P)]
    g = PU.gather_partition_set(comm, tab, 0)
    res["gather_partition_set"] = (g is not None and len(g) == P) if r == 0 else g is None
    order = PU.create_send_order(P, r)
    res["send_order"] = sorted(order) == [q for q in range(P) if q != r]
    objs = PU.broadcast_objects(comm, [IntCount(7, 8)] if r == 0 else None, 0)
    res["broadcast_objects"] = len(objs) == 1 and objs[0].val == 7
    gathered = PU.gather_objects(comm, [IntCount(r, 1)], 0)
    res["gather_objects"] = ([o.val for o in gathered] == list(range(P))) if r == 0 else gathered is None
    # table-level rotator: 2 slices rotating on their own channels, concurrently
    class _M:
        pass

    mp = _M()
    mp.comm, mp.get_num_workers = comm, (lambda: P)
    t0, t1 = Table(0), Table(1)
    t0.add(r, torch.tensor([float(r)]))
    t1.add(100 + r, torch.tensor([float(r)]))
    rot = Rotator([t0, t1], mp)
    for step in range(P):
        rot.rotate(0)
        rot.rotate(1)
        a, b = rot.get_split_map(0), rot.get_split_map(1)
    rot.stop()
    res["rotator_full_tour"] = a.get_partition_ids() == [r] and b.get_partition_ids() == [100 + r]
    # packed slices with fixed (unequal) row counts: header-free after the first hop
    p0 = PackedTable([10 * r + j for j in range(r + 1)], torch.full((r + 1, 2), float(r)))
    prot = Rotator([p0], mp, static_rows=True)
    h0 = C.STATS["rotate_header_roundtrips"]
    for step in range(P):
        prot.rotate(0)
        pa = prot.get_split_map(0)
    prot.stop()
    res["rotator_static_rows"] = (pa.ids == [10 * r + j for j in range(r + 1)] and bool((pa.buffer == float(r)).all())
                                  and C.STATS["rotate_header_roundtrips"] - h0 == (1 if P > 1 else 0))
    # checkpoint / resume across ranks
    d = os.path.join(tempfile.gettempdir(), f"harp_ck_{os.environ.get('MASTER_PORT', '0')}")
    ct = Table(0)
    ct.add(r, torch.full((3,), float(r)))
    save_checkpoint(d, {"m": ct}, r, P, iteration=3, comm=comm)
    C.barrier(comm)
    man, tabs = load_checkpoint(d, r, P)
    res["checkpoint_resume"] = man["iteration"] == 3 and torch.equal(tabs["m"][r], torch.full((3,), float(r)))
    return res
