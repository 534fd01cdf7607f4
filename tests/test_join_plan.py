"""Plan-cached graph join (GraphCollective.java:313-441) and the packed rotate header, on
3 gloo ranks: identical results to the reference semantics, and a repeated join with
unchanged layouts does no id-set all-gather."""
import torch

from harp_amd.core.combiner import ArrCombiner, Operation
from harp_amd.core.table import PackedTable, Table
from harp_amd.parallel import collectives as C
from harp_amd.runtime.launcher import launch

SUM = ArrCombiner(Operation.SUM)


def _expected(r, P, V=12):
    """Dynamic id v lives on rank v % P with value v + 1; static rows of rank q: ids q,
    q+1, q+3 (mod V). After the join rank r holds every dynamic id its static table has
    (value summed over the senders: one each), plus its own ids nobody else holds."""
    static_ids = {(r + k) % V for k in (0, 1, 3)}
    holders = {}
    for q in range(P):
        for k in (0, 1, 3):
            holders.setdefault((q + k) % V, set()).add(q)
    mine = [v for v in range(V) if v % P == r]
    exp = {}
    for v in range(V):
        if v in static_ids:
            exp[v] = float(v + 1)
    for v in mine:
        if v not in holders:
            exp[v] = float(v + 1)  # nobody needs it: stays local
    return exp


def _worker(comm):
    P, r, V = comm.world_size, comm.rank, 12
    out = {}
    # generic tables
    static = Table(0, SUM)
    for k in (0, 1, 3):
        static.add((r + k) % V, torch.zeros(1))
    res_generic = []
    for call in range(2):
        before = C.STATS["id_set_allgather"]
        dyn = Table(1, SUM)
        for v in range(r, V, P):
            dyn.add(v, torch.tensor([float(v + 1)]))
        assert C.join(comm, dyn, None, static)
        res_generic.append(({i: float(dyn[i][0]) for i in dyn.get_partition_ids()},
                            C.STATS["id_set_allgather"] - before))
    # packed tables, static layouts: no exchange at all on the repeat
    sids = sorted({(r + k) % V for k in (0, 1, 3)})
    pstatic = PackedTable(sids, torch.zeros((len(sids), 2)), combiner=SUM)
    pstatic.static_layout = True
    res_packed = []
    for call in range(2):
        b_ids, b_plans = C.STATS["id_set_allgather"], C.STATS["join_plans_built"]
        mine = list(range(r, V, P))
        pdyn = PackedTable(mine, torch.tensor([[v + 1.0, 2.0 * (v + 1)] for v in mine]), combiner=SUM)
        pdyn.static_layout = True
        assert C.join(comm, pdyn, None, pstatic)
        res_packed.append(({i: float(pdyn[i][0]) for i in pdyn.ids}, C.STATS["id_set_allgather"] - b_ids,
                           C.STATS["join_plans_built"] - b_plans,
                           all(float(pdyn[i][1]) == 2 * float(pdyn[i][0]) for i in pdyn.ids)))
    # packed rotate: one header round trip per rotation
    h0 = C.STATS["rotate_header_roundtrips"]
    t = PackedTable([r * 2, r * 2 + 1], torch.full((2, 3), float(r)), combiner=SUM)
    h = C.rotate(comm, t, None, async_op=True)
    h.wait()
    src = (r - 1) % P
    out["rotate"] = (t.ids == [src * 2, src * 2 + 1] and bool((t.buffer == float(src)).all()),
                     C.STATS["rotate_header_roundtrips"] - h0)
    # ring_rows packed rotate: row counts tracked locally after one all-gather, so
    # later rotations (ring, stride 2) send no header; unequal counts per rank
    s = PackedTable([10 * r + j for j in range(r + 1)], torch.full((r + 1, 2), float(r)), combiner=SUM)
    s.ring_rows = True
    origin, steps = r, []
    for stride in (1, 1, 2, 1):
        h0 = C.STATS["rotate_header_roundtrips"]
        assert C.rotate(comm, s, [(q + stride) % P for q in range(P)])
        origin = (origin - stride) % P
        steps.append((s.ids == [10 * origin + j for j in range(origin + 1)]
                      and bool((s.buffer == float(origin)).all()),
                      C.STATS["rotate_header_roundtrips"] - h0))
    # a map with a fixed point (ranks 0 and 1 swap, 2 keeps) drops the tracked counts on
    # every rank; the next ring rotation gathers them again
    held = [(q - 5) % P for q in range(P)]  # origin of each rank's rows after strides 1+1+2+1
    held = [held[[1, 0, 2][q]] for q in range(P)]  # the swap: rank q now holds its partner's
    assert C.rotate(comm, s, [1, 0, 2])
    h0 = C.STATS["rotate_header_roundtrips"]
    assert C.rotate(comm, s, [(q + 1) % P for q in range(P)])
    origin = held[(r - 1) % P]
    steps.append((s.ids == [10 * origin + j for j in range(origin + 1)] and bool((s.buffer == float(origin)).all()),
                  C.STATS["rotate_header_roundtrips"] - h0))
    out["ring"] = steps
    out["generic"], out["packed"], out["exp"] = res_generic, res_packed, _expected(r, P)
    return out


def test_join_plan_cached_three_ranks():
    for o in launch(_worker, 3, timeout=300):
        exp = o["exp"]
        (g1, n1), (g2, n2) = o["generic"]
        assert g1 == exp and g2 == exp
        assert n1 == 1 and n2 == 0  # the repeat reuses the plan: no id-set all-gather
        (p1, m1, b1, ok1), (p2, m2, b2, ok2) = o["packed"]
        assert p1 == exp and p2 == exp and ok1 and ok2
        assert (m1, b1) == (1, 1) and (m2, b2) == (0, 0)
        assert o["rotate"] == (True, 1)
        assert o["ring"] == [(True, 1), (True, 0), (True, 0), (True, 0), (True, 1)]


def _blk_ids(b):
    return [3 * b + j for j in range(2 + b % 2)]  # unequal row counts per block


def _rot_worker(comm):
    """Rotator(static_rows=True) under the reference's RANDOM rotation orders (maps with
    and without fixed points), a join against the rotated table after every hop, then a
    resize on one rank: every rank must raise together (no header-free hang)."""
    import random

    from harp_amd.runtime.dymoro import Rotator, RotationSchedule, create_rotation_order

    P, r = comm.world_size, comm.rank

    class _M:
        pass

    mp = _M()
    mp.comm, mp.get_num_workers = comm, (lambda: P)
    orders = create_rotation_order(random.Random(5), 3, P)
    sched = RotationSchedule(P, orders)
    tab = PackedTable(_blk_ids(r), torch.full((len(_blk_ids(r)), 2), float(r)), combiner=SUM)
    rot = Rotator([tab], mp, orders=orders, static_rows=True)
    steps = []
    for n in range(1, 2 * P + 1):
        rot.rotate(0)
        t = rot.get_split_map(0)
        it, s = divmod(n, P)
        blk = [sched.placement(it, s).index(q) for q in range(P)]
        ok_rows = t.ids == _blk_ids(blk[r]) and bool((t.buffer == float(blk[r])).all())
        # join against the rotated (ring_rows, NOT static_layout) table
        mine = [v for v in range(3 * P) if v % P == r]
        dyn = PackedTable(mine, torch.tensor([[v + 1.0] for v in mine]), combiner=SUM)
        assert C.join(comm, dyn, None, t)
        holders = {}
        for q in range(P):
            for v in _blk_ids(blk[q]):
                holders.setdefault(v, set()).add(q)
        exp = {v: float(v + 1) for v in _blk_ids(blk[r])}
        exp.update({v: float(v + 1) for v in mine if v not in holders})
        got = {i: float(dyn[i][0]) for i in dyn.ids}
        steps.append(ok_rows and got == exp and not getattr(t, "static_layout", False))
    rot.stop()
    # a resize outside rotate on rank 0 only: all ranks raise (raise_errors), none hangs
    ring = [(q + 1) % P for q in range(P)]
    assert C.rotate(comm, tab, ring)  # a derangement: every rank now tracks the row counts
    comm.raise_errors = True
    if r == 0:
        tab.set_contents(tab.ids[:1], tab.buffer[:1].clone())
    raised = False
    try:
        C.rotate(comm, tab, ring)
    except RuntimeError:
        raised = True
    comm.raise_errors = False
    return {"steps": steps, "raised": raised}


def test_rotator_random_orders_then_join_three_ranks():
    for o in launch(_rot_worker, 3, timeout=300):
        assert all(o["steps"]), o["steps"]
        assert o["raised"]
