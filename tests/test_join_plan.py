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
    # static_layout packed rotate: row counts tracked locally after one all-gather, so
    # later rotations (ring, stride 2) send no header; unequal counts per rank
    s = PackedTable([10 * r + j for j in range(r + 1)], torch.full((r + 1, 2), float(r)), combiner=SUM)
    s.static_layout = True
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
