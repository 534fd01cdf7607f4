"""Planned dense push / pull / regroup (harp_amd/parallel/plans.py) vs the generic
per-partition path, on 1..4 gloo ranks. Semantics (LocalGlobalSyncCollective.java:
456-698): push combines local rows into the owner's global row (ids nobody owns go to the
partitioner's owner as new partitions), local unchanged; pull combines the owner's global
row into every requesting local row, global unchanged; ids every worker requests take
the broadcast (all-gather) route."""
import pytest
import torch

from harp_amd.core import ArrCombiner, Operation, PackedTable, Partitioner, Table
from harp_amd.parallel import collectives as C
from harp_amd.parallel import plans
from harp_amd.runtime.launcher import launch


def _tables(r, P, op, packed):
    comb = ArrCombiner(op)
    # global: rank r owns ids r, r+P, ... < 12 (ids 12..14 owned by nobody)
    gids = list(range(r, 12, P))
    gbuf = torch.stack([torch.full((3,), float(10 * i + 1)) for i in gids]) if gids else torch.zeros(0, 3)
    # local: every rank wants 0..5 (all-wanted) + a rank-specific sparse set incl. unowned ids
    lids = list(range(6)) + [6 + r, 9 + (r % 2), 12 + (r % 3)]
    lids = sorted(set(lids))
    lbuf = torch.stack([torch.full((3,), float(r + 1) * (1 + (i % 3))) for i in lids])
    if packed:
        g = PackedTable(gids, gbuf.clone(), combiner=comb)
        l = PackedTable(lids, lbuf.clone(), combiner=comb)
    else:
        g, l = Table(1, comb), Table(2, comb)
        for i, row in zip(gids, gbuf):
            g.add(i, row.clone())
        for i, row in zip(lids, lbuf):
            l.add(i, row.clone())
    return l, g


def _dump(t):
    return {i: t[i].clone() for i in t.sorted_ids()}


def _job(comm, op_name, repeat):
    op = Operation[op_name]
    P, r = comm.world_size, comm.rank
    out = {}
    for packed in (True, False):
        l, g = _tables(r, P, op, packed)
        lbefore = _dump(l)
        for _ in range(repeat):  # second call reuses the cached plan
            assert C.push(comm, l, g, Partitioner(P))
        pushed = _dump(g)
        assert all(torch.equal(lbefore[i], l[i]) for i in lbefore), "push changed the local table"
        want = PackedTable(l.ids, torch.zeros_like(l.buffer), combiner=ArrCombiner(op)) if packed else Table(3, ArrCombiner(op))
        if not packed:
            for i in l.sorted_ids():
                want.add(i, torch.zeros(3))
        gbefore = _dump(g)
        assert C.pull(comm, want, g, True)
        assert all(torch.equal(gbefore[i], g[i]) for i in gbefore), "pull changed the global table"
        out[packed] = (pushed, _dump(want))
    return out


@pytest.mark.parametrize("P", [1, 2, 3, 4])
@pytest.mark.parametrize("op_name", ["SUM", "MAX"])
def test_dense_push_pull_match_generic(P, op_name):
    res = launch(_job, P, args=(op_name, 2 if op_name == "MAX" else 1), timeout=300)
    for r, out in enumerate(res):
        (pd, ld), (pg, lg) = out[True], out[False]
        assert sorted(pd) == sorted(pg), (r, sorted(pd), sorted(pg))
        for i in pd:
            assert torch.allclose(pd[i], pg[i]), (r, i, pd[i], pg[i])
        assert sorted(ld) == sorted(lg)
        for i in ld:
            assert torch.allclose(ld[i], lg[i]), (r, i, ld[i], lg[i])


def _plan_reuse(comm):
    P, r = comm.world_size, comm.rank
    comb = ArrCombiner(Operation.SUM)
    g = PackedTable(list(range(r, 20, P)), torch.zeros(len(range(r, 20, P)), 4), combiner=comb)
    l = PackedTable(list(range(20)), torch.ones(20, 4), combiner=comb)
    g.static_layout = l.static_layout = True
    calls = []
    orig = comm.all_gather_ints

    def spy(v):
        calls.append(len(v))
        return orig(v)

    comm.all_gather_ints = spy
    for _ in range(3):
        g.buffer.zero_()
        C.push(comm, l, g, Partitioner(P))
    n_first = len(calls)
    for _ in range(5):
        g.buffer.zero_()
        C.push(comm, l, g, Partitioner(P))
    return n_first, len(calls), g.buffer.sum().item()


def test_static_plan_has_no_per_call_metadata_exchange():
    res = launch(_plan_reuse, 2, timeout=120)
    for n_first, n_all, s in res:
        assert n_all == n_first  # 5 more pushes: zero extra metadata collectives
    assert sum(s for _, _, s in res) == 2 * 20 * 4


def test_combine_rows_ops():
    d = torch.zeros(3, 2)
    plans.combine_rows(d, torch.tensor([0, 0, 2]), torch.tensor([[1., 2], [3, 4], [5, 6]]), "SUM")
    assert d.tolist() == [[4, 6], [0, 0], [5, 6]]
    m = torch.full((2, 2), -float("inf"))
    plans.combine_rows(m, torch.tensor([1, 1]), torch.tensor([[1., 7], [3, 4]]), "MAX")
    assert m[1].tolist() == [3, 7]


def _sparse_job(comm, op_sparse):
    P, r = comm.world_size, comm.rank
    comb = ArrCombiner(Operation.SUM)
    g = PackedTable(list(range(r, 10, P)), torch.zeros(len(range(r, 10, P)), 3, 4, dtype=torch.int32), combiner=comb)
    ids = sorted({1, 3, 4, 7, 9, 11 + r})  # 11+r: nobody owns it -> inserted at its partitioner owner
    gen = torch.Generator().manual_seed(r)
    buf = torch.randint(-2, 3, (len(ids), 3, 4), generator=gen, dtype=torch.int32)
    buf[buf.abs() == 1] = 0  # sparse
    l = PackedTable(ids, buf, combiner=comb)
    assert C.push(comm, l, g, Partitioner(P), sparse=op_sparse)
    assert C.push(comm, l, g, Partitioner(P), sparse=op_sparse)  # cached plan
    return {i: g[i].clone() for i in g.sorted_ids()}


@pytest.mark.parametrize("P", [1, 2, 3])
def test_sparse_push_equals_dense_push(P):
    dense = launch(_sparse_job, P, args=(False,), timeout=300)
    sparse = launch(_sparse_job, P, args=(True,), timeout=300)
    for a, b in zip(dense, sparse):
        assert sorted(a) == sorted(b)
        for i in a:
            assert torch.equal(a[i], b[i]), (i, a[i], b[i])


def _sparse_pull_job(comm, sparse):
    P, r = comm.world_size, comm.rank
    comb = ArrCombiner(Operation.SUM)
    gids = list(range(r, 12, P))
    gen = torch.Generator().manual_seed(10 + r)
    gb = torch.randint(0, 4, (len(gids), 2, 5), generator=gen, dtype=torch.int32)
    gb[gb == 1] = 0
    g = PackedTable(gids, gb, combiner=comb)
    lids = sorted(set(list(range(4)) + [5 + r, 8 + (r % 2), 13]))  # 0..3 all-wanted, 13 owned by nobody
    out = []
    for _ in range(2):  # second call: cached plan
        l = PackedTable(lids, torch.full((len(lids), 2, 5), 7, dtype=torch.int32), combiner=comb)
        assert C.pull(comm, l, g, True, sparse=sparse)
        out.append({i: l[i].clone() for i in l.sorted_ids()})
    return out


@pytest.mark.parametrize("P", [1, 2, 3])
def test_sparse_pull_equals_dense_pull(P):
    dense = launch(_sparse_pull_job, P, args=(False,), timeout=300)
    sparse = launch(_sparse_pull_job, P, args=(True,), timeout=300)
    for a, b in zip(dense, sparse):
        for x, y in zip(a, b):
            assert sorted(x) == sorted(y)
            for i in x:
                assert torch.equal(x[i], y[i]), (i, x[i], y[i])


def _overwrite_job(comm):
    P, r = comm.world_size, comm.rank
    comb = ArrCombiner(Operation.SUM)
    gids = list(range(r, 12, P))
    g = PackedTable(gids, torch.stack([torch.full((2, 3), float(10 * i + 1)) for i in gids]), combiner=comb)
    lids = sorted(set(list(range(4)) + [5 + r, 8 + (r % 2)]))  # 0..3 wanted by all: the broadcast route
    out = []
    for over in (False, True):
        for _ in range(2):  # second call: cached plan (identity flags reused)
            l = PackedTable(lids, torch.full((len(lids), 2, 3), -7.0), combiner=comb)
            if not over:
                l.buffer.zero_()
            assert C.pull(comm, l, g, True, overwrite=over)
        out.append({i: l[i].clone() for i in l.sorted_ids()})
    return out


@pytest.mark.parametrize("P", [1, 2, 3])
def test_overwrite_pull_equals_zero_then_sum(P):
    for zeroed, over in launch(_overwrite_job, P, timeout=300):
        assert sorted(zeroed) == sorted(over)
        for i in zeroed:
            assert torch.equal(zeroed[i], over[i]), (i, zeroed[i], over[i])
            assert float(over[i][0, 0]) == 10 * i + 1


def test_identity_fast_path_matches_index_ops():
    d = torch.arange(12.).reshape(4, 3)
    a, b = d.clone(), d.clone()
    rows = torch.ones(4, 3) * 2
    idx = torch.arange(4)
    assert plans._is_identity(idx, 4) and not plans._is_identity(idx.flip(0), 4)
    plans.combine_rows(a, idx, rows, "SUM", ident=True)
    plans.combine_rows(b, idx, rows, "SUM")
    assert torch.equal(a, b)
    plans.combine_rows(a, idx, rows * 5, "MAX", ident=True)
    plans.combine_rows(b, idx, rows * 5, "MAX")
    assert torch.equal(a, b)
