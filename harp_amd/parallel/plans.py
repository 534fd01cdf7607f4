"""Cached communication plans for the dense (``PackedTable``) parameter-server and shuffle
collectives (SURVEY §5.8 "CommPlan").

The reference re-derives the routing of every push / pull / regroup call from scratch:
an all-to-all of partition counts and an allgather of partition-id sets per call
(core/harp-collective/.../partition/PartitionUtil.java:132-207, 270-428;
LocalGlobalSyncCollective.java:456-698), then per-partition encode / send / decode.

Here the routing of a (local table layout, global table layout, partitioner) triple is
computed ONCE and kept as device index tensors:

* **push**: ``send_idx`` (local rows sorted by destination owner), per-rank row counts,
  and ``recv_dst`` (rows of the global slab each received row combines into; ids no
  worker owned yet are appended at the partitioner's owner, filled with the combiner's
  identity). A push is then ``index_select`` -> one ``all_to_all_single`` ->
  ``index_add_`` / ``scatter_reduce_``: no per-partition objects, no host sync.
* **pull**: ids requested by EVERY worker travel by a padded all-gather of each owner's
  slab (the reference chain-broadcasts them, LocalGlobalSyncCollective.java:654-660);
  the rest by one all-to-all-v; received rows combine into the requester's rows.
* **regroup**: owner-sorted row permutation + counts for the reduce-scatter path.

A plan is valid while every rank's layouts are unchanged. Each rank detects its own
changes through ``PackedTable.version``; agreement across ranks costs one 2-int
all-gather per call, skipped entirely when both tables are flagged ``static_layout``
(the application's promise that it never changes their ids).
"""
from __future__ import annotations

import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..core.partition import UNKNOWN_WORKER_ID, Partitioner
from ..core.table import PackedTable
from .comm import Communicator

_REDUCE = {"SUM": "sum", "PLUS": "sum", "MAX": "amax", "MIN": "amin", "MULTIPLY": "prod", "PROD": "prod"}


def _op_name(table: PackedTable) -> str:
    op = getattr(table.combiner, "operation", None)
    return (op.name if op is not None else "SUM").upper()


def identity_value(op: str, dtype: torch.dtype):
    if op in ("MAX",):
        return -float("inf") if dtype.is_floating_point else torch.iinfo(dtype).min
    if op in ("MIN",):
        return float("inf") if dtype.is_floating_point else torch.iinfo(dtype).max
    if op in ("MULTIPLY", "PROD"):
        return 1
    return 0


_ELEMENTWISE = {"SUM": torch.Tensor.add_, "PLUS": torch.Tensor.add_, "MULTIPLY": torch.Tensor.mul_,
                "PROD": torch.Tensor.mul_,
                "MAX": lambda d, r: torch.maximum(d, r, out=d), "MIN": lambda d, r: torch.minimum(d, r, out=d)}


def _is_identity(idx: Optional[torch.Tensor], n: int) -> bool:
    """``idx`` == arange(n) (checked once per plan; one device sync at plan build)."""
    if idx is None or idx.numel() != n:
        return False
    return n == 0 or bool(torch.equal(idx, torch.arange(n, dtype=idx.dtype, device=idx.device)))


def _flag(plan: "_Plan", name: str, idx: Optional[torch.Tensor], n: int) -> bool:
    v = getattr(plan, name, None)
    if v is None:
        v = _is_identity(idx, n)
        setattr(plan, name, v)
    return v


def _take(buf: torch.Tensor, idx: torch.Tensor, ident: bool) -> torch.Tensor:
    """Rows ``buf[idx]``; the buffer itself when ``idx`` is every row in order (no copy)."""
    if ident:
        return buf
    return buf.index_select(0, idx) if idx.numel() else buf[:0]


def combine_rows(dst: torch.Tensor, idx: torch.Tensor, rows: torch.Tensor, op: str, ident: bool = False) -> None:
    """``dst[idx[j]] (op)= rows[j]`` for every j (duplicates in ``idx`` all combine).
    ``ident``: ``idx`` is arange(len(dst)) -- one elementwise pass instead of an index op."""
    if rows.numel() == 0:
        return
    if op == "REPLACE":  # overwrite pull: each destination row receives exactly one row
        if ident and rows.shape == dst.shape:
            dst.copy_(rows)
        else:
            dst.index_copy_(0, idx, rows.to(dst.dtype))
        return
    if ident and rows.shape == dst.shape and op in _ELEMENTWISE:
        _ELEMENTWISE[op](dst, rows.to(dst.dtype))
        return
    if op in ("SUM", "PLUS"):
        dst.index_add_(0, idx, rows.to(dst.dtype))
        return
    red = _REDUCE.get(op)
    if red is None:
        raise ValueError(f"combiner {op} has no dense form")
    flat = dst.reshape(dst.shape[0], -1)
    src = rows.reshape(rows.shape[0], -1).to(dst.dtype)
    flat.scatter_reduce_(0, idx[:, None].expand_as(src), src, reduce=red, include_self=True)


def _all_id_sets(comm: Communicator, ids: Sequence[int]) -> List[torch.Tensor]:
    """Variable-length int64 id lists of every rank (one padded all-gather)."""
    t = torch.tensor(list(ids), dtype=torch.int64)
    msgs = comm.all_gather_bytes(t.view(torch.uint8).to(comm.device)) if comm.world_size > 1 else [t.view(torch.uint8)]
    return [m.cpu().view(torch.int64) if m.numel() else torch.zeros(0, dtype=torch.int64) for m in msgs]


def _exchange_ids(comm: Communicator, per_dest: List[torch.Tensor]) -> List[torch.Tensor]:
    """All-to-all-v of int64 id lists: ``per_dest[r]`` goes to rank r; returns per source."""
    P = comm.world_size
    if P == 1:
        return [per_dest[0]]
    msgs = [x.contiguous().view(torch.uint8).to(comm.device) for x in per_dest]
    got = comm.all_to_all_bytes(msgs)
    return [g.cpu().view(torch.int64) if g.numel() else torch.zeros(0, dtype=torch.int64) for g in got]


def _owner_of(comm: Communicator, glob: PackedTable) -> Dict[int, int]:
    """id -> lowest rank whose global table holds it."""
    owner: Dict[int, int] = {}
    for r, ids in enumerate(_all_id_sets(comm, glob.ids)):
        for i in ids.tolist():
            owner.setdefault(i, r)
    return owner


@dataclass
class _Plan:
    key: Tuple
    send_idx: torch.Tensor = None
    send_counts: List[int] = field(default_factory=list)
    recv_counts: List[int] = field(default_factory=list)
    recv_dst: torch.Tensor = None
    new_ids: List[int] = field(default_factory=list)
    # pull broadcast part
    bc_idx: torch.Tensor = None      # owner: its rows wanted by every rank
    bc_counts: List[int] = field(default_factory=list)
    bc_src: torch.Tensor = None      # requester: rows of the gathered [P, mx] block to take
    bc_dst: torch.Tensor = None      # requester: local rows they combine into
    # push: for every local row, its destination rank and row index in the owner's slab
    owner_row: torch.Tensor = None
    dest_rank: torch.Tensor = None


def _plan_key(comm: Communicator, kind: str, local: PackedTable, glob: PackedTable, extra=()) -> Tuple:
    """Global layout key: every rank's (local, global) id hashes. Static tables that were
    verified before skip the all-gather."""
    mine = (local.ids_hash(), glob.ids_hash(), len(local), len(glob))
    if comm.world_size == 1:
        return (kind, mine) + tuple(extra)
    cache = getattr(local, "_plans", {})
    stat = getattr(local, "static_layout", False) and getattr(glob, "static_layout", False)
    if stat:
        for k, p in cache.items():
            if k[0] == kind and k[2:] == tuple(extra) and getattr(p, "_mine", None) == mine:
                return k
    allv = comm.all_gather_ints(list(mine))
    return (kind, tuple(tuple(r) for r in allv.tolist())) + tuple(extra)


def _cached(local: PackedTable, key) -> Optional[_Plan]:
    cache = getattr(local, "_plans", None)
    return None if cache is None else cache.get(key)


def _store(local: PackedTable, plan: _Plan, mine) -> None:
    cache = getattr(local, "_plans", None)
    if cache is None:
        cache = local._plans = {}
    if len(cache) > 8:
        cache.clear()
    plan._mine = mine
    cache[plan.key] = plan


def _part_key(p: Partitioner) -> Tuple:
    """Value identity of a partitioner (class + scalar fields), so an equal partitioner
    object created per call still hits the cached plan."""
    return (type(p).__qualname__,
            tuple(sorted((k, v) for k, v in vars(p).items() if isinstance(v, (int, float, str, bool)))))


def dense_pair(comm: Communicator, local, glob) -> bool:
    """True when ``local`` / ``glob`` can take the dense path on EVERY rank: both packed,
    one part shape + dtype, a combiner with a dense form. Uniformity costs one 1-int
    all-gather unless both tables are ``static_layout`` (then this rank's answer is
    assumed for all, as the flag promises)."""
    ok = (isinstance(local, PackedTable) and isinstance(glob, PackedTable)
          and local.part_shape == glob.part_shape and local.buffer.dtype == glob.buffer.dtype
          and _op_name(glob) in _REDUCE and _op_name(local) in _REDUCE)
    if comm.world_size == 1 or (ok and getattr(local, "static_layout", False) and getattr(glob, "static_layout", False)):
        return ok
    sig = zlib.crc32(repr((local.part_shape, str(local.buffer.dtype))).encode()) & 0x7FFFFFFF if ok else 0
    v = comm.all_gather_ints([sig])[:, 0]
    return bool(ok and (v == sig).all())


# ------------------------------------------------------------------------------- push
def _build_push(comm: Communicator, local: PackedTable, glob: PackedTable, partitioner: Partitioner, key) -> _Plan:
    P, me = comm.world_size, comm.rank
    owner = _owner_of(comm, glob)
    ids = local.ids
    dest = []
    for i in ids:
        w = owner.get(i)
        if w is None:
            w = partitioner.get_worker_id(i)
        dest.append(w if (w != UNKNOWN_WORKER_ID and 0 <= w < P) else -1)
    d = torch.tensor(dest, dtype=torch.int64)
    keep = torch.nonzero(d >= 0).flatten()
    order = keep[torch.argsort(d[keep], stable=True)]
    send_counts = torch.bincount(d[keep], minlength=P).tolist() if keep.numel() else [0] * P
    ids_t = torch.tensor(ids, dtype=torch.int64)
    per_dest, o = [], 0
    sorted_ids = ids_t[order]
    for r in range(P):
        per_dest.append(sorted_ids[o:o + send_counts[r]])
        o += send_counts[r]
    got = _exchange_ids(comm, per_dest)
    recv_counts = [g.numel() for g in got]
    row = dict(glob._row)
    new_ids: List[int] = []
    dst = []
    n0 = len(glob)
    for g in got:
        for i in g.tolist():
            j = row.get(i)
            if j is None:
                j = row[i] = n0 + len(new_ids)
                new_ids.append(i)
            dst.append(j)
    dev = local.buffer.device
    # send each source the owner-side rows of what it sent (sparse pushes address elements)
    per_src, o = [], 0
    for g in got:
        per_src.append(torch.tensor(dst[o:o + g.numel()], dtype=torch.int64))
        o += g.numel()
    back = _exchange_ids(comm, per_src)
    owner_row = torch.full((len(ids),), -1, dtype=torch.int64)
    dest_rank = torch.full((len(ids),), -1, dtype=torch.int64)
    o = 0
    for r in range(P):
        rows_r = order[o:o + send_counts[r]]
        owner_row[rows_r] = back[r]
        dest_rank[rows_r] = r
        o += send_counts[r]
    return _Plan(key, send_idx=order.to(dev), send_counts=send_counts, recv_counts=recv_counts,
                 recv_dst=torch.tensor(dst, dtype=torch.int64, device=glob.buffer.device), new_ids=new_ids,
                 owner_row=owner_row.to(dev), dest_rank=dest_rank.to(dev))


def push_dense(comm: Communicator, local: PackedTable, glob: PackedTable, partitioner: Partitioner) -> None:
    """Dense push (see module doc). ``local`` and ``glob`` must share part shape / dtype."""
    mine = (local.ids_hash(), glob.ids_hash(), len(local), len(glob))
    key = _plan_key(comm, "push", local, glob, (_part_key(partitioner),))
    plan = _cached(local, key) or _build_push(comm, local, glob, partitioner, key)
    op = _op_name(glob)
    if plan.new_ids:
        fill = torch.full((len(plan.new_ids),) + glob.part_shape, identity_value(op, glob.buffer.dtype),
                          dtype=glob.buffer.dtype, device=glob.buffer.device)
        glob.set_contents(glob.ids + plan.new_ids, torch.cat([glob.buffer, fill]))
        plan.new_ids = []  # the layout now includes them; the cached plan stays valid
    send = _take(local.buffer, plan.send_idx, _flag(plan, "_send_ident", plan.send_idx, len(local)))
    recv = _alltoall_rows(comm, send, plan.send_counts, plan.recv_counts, glob.buffer)
    combine_rows(glob.buffer, plan.recv_dst, recv, op, _flag(plan, "_recv_ident", plan.recv_dst, len(glob)))
    _store(local, plan, mine)


def push_sparse(comm: Communicator, local: PackedTable, glob: PackedTable, partitioner: Partitioner) -> int:
    """Push only the NONZERO elements of ``local`` (e.g. a count delta): each element goes
    to its row's owner as (flat index in the owner's slab, value) and is index-added there.
    Routing comes from the cached push plan (owner rank + owner row per local row); ids no
    worker owns yet are inserted first exactly as a dense push would. Moves 12-16 bytes per
    nonzero instead of the whole rows (the reference's sparse TopicCountList payloads,
    LDAUtil.java:159-213). SUM semantics. Returns the number of elements this rank sent."""
    if _op_name(glob) not in ("SUM", "PLUS"):
        raise ValueError("sparse push combines by addition")
    mine = (local.ids_hash(), glob.ids_hash(), len(local), len(glob))
    key = _plan_key(comm, "push", local, glob, (_part_key(partitioner),))
    plan = _cached(local, key) or _build_push(comm, local, glob, partitioner, key)
    if plan.new_ids:
        fill = torch.zeros((len(plan.new_ids),) + glob.part_shape, dtype=glob.buffer.dtype, device=glob.buffer.device)
        glob.set_contents(glob.ids + plan.new_ids, torch.cat([glob.buffer, fill]))
        plan.new_ids = []
    _store(local, plan, mine)
    P = comm.world_size
    rs = 1
    for x in local.part_shape:
        rs *= int(x)
    flat = local.buffer.reshape(-1)
    nz = nonzero_flat(flat)
    vals = flat[nz]
    row = nz // rs
    dest = plan.dest_rank[row]
    keep = dest >= 0
    nz, vals, row, dest = nz[keep], vals[keep], row[keep], dest[keep]
    gidx = plan.owner_row[row] * rs + (nz - row * rs)
    order = torch.argsort(dest, stable=True)
    gidx, vals = gidx[order], vals[order]
    counts = torch.bincount(dest, minlength=P).to(torch.int64)
    if P == 1:
        r_idx, r_val = gidx, vals
    else:
        dev = comm.device
        rc = torch.empty(P, dtype=torch.int64, device=dev)
        comm.all_to_all_single(rc, counts.to(dev))
        ss, rr = counts.tolist(), rc.cpu().tolist()
        r_idx = torch.empty(sum(rr), dtype=torch.int64, device=dev)
        r_val = torch.empty(sum(rr), dtype=vals.dtype, device=dev)
        comm.all_to_all_single(r_idx, gidx.contiguous().to(dev), rr, ss)
        comm.all_to_all_single(r_val, vals.contiguous().to(dev), rr, ss)
    glob.buffer.view(-1).index_add_(0, r_idx.to(glob.buffer.device), r_val.to(glob.buffer.dtype))
    return int(gidx.numel())


def _alltoall_rows(comm: Communicator, send: torch.Tensor, send_counts, recv_counts, like: torch.Tensor):
    dev = comm.device
    shape = tuple(like.shape[1:])
    if comm.world_size == 1:  # the rows stay on this rank: no staging copy
        return send if send.device == like.device else send.to(like.device)
    recv = torch.empty((sum(recv_counts),) + shape, dtype=like.dtype, device=dev)
    if sum(send_counts) or sum(recv_counts):
        s = send.contiguous().to(dev)
        if s.dtype == torch.bool:  # both sides as uint8 bytes (same width)
            s = s.to(torch.uint8)
        comm.all_to_all_single(recv.view(torch.uint8) if recv.dtype == torch.bool else recv, s,
                               list(recv_counts), list(send_counts))
    return recv if recv.device == like.device else recv.to(like.device)


# ------------------------------------------------------------------------------- pull
def _build_pull(comm: Communicator, local: PackedTable, glob: PackedTable, use_bcast: bool, key) -> _Plan:
    P, me = comm.world_size, comm.rank
    owner = _owner_of(comm, glob)
    want = [i for i in local.ids if i in owner]
    per_owner: List[List[int]] = [[] for _ in range(P)]
    for i in want:
        per_owner[owner[i]].append(i)
    got = _exchange_ids(comm, [torch.tensor(x, dtype=torch.int64) for x in per_owner])  # requests per requester
    # ids every rank requested from me -> broadcast block
    bc_ids: List[int] = []
    if use_bcast and P > 1:
        cnt: Dict[int, int] = {}
        for g in got:
            for i in g.tolist():
                cnt[i] = cnt.get(i, 0) + 1
        bc_ids = sorted(i for i, c in cnt.items() if c == P)
    bcs = set(bc_ids)
    # alltoall part (owner side): rows to send to each requester, in its request order
    send_rows, send_counts = [], []
    for r in range(P):
        rows = [glob._row[i] for i in got[r].tolist() if i not in bcs]
        send_rows += rows
        send_counts.append(len(rows))
    all_bc = _all_id_sets(comm, bc_ids) if (use_bcast and P > 1) else [torch.zeros(0, dtype=torch.int64)] * P
    bc_counts = [x.numel() for x in all_bc]
    all_bc_sets = [set(x.tolist()) for x in all_bc]
    # requester side: what arrives from each owner (its alltoall rows in my request order)
    recv_dst, recv_counts = [], []
    for o in range(P):
        rows = [local._row[i] for i in per_owner[o] if i not in all_bc_sets[o]]
        recv_dst += rows
        recv_counts.append(len(rows))
    mx = max(bc_counts) if bc_counts else 0
    bc_src, bc_dst = [], []
    for o in range(P):
        for j, i in enumerate(all_bc[o].tolist()):
            if i in local._row:
                bc_src.append(o * mx + j)
                bc_dst.append(local._row[i])
    ldev, gdev = local.buffer.device, glob.buffer.device
    t = lambda x, dev: torch.tensor(x, dtype=torch.int64, device=dev)  # noqa: E731
    return _Plan(key, send_idx=t(send_rows, gdev), send_counts=send_counts, recv_counts=recv_counts,
                 recv_dst=t(recv_dst, ldev), bc_idx=t([glob._row[i] for i in bc_ids], gdev), bc_counts=bc_counts,
                 bc_src=t(bc_src, ldev), bc_dst=t(bc_dst, ldev))


def pull_dense(comm: Communicator, local: PackedTable, glob: PackedTable, use_bcast: bool = True,
               overwrite: bool = False) -> None:
    """Dense pull (see module doc): every local row whose id some global table holds
    receives (combines) the owner's row. ``overwrite``: it is replaced instead, which
    equals zeroing those rows first and combining by SUM, in one pass fewer."""
    mine = (local.ids_hash(), glob.ids_hash(), len(local), len(glob))
    key = _plan_key(comm, "pull", local, glob, (bool(use_bcast),))
    plan = _cached(local, key) or _build_pull(comm, local, glob, use_bcast, key)
    op = "REPLACE" if overwrite else _op_name(local)
    mx = max(plan.bc_counts) if plan.bc_counts else 0
    if mx:
        blk = torch.zeros((mx,) + glob.part_shape, dtype=glob.buffer.dtype, device=comm.device)
        n = plan.bc_idx.numel()
        if n:
            blk[:n] = glob.buffer.index_select(0, plan.bc_idx).to(comm.device)
        allb = torch.empty((comm.world_size * mx,) + glob.part_shape, dtype=blk.dtype, device=comm.device)
        comm.all_gather_into(allb, blk)
        if plan.bc_src.numel():
            rows = allb.index_select(0, plan.bc_src.to(comm.device))
            combine_rows(local.buffer, plan.bc_dst, rows.to(local.buffer.device), op)
    send = _take(glob.buffer, plan.send_idx, _flag(plan, "_send_ident", plan.send_idx, len(glob)))
    recv = _alltoall_rows(comm, send, plan.send_counts, plan.recv_counts, local.buffer)
    combine_rows(local.buffer, plan.recv_dst, recv, op, _flag(plan, "_recv_ident", plan.recv_dst, len(local)))
    _store(local, plan, mine)


def nonzero_flat(x: torch.Tensor, step: int = 1 << 30) -> torch.Tensor:
    """Flat int64 indices of the nonzeros of ``x``, in chunks of ``step`` elements (one
    nonzero call over > 2^31 elements is not supported by every backend)."""
    flat = x.reshape(-1)
    n = flat.numel()
    if n <= step:
        return torch.nonzero(flat).reshape(-1)
    parts = [torch.nonzero(flat[a:a + step]).reshape(-1) + a for a in range(0, n, step)]
    return torch.cat(parts)


def _gather_var(comm: Communicator, t: torch.Tensor) -> List[torch.Tensor]:
    """Variable-length all-gather of a 1-D tensor (size exchange + one padded all-gather)."""
    P = comm.world_size
    if P == 1:
        return [t]
    sizes = comm.all_gather_ints([t.numel()])[:, 0].tolist()
    mx = max(max(sizes), 1)
    buf = torch.zeros(mx, dtype=t.dtype, device=comm.device)
    buf[: t.numel()] = t.to(comm.device)
    out = torch.empty(P * mx, dtype=t.dtype, device=comm.device)
    comm.all_gather_into(out, buf)
    return [out[r * mx:r * mx + sizes[r]] for r in range(P)]


def pull_sparse(comm: Communicator, local: PackedTable, glob: PackedTable, use_bcast: bool = True) -> int:
    """Pull moving only the NONZERO elements of the owners' rows (word-topic counts are
    mostly zero): routing from the cached pull plan; the ids every worker wants go by a
    variable-size all-gather of (position, value) pairs, the rest by one all-to-all-v.
    SUM-combined into the local rows like a dense pull. Returns elements received."""
    if _op_name(local) not in ("SUM", "PLUS"):
        raise ValueError("sparse pull combines by addition")
    mine = (local.ids_hash(), glob.ids_hash(), len(local), len(glob))
    key = _plan_key(comm, "pull", local, glob, (bool(use_bcast),))
    plan = _cached(local, key) or _build_pull(comm, local, glob, use_bcast, key)
    _store(local, plan, mine)
    P, dev = comm.world_size, comm.device
    rs = 1
    for x in local.part_shape:
        rs *= int(x)
    lflat = local.buffer.view(-1)
    got = 0
    # broadcast part: every owner's all-wanted rows, as (position in its bc block, value)
    mx = max(plan.bc_counts) if plan.bc_counts else 0
    if mx:
        if plan.bc_idx.numel():
            blk = glob.buffer.index_select(0, plan.bc_idx).reshape(-1)
            nz = nonzero_flat(blk)
            pos, val = nz, blk[nz]
        else:
            pos = torch.zeros(0, dtype=torch.int64, device=glob.buffer.device)
            val = torch.zeros(0, dtype=glob.buffer.dtype, device=glob.buffer.device)
        lmap = getattr(plan, "bc_lmap", None)
        if lmap is None:
            lmap = torch.full((P * mx,), -1, dtype=torch.int64, device=local.buffer.device)
            lmap[plan.bc_src] = plan.bc_dst
            plan.bc_lmap = lmap
        allp, allv = _gather_var(comm, pos), _gather_var(comm, val)
        for o in range(P):
            p_o, v_o = allp[o].to(local.buffer.device), allv[o].to(local.buffer.device)
            if not p_o.numel():
                continue
            lrow = lmap[o * mx + p_o // rs]
            ok = lrow >= 0
            lflat.index_add_(0, lrow[ok] * rs + p_o[ok] % rs, v_o[ok].to(lflat.dtype))
            got += int(ok.sum())
    # all-to-all part: rows in each requester's request order
    if plan.send_idx.numel():
        rows = glob.buffer.index_select(0, plan.send_idx).reshape(-1)
        nz = nonzero_flat(rows)
        val = rows[nz]
        seq = nz // rs  # row position in the send sequence
        starts = torch.tensor([0] + list(torch.tensor(plan.send_counts).cumsum(0).tolist()), dtype=torch.int64,
                              device=seq.device)
        dest = torch.searchsorted(starts[1:], seq, right=True)
        rel = (seq - starts[dest]) * rs + nz % rs
        counts = torch.bincount(dest, minlength=P).to(torch.int64)
    else:
        rel = torch.zeros(0, dtype=torch.int64, device=dev)
        val = torch.zeros(0, dtype=glob.buffer.dtype, device=dev)
        counts = torch.zeros(P, dtype=torch.int64, device=dev)
    if P == 1:
        r_rel, r_val, rr = rel, val, counts.tolist()
    else:
        rc = torch.empty(P, dtype=torch.int64, device=dev)
        comm.all_to_all_single(rc, counts.to(dev))
        ss, rr = counts.tolist(), rc.cpu().tolist()
        r_rel = torch.empty(sum(rr), dtype=torch.int64, device=dev)
        r_val = torch.empty(sum(rr), dtype=val.dtype, device=dev)
        comm.all_to_all_single(r_rel, rel.contiguous().to(dev), rr, ss)
        comm.all_to_all_single(r_val, val.contiguous().to(dev), rr, ss)
    if r_rel.numel():
        rstart = torch.tensor([0] + list(torch.tensor(plan.recv_counts).cumsum(0).tolist()), dtype=torch.int64)
        src = torch.repeat_interleave(torch.arange(P), torch.tensor(rr)).to(r_rel.device)
        lrow = plan.recv_dst.to(r_rel.device)[rstart.to(r_rel.device)[src] + r_rel // rs]
        lflat.index_add_(0, (lrow * rs + r_rel % rs).to(lflat.device), r_val.to(lflat.dtype).to(lflat.device))
        got += int(r_rel.numel())
    return got


# ------------------------------------------------------------------------------- regroup
@dataclass
class RegroupPlan:
    per: List[List[int]]
    mx: int
    idx: Optional[torch.Tensor]  # None: the slab is already owner-sorted and balanced


def regroup_plan(table: PackedTable, partitioner: Partitioner, P: int) -> Optional[RegroupPlan]:
    """Owner-sorted row layout for the reduce-scatter regroup, cached on the table per
    (layout version, partitioner). None when some id has no valid owner."""
    key = (table.version, _part_key(partitioner), P)
    c = getattr(table, "_regroup_plan", None)
    if c is not None and c[0] == key:
        return c[1]
    ids = table.ids
    owners = [partitioner.get_worker_id(i) for i in ids]
    if not all(0 <= o < P for o in owners):
        plan = None
    else:
        per = [[] for _ in range(P)]
        for i, o in enumerate(owners):
            per[o].append(i)
        mx = max(len(x) for x in per)
        order = []
        for r in range(P):
            order += per[r] + [-1] * (mx - len(per[r]))
        if order == list(range(len(ids))) and mx * P == len(ids):
            idx = None
        else:
            idx = torch.tensor([max(i, 0) for i in order], dtype=torch.long, device=table.buffer.device)
        plan = RegroupPlan(per, mx, idx)
    table._regroup_plan = (key, plan)
    return plan
