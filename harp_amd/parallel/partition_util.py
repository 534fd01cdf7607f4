"""Collective building blocks (Harp ``PartitionUtil`` + ``Communication`` object ops).

Reference: partition/PartitionUtil.java — receivePartitions (:55), addPartitionsToTable
(:92, combine per id), regroupPartitionCount (:132, P x P counts), rotatePartitionCount
(:209), regroupPartitionSet (:270), allgatherPartitionSet (:374), gatherPartitionSet
(:402), createSendOrder (:429, Fisher-Yates); collective/Communication.java — gather /
allgather / chain- and MST-broadcast of object lists (:196-442).

Here each is one small device-tensor collective (no per-message sockets)."""
from __future__ import annotations

import random
from typing import Any, Dict, List, Optional, Sequence

import torch

from ..core.control import PartitionCount, PartitionSet
from ..core.partition import UNKNOWN_WORKER_ID, Partition, Partitioner
from ..core.table import Table
from .codec import encode_partitions, pack_message, unpack_message
from .comm import Communicator


def add_partitions_to_table(parts: Sequence[Partition], table: Table) -> None:
    for p in parts:
        table.add_partition(p)


def create_send_order(num_workers: int, self_id: int, rng: Optional[random.Random] = None) -> List[int]:
    """Random order of the other workers (Fisher-Yates)."""
    order = [w for w in range(num_workers) if w != self_id]
    (rng or random.Random()).shuffle(order)
    return order


def regroup_partition_count(comm: Communicator, table: Table, partitioner: Partitioner) -> torch.Tensor:
    """[P, P] matrix C[src][dst] = partitions src sends to dst (diagonal = kept)."""
    P = comm.world_size
    counts = [0] * P
    for pid in table.get_partition_ids():
        w = partitioner.get_worker_id(pid)
        counts[comm.rank if w == UNKNOWN_WORKER_ID else w] += 1
    return comm.all_gather_ints(counts)


def allgather_partition_set(comm: Communicator, table: Table) -> List[PartitionSet]:
    ids = torch.tensor(sorted(table.get_partition_ids()), dtype=torch.int64)
    msgs = comm.all_gather_bytes(ids.view(torch.uint8).to(comm.device))
    return [PartitionSet(r, m.cpu().view(torch.int64).tolist() if m.numel() else []) for r, m in enumerate(msgs)]


def gather_partition_set(comm: Communicator, table: Table, root: int = 0) -> Optional[List[PartitionSet]]:
    ids = torch.tensor(sorted(table.get_partition_ids()), dtype=torch.int64)
    msgs = comm.gather_bytes(ids.view(torch.uint8).to(comm.device), root)
    if msgs is None:
        return None
    return [PartitionSet(r, m.cpu().view(torch.int64).tolist() if m.numel() else []) for r, m in enumerate(msgs)]


def rotate_partition_count(comm: Communicator, table: Table, dest: int) -> PartitionCount:
    """Send my partition count to ``dest``; receive the count of whoever sends to me."""
    P = comm.world_size
    allc = comm.all_gather_ints([len(table), dest])
    for src in range(P):
        if int(allc[src, 1]) == comm.rank:
            return PartitionCount(src, int(allc[src, 0]))
    return PartitionCount(comm.rank, 0)


# ------------------------------------------------------------ object-list communication
def _msg(objs: Sequence[Any], comm: Communicator) -> torch.Tensor:
    meta, payload = encode_partitions([Partition(i, o) for i, o in enumerate(objs)], comm.device)
    return pack_message(meta, payload, comm.device)


def _objs(msg: torch.Tensor) -> List[Any]:
    return [p.get() for p in unpack_message(msg, None)]


def gather_objects(comm: Communicator, objs: Sequence[Any], root: int = 0) -> Optional[List[Any]]:
    msgs = comm.gather_bytes(_msg(objs, comm), root)
    if msgs is None:
        return None
    out: List[Any] = []
    for m in msgs:
        out += _objs(m)
    return out


def allgather_objects(comm: Communicator, objs: Sequence[Any]) -> List[Any]:
    out: List[Any] = []
    for m in comm.all_gather_bytes(_msg(objs, comm)):
        out += _objs(m)
    return out


def broadcast_objects(comm: Communicator, objs: Optional[Sequence[Any]], root: int = 0) -> List[Any]:
    """Chain / MST broadcast of an object list (RCCL picks the tree)."""
    msg = _msg(objs or [], comm) if comm.rank == root else None
    return _objs(comm.broadcast_bytes(msg, root)) if comm.world_size > 1 else list(objs or [])
