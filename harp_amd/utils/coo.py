"""COO data-source pipeline: group -> remap IDs -> regroup -> CSR.

Reference: core/harp-daal-interface/.../datasource/HarpDAALDataSource.java —
``groupCOOByIDs`` (:358, MTReader.regroupCOO: a HashMap row -> COOGroup of (ids, vals)),
``remapCOOIDs`` (:365-397: allgather every worker's row IDs, assign compact 1-based IDs in
worker order, first occurrence wins), ``regroupCOOList`` (:399-437: re-key the groups by
compact ID, allreduce the max ID, regroup with COORegroupPartitioner — contiguous blocks of
``(maxID + 1 + P) // P`` IDs per worker — where COOGroupCombiner appends the entries of
equal IDs) and ``COOToCSR`` (:439-494: 1-based DAAL CSR, row offsets from 1, column
indices remapped, nFeatures = max column).

MI355X-first: a group set is four flat tensors (``gids``, ``offsets``, ``ids``, ``vals``)
instead of a HashMap of objects; the ID remap is one all-gather of the sorted unique IDs +
a searchsorted lookup table; the regroup is one all-to-all-v per array
(``models.mf_common.shuffle_coo``); the combine of equal IDs is a stable sort.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from ..parallel.comm import Communicator


@dataclass
class COOGroups:
    """Groups of COO entries keyed by ``gids`` (sorted, unique): group g holds
    ``ids[offsets[g]:offsets[g+1]]`` / ``vals[...]`` (the COOGroup payload)."""

    gids: torch.Tensor     # [G] int64
    offsets: torch.Tensor  # [G + 1] int64
    ids: torch.Tensor      # [n] int64, the other coordinate
    vals: torch.Tensor     # [n]

    @property
    def num_groups(self) -> int:
        return self.gids.numel()

    def group(self, g: int) -> Tuple[int, torch.Tensor, torch.Tensor]:
        a, b = int(self.offsets[g]), int(self.offsets[g + 1])
        return int(self.gids[g]), self.ids[a:b], self.vals[a:b]


def _groups_from(keys: torch.Tensor, ids: torch.Tensor, vals: torch.Tensor) -> COOGroups:
    order = torch.sort(keys, stable=True).indices
    k = keys[order]
    gids, counts = torch.unique_consecutive(k, return_counts=True)
    off = torch.zeros(gids.numel() + 1, dtype=torch.int64, device=keys.device)
    off[1:] = torch.cumsum(counts, 0)
    return COOGroups(gids.long(), off, ids[order].long(), vals[order])


def group_coo_by_ids(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, is_row: bool = True) -> COOGroups:
    """``groupCOOByIDs``: group the triples by row (``is_row``) or by column; entries keep
    their input order inside a group."""
    return _groups_from(rows, cols, vals) if is_row else _groups_from(cols, rows, vals)


@dataclass
class IDRemap:
    """Original ID -> compact 1-based ID (``remapCOOIDs``); lookup by binary search."""

    keys: torch.Tensor     # sorted original IDs
    compact: torch.Tensor  # compact ID of keys[i]

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        pos = torch.searchsorted(self.keys, x.long().to(self.keys.device))
        pos = pos.clamp_max(max(self.keys.numel() - 1, 0))
        if self.keys.numel() == 0 or not bool((self.keys[pos] == x.long().to(self.keys.device)).all()):
            raise KeyError("ID not in the remap table")
        return self.compact[pos]

    @property
    def max_id(self) -> int:
        return int(self.compact.max()) if self.compact.numel() else 0


def remap_coo_ids(comm: Communicator, gids: torch.Tensor) -> IDRemap:
    """All-gather every worker's group IDs; compact IDs 1, 2, ... are assigned in worker
    order (and ascending ID order within a worker), first occurrence wins."""
    mine = torch.unique(gids.long()).cpu()
    if comm.world_size > 1:
        from ..parallel.partition_util import allgather_objects

        per = allgather_objects(comm, [mine])
        allids = torch.cat([a.cpu().long() for a in per]) if per else mine
    else:
        allids = mine
    uniq, inv = torch.unique(allids, return_inverse=True)
    first = torch.full((uniq.numel(),), allids.numel(), dtype=torch.int64)
    first.scatter_reduce_(0, inv, torch.arange(allids.numel()), reduce="amin")
    rank_of = torch.empty(uniq.numel(), dtype=torch.int64)
    rank_of[torch.argsort(first)] = torch.arange(uniq.numel())
    return IDRemap(uniq, rank_of + 1)


def coo_regroup_owner(ids: torch.Tensor, max_id: int, P: int) -> torch.Tensor:
    """COORegroupPartitioner: IDs 1..max_id in contiguous blocks of (max_id + 1 + P) // P."""
    per = (max_id + 1 + P) // P
    ids = ids.long()
    ids = torch.where(ids > max_id, ids - (max_id + 1), ids)
    return torch.where(ids >= 0, ids // per, torch.zeros_like(ids)).clamp_max(P - 1)


def regroup_coo_list(comm: Communicator, groups: COOGroups, remap: IDRemap) -> Tuple[COOGroups, int]:
    """``regroupCOOList``: re-key groups by compact ID, allreduce the max compact ID, send
    every group to its COORegroupPartitioner owner and append the entries of equal IDs.
    Returns (the groups this worker owns, global max compact ID)."""
    counts = groups.offsets[1:] - groups.offsets[:-1]
    cg = remap(groups.gids).to(groups.ids.device)
    local_max = int(cg.max()) if cg.numel() else -1
    if comm.world_size > 1:
        import torch.distributed as dist

        t = torch.tensor([local_max], dtype=torch.int64, device=comm.device)
        comm.all_reduce(t, op=dist.ReduceOp.MAX)
        max_id = int(t.item())
    else:
        max_id = local_max
    key = torch.repeat_interleave(cg, counts)
    if comm.world_size > 1:
        from ..models.mf_common import shuffle_coo

        owner = coo_regroup_owner(key, max_id, comm.world_size)
        key, ids, vals = shuffle_coo(comm, owner.to(comm.device), key.to(comm.device), groups.ids.to(comm.device),
                                     groups.vals.to(comm.device))
        key, ids, vals = key.to(groups.ids.device), ids.to(groups.ids.device), vals.to(groups.ids.device)
    else:
        ids, vals = groups.ids, groups.vals
    return _groups_from(key, ids, vals), max_id


@dataclass
class DAALCSR:
    """DAAL-style 1-based CSR (``CSRNumericTable`` arrays)."""

    row_offsets: torch.Tensor  # [rows + 1], starts at 1
    col_index: torch.Tensor    # [nnz], 1-based
    values: torch.Tensor       # [nnz]
    n_features: int

    def to_torch(self) -> torch.Tensor:
        """0-based ``torch.sparse_csr_tensor`` of the same matrix."""
        return torch.sparse_csr_tensor(self.row_offsets - 1, self.col_index - 1, self.values,
                                       size=(self.row_offsets.numel() - 1, self.n_features))


def coo_to_csr(groups: COOGroups, col_remap: Optional[IDRemap] = None) -> Optional[DAALCSR]:
    """``COOToCSR``: one CSR row per group in ascending group-ID order; column indices are
    remapped with ``col_remap`` (1-based) or shifted to 1-based. None for an empty or
    inconsistent table (the reference logs "Wrong CSR format" and returns null)."""
    if groups.num_groups == 0:
        return None
    offs = groups.offsets + 1
    col = col_remap(groups.ids) if col_remap is not None else groups.ids + 1
    nf = int(col.max()) if col.numel() else 0
    if int(offs[-1]) - 1 != groups.vals.numel() or nf == 0:
        return None
    return DAALCSR(offs, col.long(), groups.vals, nf)
