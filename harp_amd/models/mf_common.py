"""Shared plumbing for the matrix-factorisation family (ALS, CCD++).

Reference: ratings are read as ``row col value`` text per worker and regrouped by row
(or column) owner (ml/java/.../ccd/CCDMPCollectiveMapper.java:330 regroup,
harp-daal-interface HarpDAALDataSource.regroupCOOList). Here the regroup of COO triples
is one all-to-all-v per array (``alltoall`` over RCCL), and factor blocks owned by
different workers are assembled with one all-gather.
"""
from __future__ import annotations

from typing import Tuple

import torch

from ..parallel.comm import Communicator


def shuffle_coo(comm: Communicator, owner: torch.Tensor, *arrays: torch.Tensor) -> Tuple[torch.Tensor, ...]:
    """Send element k of every array to worker ``owner[k]`` (all-to-all-v)."""
    P = comm.world_size
    if P == 1:
        return arrays
    dev = comm.device
    order = torch.argsort(owner, stable=True)
    counts = torch.bincount(owner, minlength=P).to(torch.int64)
    rc = torch.empty(P, dtype=torch.int64, device=dev)
    comm.all_to_all_single(rc, counts.to(dev))
    ss, rs = counts.tolist(), rc.cpu().tolist()
    out = []
    for a in arrays:
        send = a[order].contiguous().to(dev)
        recv = torch.empty(sum(rs), dtype=a.dtype, device=dev)
        comm.all_to_all_single(recv, send, rs, ss)
        out.append(recv)
    return tuple(out)


def gather_factors(comm: Communicator, ids: torch.Tensor, F: torch.Tensor, n_total: int) -> torch.Tensor:
    """Assemble the full factor matrix [n_total, f] from each worker's owned rows.

    The int64 row ids and the factor rows travel as two separate all-gathers (ids are
    never cast to the factor dtype: fp32 cannot hold every id above 2^24)."""
    if comm.world_size == 1:
        out = torch.zeros((n_total, F.shape[1]), dtype=F.dtype, device=F.device)
        out[ids.to(F.device)] = F
        return out
    from .common import gather_rows

    all_ids = gather_rows(comm, ids.to(comm.device, torch.int64).reshape(-1, 1))[:, 0]
    all_rows = gather_rows(comm, F.to(comm.device).contiguous())
    out = torch.zeros((n_total, F.shape[1]), dtype=F.dtype, device=comm.device)
    out[all_ids] = all_rows.to(F.dtype)
    return out


class FactorCheckpoint:
    """Periodic ``.hpt`` checkpoints of row-sharded factor matrices (CCD W/H, ALS X/Y):
    each rank saves its owned rows under their global ids, so a restart with any world
    size re-shards by id (rank r keeps the ids it owns under its own layout)."""

    def __init__(self, comm: Communicator, directory: str, every: int):
        from ..utils.checkpoint import Checkpointer

        self.ck = Checkpointer(directory, comm, every)

    def maybe_save(self, it: int, factors, history) -> None:
        from ..utils.checkpoint import tensor_table

        if self.ck.due(it):
            self.ck.save(it, {n: tensor_table(F, ids) for n, (F, ids) in factors.items()},
                         extra={"history": list(history)})

    def resume(self, factors, history):
        """Fill every ``factors[name] = (F, ids, n_total)`` in place from the latest
        checkpoint; returns (first iteration to run, restored history)."""
        got = self.ck.load_latest(device="cpu", rng=True)
        if got is None:
            return 0, history
        man, tabs = got
        for name, (F, ids, n_total) in factors.items():
            t = tabs[name]
            full = torch.zeros((n_total, F.shape[1]), dtype=F.dtype)
            full[torch.tensor(t.ids, dtype=torch.long)] = t.buffer.to(F.dtype)
            F.copy_(full[ids.cpu()].to(F.device))
        return int(man["iteration"]) + 1, list(man["extra"].get("history", []))


def save_factor_models(comm: Communicator, folder: str, factors) -> None:
    """Text dumps ``<name>-<worker>`` (``id : v1 .. vr``, SGDCollectiveMapper.java:737-818)."""
    from ..utils.model_io import write_factor_rows

    for name, (F, ids) in factors.items():
        write_factor_rows(f"{folder}/{name}-{comm.rank}", ids, F)


def local_index(ids_sorted: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Position of every x in the sorted id array."""
    return torch.searchsorted(ids_sorted, x)


def rmse(comm: Communicator, sse: torch.Tensor, n: int) -> float:
    from .common import reduce_partials

    r = reduce_partials(comm, {"s": sse.reshape(1).double().cpu(), "n": torch.tensor([float(n)])})
    return float((r["s"][0] / max(float(r["n"][0]), 1.0)) ** 0.5)
