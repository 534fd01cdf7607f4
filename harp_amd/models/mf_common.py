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
    """Assemble the full factor matrix [n_total, f] from each worker's owned rows."""
    if comm.world_size == 1:
        out = torch.zeros((n_total, F.shape[1]), dtype=F.dtype, device=F.device)
        out[ids.to(F.device)] = F
        return out
    from .common import gather_rows

    packed = torch.cat([ids.to(F.dtype).reshape(-1, 1), F], 1).to(comm.device)
    allr = gather_rows(comm, packed.double() if F.dtype != torch.float64 else packed)
    out = torch.zeros((n_total, F.shape[1]), dtype=F.dtype, device=comm.device)
    out[allr[:, 0].long()] = allr[:, 1:].to(F.dtype)
    return out


def local_index(ids_sorted: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Position of every x in the sorted id array."""
    return torch.searchsorted(ids_sorted, x)


def rmse(comm: Communicator, sse: torch.Tensor, n: int) -> float:
    from .common import reduce_partials

    r = reduce_partials(comm, {"s": sse.reshape(1).double().cpu(), "n": torch.tensor([float(n)])})
    return float((r["s"][0] / max(float(r["n"][0]), 1.0)) ** 0.5)
