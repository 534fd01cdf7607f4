"""Shared plumbing for the partial-result applications (the ml/daal family).

Reference pattern A: ``DistributedStep1Local.compute()`` on every worker
-> ``harpdaal_gather`` (a reduce of Java-serialized partial results onto the master,
harp-daal-interface data_comm/HarpDAALComm.java:158-294) -> ``DistributedStep2Master``
finalize; some algorithms broadcast the master's result for a step 3
(HarpDAALComm.java:78-156).

MI355X design: partial results are tensors; :func:`reduce_partials` packs a dict of them
into ONE flat device buffer (a single-partition :class:`PackedTable` with a SUM/MIN/MAX
combiner) and moves it with ONE RCCL allreduce (or reduce to the master), instead of
serialising objects. ``allreduce`` is the default so every worker can finalize locally
(no step-3 broadcast needed); ``to_master=True`` mirrors the reference's gather.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..core.combiner import ArrCombiner, Operation
from ..core.table import PackedTable
from ..parallel import collectives as C
from ..parallel.comm import Communicator


def reduce_partials(comm: Communicator, parts: Dict[str, torch.Tensor], op: Operation = Operation.SUM,
                    to_master: bool = False, dtype: torch.dtype = torch.float64) -> Optional[Dict[str, torch.Tensor]]:
    """Combine same-shaped partial tensors across workers with one collective."""
    if comm.world_size == 1:
        return {k: v.to(dtype) for k, v in parts.items()}
    keys = sorted(parts)
    shapes = [parts[k].shape for k in keys]
    flat = torch.cat([parts[k].reshape(-1).to(device=comm.device, dtype=dtype) for k in keys])
    t = PackedTable([0], flat.unsqueeze(0), combiner=ArrCombiner(op))
    t.static_layout = True
    ok = C.reduce(comm, t, 0) if to_master else C.allreduce(comm, t)
    if not ok:
        raise IOError("partial-result reduction failed")
    if to_master and comm.rank != 0:
        return None
    out, o = {}, 0
    buf = t.buffer[0]
    for k, s in zip(keys, shapes):
        n = 1
        for x in s:
            n *= x
        out[k] = buf[o:o + n].reshape(s)
        o += n
    return out


def broadcast_tensor(comm: Communicator, t: Optional[torch.Tensor], shape, dtype=torch.float64, root: int = 0):
    """Master -> all (the reference's step-2 -> step-3 harpdaal_braodcast)."""
    if comm.world_size == 1:
        return t
    buf = t.to(device=comm.device, dtype=dtype).contiguous() if comm.rank == root else torch.empty(
        shape, dtype=dtype, device=comm.device)
    comm.broadcast(buf, root)
    return buf


def gather_rows(comm: Communicator, rows: torch.Tensor) -> torch.Tensor:
    """All-gather variable-count row blocks [n_i, d] -> [sum n_i, d] (rank order)."""
    if comm.world_size == 1:
        return rows
    P = comm.world_size
    counts = comm.all_gather_ints([rows.shape[0]])[:, 0].tolist()
    mx = max(counts)
    if mx == 0:
        return rows.new_zeros((0,) + tuple(rows.shape[1:])).to(comm.device)
    buf = torch.zeros((mx,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=comm.device)
    buf[: rows.shape[0]] = rows.to(comm.device)
    out = torch.empty((P * mx,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=comm.device)
    comm.all_gather_into(out, buf)  # one padded all-gather (equal-size slabs)
    return torch.cat([out[r * mx:r * mx + counts[r]] for r in range(P)])


def dense_or_csr(x):
    """Accept a dense tensor or a torch sparse CSR/COO tensor."""
    return x.to_sparse_csr() if x.is_sparse else x
