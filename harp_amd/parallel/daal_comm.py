"""Object-level communication of partial results (harp-daal-interface HarpDAALComm).

Reference: core/harp-daal-interface/.../data_comm/HarpDAALComm.java:78-337 — Java-serialize
a DAAL ``SerializableBase`` into a one-partition ``Table<ByteArray>`` and move it:
``harpdaal_braodcast`` (barrier + broadcast + barrier), ``harpdaal_gather`` (reduce of
distinct-id partitions onto the root), ``harpdaal_allgather`` (allreduce over distinct ids).

Here partial results are tensors / Writables / plain Python values encoded by the
framework codec (no pickle on the wire for tensors: raw bytes + a small header); the
single-buffer tensor fast path (:func:`models.common.reduce_partials`) is what the apps
use, this class keeps the reference's object-granular API for user code.
"""
from __future__ import annotations

from typing import Any, List, Optional

from .comm import Communicator
from .partition_util import allgather_objects, broadcast_objects, gather_objects


class HarpDAALComm:
    def __init__(self, comm: Communicator, root: int = 0):
        self.comm, self.root = comm, root

    def harpdaal_braodcast(self, obj: Any = None, root: Optional[int] = None) -> Any:
        """Root's object on every worker (the reference's spelling kept as an alias)."""
        r = self.root if root is None else root
        self.comm.barrier()
        out = broadcast_objects(self.comm, [obj] if self.comm.rank == r else None, r)[0]
        self.comm.barrier()
        return out

    harpdaal_broadcast = harpdaal_braodcast

    def harpdaal_gather(self, obj: Any, root: Optional[int] = None) -> Optional[List[Any]]:
        """Every worker's object, in rank order, on the root (None elsewhere)."""
        r = self.root if root is None else root
        return gather_objects(self.comm, [obj], r)

    def harpdaal_allgather(self, obj: Any) -> List[Any]:
        return allgather_objects(self.comm, [obj])
