"""Partition, Partitioner, PartitionFunction (Harp L2).

Reference:
  * ``Partition``: (int id, payload) — partition/Partition.java:32; encoded as payload
    then int id (:66-78).
  * ``Partitioner``: partition id -> worker id, default ``abs(id % P)``
    (partition/Partitioner.java:36-43). ``UNKNOWN_WORKER_ID`` keeps a partition local
    (partition/PartitionUtil.java:143-161).
  * ``PartitionFunction``: per-partition UDF applied after regroup
    (partition/PartitionFunction.java:25-27).
"""
from __future__ import annotations

import random
from typing import Any, Generic, TypeVar

import torch

from .arrays import Array

UNKNOWN_WORKER_ID = -1
UNKNOWN_PARTITION_ID = -1

P = TypeVar("P")


class Partition(Generic[P]):
    __slots__ = ("_id", "_data")

    def __init__(self, partition_id: int, data: P):
        self._id = int(partition_id)
        self._data = data

    def id(self) -> int:
        return self._id

    @property
    def pid(self) -> int:
        return self._id

    def get(self) -> P:
        return self._data

    @property
    def data(self) -> P:
        return self._data

    def set(self, data: P) -> None:
        self._data = data

    def release(self) -> None:
        rel = getattr(self._data, "release", None)
        if rel is not None:
            rel()

    def free(self) -> None:
        fr = getattr(self._data, "free", None)
        if fr is not None:
            fr()

    def num_encode_bytes(self) -> int:
        d = self._data
        if isinstance(d, torch.Tensor):
            return 5 + d.numel() * d.element_size() + 4
        if isinstance(d, Array):
            return d.num_encode_bytes() + 4
        nb = getattr(d, "num_write_bytes", None)
        return (nb() if nb else 0) + 4

    def __repr__(self) -> str:
        d = self._data
        desc = f"{tuple(d.shape)} {d.dtype} {d.device}" if isinstance(d, torch.Tensor) else type(d).__name__
        return f"Partition({self._id}, {desc})"


class Partitioner:
    """Default partitioner: ``abs(id % num_workers)``."""

    def __init__(self, num_workers: int):
        if num_workers <= 0:
            raise ValueError("num_workers must be positive")
        self.num_workers = int(num_workers)

    def get_worker_id(self, partition_id: int) -> int:
        # Java's % keeps the dividend's sign; Harp then takes abs().
        r = abs(int(partition_id)) % self.num_workers
        return r

    # vectorised form used by the packed fast paths
    def worker_ids(self, ids: torch.Tensor) -> torch.Tensor:
        return ids.abs() % self.num_workers

    def __call__(self, partition_id: int) -> int:
        return self.get_worker_id(partition_id)


class MapPartitioner(Partitioner):
    """Explicit id -> worker map; ids not in the map use ``default`` (UNKNOWN keeps local)."""

    def __init__(self, num_workers: int, mapping: dict[int, int], default: int = UNKNOWN_WORKER_ID):
        super().__init__(num_workers)
        self.mapping = dict(mapping)
        self.default = default

    def get_worker_id(self, partition_id: int) -> int:
        return self.mapping.get(int(partition_id), self.default)

    def worker_ids(self, ids: torch.Tensor) -> torch.Tensor:
        return torch.tensor([self.get_worker_id(int(i)) for i in ids.tolist()], dtype=torch.long)


class RandomPartitioner(Partitioner):
    """Seeded random owner per partition id (ml/java/.../sgd/RandomPartitioner.java):
    every worker computes the same assignment from the shared seed."""

    def __init__(self, num_workers: int, seed: int):
        super().__init__(num_workers)
        self.seed = int(seed)
        self._cache: dict[int, int] = {}

    def get_worker_id(self, partition_id: int) -> int:
        pid = int(partition_id)
        w = self._cache.get(pid)
        if w is None:
            w = random.Random((self.seed << 32) ^ pid).randrange(self.num_workers)
            self._cache[pid] = w
        return w

    def worker_ids(self, ids: torch.Tensor) -> torch.Tensor:
        return torch.tensor([self.get_worker_id(int(i)) for i in ids.tolist()], dtype=torch.long)


class PartitionFunction:
    """UDF applied to each partition after regroup (regroupAggregate / aggregate)."""

    def apply(self, data: Any) -> Any:  # pragma: no cover - abstract
        raise NotImplementedError

    def __call__(self, data: Any) -> Any:
        return self.apply(data)
