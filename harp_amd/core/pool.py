"""Array resource pools (Harp ``ResourcePool`` / ``ArrayPool``).

Reference: core/harp-collective/.../resource/ArrayPool.java — per-type free lists keyed
by exact size, or by the next power of two when ``approximate`` is requested
(:73-84 getAdjustedArraySize, :113 getArray, :177 releaseArray, :243 log); the
process-wide singleton is ResourcePool.java:41. Tests check 100 -> 128 rounding and
identity reuse after release (test/.../resource/DoublesPoolTest.java).

MI355X design: one pool keyed by (dtype, device, size). On a HIP device the pool sits
on top of torch's caching allocator, so it is a second-level free list that keeps hot
communication/packing buffers pinned to a size class across iterations (no
hipMalloc/hipFree in the iteration loop, graph-capture safe). HBM3E is the only
memory tier, so the reference's memkind/MCDRAM placement has no equivalent.
"""
from __future__ import annotations

import threading
from collections import defaultdict
from typing import Dict, List, Tuple

import torch


def adjusted_size(size: int, approximate: bool) -> int:
    """Exact size, or the next power of two >= size when approximate."""
    if size < 0:
        raise ValueError("negative array size")
    if not approximate or size <= 1:
        return max(size, 0)
    return 1 << (size - 1).bit_length()


class ArrayPool:
    def __init__(self):
        self._free: Dict[Tuple[torch.dtype, str, int], List[torch.Tensor]] = defaultdict(list)
        self._in_use: Dict[int, Tuple[torch.dtype, str, int]] = {}
        self._lock = threading.Lock()
        self.hits = 0
        self.misses = 0

    def get_array(self, dtype: torch.dtype, size: int, approximate: bool = True,
                  device: torch.device | str = "cpu") -> torch.Tensor:
        dev = str(torch.device(device))
        n = adjusted_size(size, approximate)
        key = (dtype, dev, n)
        with self._lock:
            free = self._free.get(key)
            if free:
                t = free.pop()
                self.hits += 1
            else:
                t = torch.empty(n, dtype=dtype, device=dev)
                self.misses += 1
            self._in_use[id(t)] = key
        return t

    def release_array(self, t: torch.Tensor) -> bool:
        with self._lock:
            key = self._in_use.pop(id(t), None)
            if key is None:
                return False
            self._free[key].append(t)
            return True

    def free_array(self, t: torch.Tensor) -> bool:
        with self._lock:
            return self._in_use.pop(id(t), None) is not None

    def clean(self) -> None:
        with self._lock:
            self._free.clear()

    def stats(self) -> dict:
        with self._lock:
            return {
                "in_use": len(self._in_use),
                "free": sum(len(v) for v in self._free.values()),
                "free_bytes": sum(t.numel() * t.element_size() for v in self._free.values() for t in v),
                "hits": self.hits,
                "misses": self.misses,
            }

    def log(self) -> str:
        return f"ArrayPool {self.stats()}"


class ResourcePool:
    """Process-wide singleton (ResourcePool.get())."""

    _instance: "ResourcePool | None" = None
    _lock = threading.Lock()

    def __init__(self):
        self.arrays = ArrayPool()
        from .writable import WritablePool

        self.writables = WritablePool()

    @classmethod
    def get(cls) -> "ResourcePool":
        with cls._lock:
            if cls._instance is None:
                cls._instance = ResourcePool()
            return cls._instance

    def log(self) -> str:
        return f"{self.arrays.log()} {self.writables.log()}"
