"""Typed arrays (Harp ``ByteArray`` … ``DoubleArray``).

Reference: core/harp-collective/.../resource/Array.java:23-75 — an array is
(array, start, size); ``DoubleArray.create(size, approximate)`` draws from the pool
(DoubleArray.java:69), ``release()`` returns it, ``free()`` drops it. Wire encoding
``[type byte][int size][elements, big-endian]`` (DoubleArray.java:43-59) is provided by
:mod:`harp_amd.core.serialize`.

Here an ``Array`` is a view ``tensor[start:start+size]`` of a 1-D torch tensor, so a
typed array can live in HBM and be handed to RCCL / HIP kernels without copies.
Combiners and collectives accept either an ``Array`` or a bare ``torch.Tensor``.
"""
from __future__ import annotations

from typing import ClassVar

import torch

from .pool import ResourcePool

# Harp DataType codes (io/DataType.java:24-33)
BYTE_ARRAY = 1
SHORT_ARRAY = 2
INT_ARRAY = 3
FLOAT_ARRAY = 4
LONG_ARRAY = 5
DOUBLE_ARRAY = 6
WRITABLE = 7
SIMPLE_LIST = 8
PARTITION_LIST = 9
UNKNOWN_DATA_TYPE = 255

DTYPE_TO_CODE = {
    torch.int8: BYTE_ARRAY,
    torch.uint8: BYTE_ARRAY,
    torch.int16: SHORT_ARRAY,
    torch.int32: INT_ARRAY,
    torch.float32: FLOAT_ARRAY,
    torch.int64: LONG_ARRAY,
    torch.float64: DOUBLE_ARRAY,
}
CODE_TO_DTYPE = {
    BYTE_ARRAY: torch.int8,
    SHORT_ARRAY: torch.int16,
    INT_ARRAY: torch.int32,
    FLOAT_ARRAY: torch.float32,
    LONG_ARRAY: torch.int64,
    DOUBLE_ARRAY: torch.float64,
}


class Array:
    """A (tensor, start, size) view. Subclasses fix the element dtype."""

    dtype: ClassVar[torch.dtype] = torch.float64
    type_code: ClassVar[int] = DOUBLE_ARRAY

    __slots__ = ("_base", "start", "size", "_pooled")

    def __init__(self, base: torch.Tensor, start: int = 0, size: int | None = None):
        if base.dim() != 1:
            base = base.reshape(-1)
        if base.dtype != self.dtype:
            raise TypeError(f"{type(self).__name__} needs {self.dtype}, got {base.dtype}")
        self._base = base
        self.start = int(start)
        self.size = int(base.numel() - start if size is None else size)
        if self.start < 0 or self.start + self.size > base.numel():
            raise ValueError("array view out of range")
        self._pooled = False

    # -- construction -----------------------------------------------------
    @classmethod
    def create(cls, size: int, approximate: bool = True, device: str | torch.device = "cpu") -> "Array":
        t = ResourcePool.get().arrays.get_array(cls.dtype, size, approximate, device)
        a = cls(t, 0, size)
        a._pooled = True
        return a

    @classmethod
    def wrap(cls, data, device: str | torch.device | None = None) -> "Array":
        t = torch.as_tensor(data, dtype=cls.dtype, device=device).reshape(-1)
        return cls(t)

    # -- access -------------------------------------------------------------
    def get(self) -> torch.Tensor:
        """The backing tensor (Harp's ``get()`` returns the whole backing array)."""
        return self._base

    @property
    def tensor(self) -> torch.Tensor:
        return self._base[self.start:self.start + self.size]

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, i):
        return self.tensor[i]

    def __setitem__(self, i, v):
        self.tensor[i] = v

    def num_encode_bytes(self) -> int:
        # [type byte][int size][elements]
        return 5 + self.size * self.tensor.element_size()

    def release(self) -> None:
        if self._pooled:
            ResourcePool.get().arrays.release_array(self._base)
            self._pooled = False

    def free(self) -> None:
        if self._pooled:
            ResourcePool.get().arrays.free_array(self._base)
            self._pooled = False

    def __repr__(self) -> str:
        return f"{type(self).__name__}(size={self.size}, start={self.start}, device={self._base.device})"


class ByteArray(Array):
    dtype = torch.int8
    type_code = BYTE_ARRAY


class ShortArray(Array):
    dtype = torch.int16
    type_code = SHORT_ARRAY


class IntArray(Array):
    dtype = torch.int32
    type_code = INT_ARRAY


class FloatArray(Array):
    dtype = torch.float32
    type_code = FLOAT_ARRAY


class LongArray(Array):
    dtype = torch.int64
    type_code = LONG_ARRAY


class DoubleArray(Array):
    dtype = torch.float64
    type_code = DOUBLE_ARRAY


ARRAY_CLASSES = {c.type_code: c for c in (ByteArray, ShortArray, IntArray, FloatArray, LongArray, DoubleArray)}


def as_tensor(x) -> torch.Tensor | None:
    if isinstance(x, torch.Tensor):
        return x
    if isinstance(x, Array):
        return x.tensor
    return None
