"""User-serializable objects (Harp ``Writable``) and the big-endian data streams.

Reference:
  * ``Writable``: encoding ``[WRITABLE byte][UTF class name][payload]``, instantiated by
    class name on decode (resource/Writable.java:36-51, :93 forClass, :127-152 abstract
    write/read/clear/getNumWriteBytes).
  * ``Serializer`` / ``Deserializer``: DataOutput/DataInput over a byte buffer; big-endian
    ints/longs (io/Serializer.java:167-193), floats/doubles by bit casts (:199-209),
    ``writeUTF`` = int length + UTF-16 chars (:223-239).
  * ``WritablePool``: per-class free lists (resource/WritablePool.java:62-189).

Decoding only instantiates classes registered with :func:`register_writable` (or
``Writable`` subclasses, which auto-register) — never arbitrary code from the stream.
"""
from __future__ import annotations

import struct
import threading
from collections import defaultdict
from typing import Dict, List, Type


class DataOutput:
    """Big-endian output stream (Serializer.java)."""

    __slots__ = ("_buf",)

    def __init__(self):
        self._buf = bytearray()

    def write_byte(self, v: int) -> None:
        self._buf += struct.pack(">b", v if v < 128 else v - 256)

    def write_ubyte(self, v: int) -> None:
        self._buf.append(v & 0xFF)

    def write_boolean(self, v: bool) -> None:
        self._buf.append(1 if v else 0)

    def write_short(self, v: int) -> None:
        self._buf += struct.pack(">h", v)

    def write_int(self, v: int) -> None:
        self._buf += struct.pack(">i", v)

    def write_long(self, v: int) -> None:
        self._buf += struct.pack(">q", v)

    def write_float(self, v: float) -> None:
        self._buf += struct.pack(">f", v)

    def write_double(self, v: float) -> None:
        self._buf += struct.pack(">d", v)

    def write_chars(self, s: str) -> None:
        self._buf += s.encode("utf-16-be")

    def write_utf(self, s: str) -> None:
        # Harp's writeUTF: int char count, then UTF-16 chars (Serializer.java:223-239)
        enc = s.encode("utf-16-be")
        self.write_int(len(enc) // 2)
        self._buf += enc

    def write_bytes(self, b: bytes) -> None:
        self._buf += b

    def getvalue(self) -> bytes:
        return bytes(self._buf)

    def __len__(self) -> int:
        return len(self._buf)


class DataInput:
    """Big-endian input stream (Deserializer.java)."""

    __slots__ = ("_buf", "pos")

    def __init__(self, buf: bytes | bytearray | memoryview, pos: int = 0):
        self._buf = memoryview(buf)
        self.pos = pos

    def _take(self, fmt: str, n: int):
        if self.pos + n > len(self._buf):
            raise EOFError("read past end of buffer")
        (v,) = struct.unpack_from(fmt, self._buf, self.pos)
        self.pos += n
        return v

    def read_byte(self) -> int:
        return self._take(">b", 1)

    def read_ubyte(self) -> int:
        return self._take(">B", 1)

    def read_boolean(self) -> bool:
        return self._take(">B", 1) != 0

    def read_short(self) -> int:
        return self._take(">h", 2)

    def read_int(self) -> int:
        return self._take(">i", 4)

    def read_long(self) -> int:
        return self._take(">q", 8)

    def read_float(self) -> float:
        return self._take(">f", 4)

    def read_double(self) -> float:
        return self._take(">d", 8)

    def read_utf(self) -> str:
        n = self.read_int()
        raw = self.read_bytes(2 * n)
        return raw.decode("utf-16-be")

    def read_bytes(self, n: int) -> bytes:
        if self.pos + n > len(self._buf):
            raise EOFError("read past end of buffer")
        b = bytes(self._buf[self.pos:self.pos + n])
        self.pos += n
        return b

    def remaining(self) -> int:
        return len(self._buf) - self.pos


_REGISTRY: Dict[str, Type["Writable"]] = {}
_REG_LOCK = threading.Lock()


def register_writable(cls: type, name: str | None = None) -> type:
    with _REG_LOCK:
        _REGISTRY[name or f"{cls.__module__}.{cls.__qualname__}"] = cls
    return cls


def writable_class(name: str) -> Type["Writable"]:
    try:
        return _REGISTRY[name]
    except KeyError:
        raise KeyError(f"Writable class {name!r} is not registered; refusing to decode") from None


def class_name(obj_or_cls) -> str:
    cls = obj_or_cls if isinstance(obj_or_cls, type) else type(obj_or_cls)
    return getattr(cls, "WRITABLE_NAME", None) or f"{cls.__module__}.{cls.__qualname__}"


class Writable:
    """Base class for user-defined serializable partition payloads."""

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        register_writable(cls, class_name(cls))

    # -- to override -----------------------------------------------------
    def write(self, out: DataOutput) -> None:  # pragma: no cover - abstract
        raise NotImplementedError

    def read(self, inp: DataInput) -> None:  # pragma: no cover - abstract
        raise NotImplementedError

    def clear(self) -> None:
        pass

    def num_write_bytes(self) -> int:
        out = DataOutput()
        self.write(out)
        return len(out)

    # -- lifecycle (pool) --------------------------------------------------
    @classmethod
    def create(cls):
        from .pool import ResourcePool

        return ResourcePool.get().writables.get_writable(cls)

    def release(self) -> None:
        from .pool import ResourcePool

        ResourcePool.get().writables.release_writable(self)

    def free(self) -> None:
        from .pool import ResourcePool

        ResourcePool.get().writables.free_writable(self)

    # -- helpers ------------------------------------------------------------
    def to_bytes(self) -> bytes:
        out = DataOutput()
        self.write(out)
        return out.getvalue()

    @classmethod
    def from_bytes(cls, b: bytes):
        obj = cls()
        obj.read(DataInput(b))
        return obj


class WritablePool:
    def __init__(self):
        self._free: Dict[type, List[Writable]] = defaultdict(list)
        self._in_use: Dict[int, type] = {}
        self._lock = threading.Lock()

    def get_writable(self, cls):
        with self._lock:
            free = self._free.get(cls)
            obj = free.pop() if free else cls()
            self._in_use[id(obj)] = cls
            return obj

    def release_writable(self, obj) -> bool:
        with self._lock:
            cls = self._in_use.pop(id(obj), None)
            if cls is None:
                return False
            obj.clear()
            self._free[cls].append(obj)
            return True

    def free_writable(self, obj) -> bool:
        with self._lock:
            return self._in_use.pop(id(obj), None) is not None

    def log(self) -> str:
        with self._lock:
            return f"WritablePool(in_use={len(self._in_use)}, free={sum(len(v) for v in self._free.values())})"
