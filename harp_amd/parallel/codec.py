"""Partition-list codec for the generic (heterogeneous) collective path.

The reference encodes every partition element-by-element, big-endian, into a Java
byte[] and decodes it on the receiver (io/DataUtil.java:288-394, Partition.java:74,
DoubleArray.java:51-59; SURVEY §3.2 calls this the hot loop). Here:

  * tensor payloads are never serialized element-wise: their raw bytes are viewed as
    ``uint8`` and concatenated *on the communication device* (HBM for RCCL), so the
    whole table moves as one device buffer and decodes into zero-copy views;
  * only the small metadata record (ids, dtype, shape, byte offsets) and non-tensor
    payloads (Writables, KV maps) are built on the host.

Metadata layout (little-endian): ``int32 n`` then per partition
``int32 id, uint8 kind, ...`` — kind TENSOR: ``uint8 dtype, uint8 device_kind,
uint8 ndim, int64 shape[ndim]``; kind ARRAY: ``uint8 type_code``; kind WRITABLE:
``uint16 len, utf8 class name``; all kinds end with ``int64 nbytes``. Each payload
chunk starts at a 16-byte aligned offset (so ``view(dtype)`` is legal).
"""
from __future__ import annotations

import struct
from typing import List, Sequence, Tuple

import torch

from ..core.arrays import ARRAY_CLASSES, Array
from ..core.partition import Partition
from ..core.writable import DataInput, DataOutput, class_name, writable_class

KIND_TENSOR = 0
KIND_ARRAY = 1
KIND_WRITABLE = 2

_DTYPES = [
    torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int8, torch.uint8,
    torch.int16, torch.int32, torch.int64, torch.bool, torch.complex64, torch.complex128,
]
_DTYPE_CODE = {d: i for i, d in enumerate(_DTYPES)}
ALIGN = 16


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _payload(data) -> Tuple[int, tuple, object]:
    """Returns (kind, meta fields, raw) where raw is a tensor or bytes."""
    if isinstance(data, torch.Tensor):
        dev_kind = 1 if data.device.type == "cuda" else 0
        return KIND_TENSOR, (_DTYPE_CODE[data.dtype], dev_kind, tuple(data.shape)), data
    if isinstance(data, Array):
        return KIND_ARRAY, (data.type_code,), data.tensor
    if hasattr(data, "write") and hasattr(data, "read"):
        out = DataOutput()
        data.write(out)
        return KIND_WRITABLE, (class_name(data),), out.getvalue()
    raise TypeError(f"cannot encode partition payload of type {type(data).__name__}")


def encode_partitions(parts: Sequence[Partition], device: torch.device) -> Tuple[bytes, torch.Tensor]:
    """Encode partitions into (meta bytes, uint8 payload tensor on ``device``)."""
    meta = bytearray(struct.pack("<i", len(parts)))
    chunks: List[torch.Tensor] = []
    offset = 0
    for p in parts:
        kind, fields, raw = _payload(p.get())
        meta += struct.pack("<iB", p.id(), kind)
        if kind == KIND_TENSOR:
            code, dev_kind, shape = fields
            meta += struct.pack("<BBB", code, dev_kind, len(shape))
            meta += struct.pack(f"<{len(shape)}q", *shape) if shape else b""
        elif kind == KIND_ARRAY:
            meta += struct.pack("<B", fields[0])
        else:
            name = fields[0].encode("utf-8")
            meta += struct.pack("<H", len(name)) + name
        if isinstance(raw, torch.Tensor):
            t = raw.detach()
            if not t.is_contiguous():
                t = t.contiguous()
            b = t.reshape(-1).view(torch.uint8)
            if b.device != device:
                b = b.to(device, non_blocking=True)
        else:
            b = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.empty(0, dtype=torch.uint8)
            if b.device != device:
                b = b.to(device)
        nbytes = b.numel()
        meta += struct.pack("<q", nbytes)
        chunks.append(b)
        pad = _align(nbytes) - nbytes
        if pad:
            chunks.append(torch.zeros(pad, dtype=torch.uint8, device=device))
        offset += nbytes + pad
    payload = torch.cat(chunks) if chunks else torch.empty(0, dtype=torch.uint8, device=device)
    return bytes(meta), payload


def decode_partitions(meta: bytes | memoryview, payload: torch.Tensor,
                      home_device: torch.device | None = None) -> List[Partition]:
    """Decode partitions. Tensor payloads become views into ``payload`` (moved to the
    CPU when they originated on the host, or to ``home_device`` otherwise)."""
    mv = memoryview(meta)
    (n,) = struct.unpack_from("<i", mv, 0)
    pos = 4
    off = 0
    out: List[Partition] = []
    for _ in range(n):
        pid, kind = struct.unpack_from("<iB", mv, pos)
        pos += 5
        if kind == KIND_TENSOR:
            code, dev_kind, ndim = struct.unpack_from("<BBB", mv, pos)
            pos += 3
            shape = struct.unpack_from(f"<{ndim}q", mv, pos) if ndim else ()
            pos += 8 * ndim
        elif kind == KIND_ARRAY:
            (tcode,) = struct.unpack_from("<B", mv, pos)
            pos += 1
        else:
            (ln,) = struct.unpack_from("<H", mv, pos)
            pos += 2
            name = bytes(mv[pos:pos + ln]).decode("utf-8")
            pos += ln
        (nbytes,) = struct.unpack_from("<q", mv, pos)
        pos += 8
        raw = payload[off:off + nbytes]
        off += _align(nbytes)
        if kind == KIND_TENSOR:
            dt = _DTYPES[code]
            t = raw.view(dt).reshape(shape) if nbytes else torch.empty(shape, dtype=dt, device=payload.device)
            if dev_kind == 0 and t.device.type != "cpu":
                t = t.cpu()
            elif dev_kind == 1 and home_device is not None and t.device != home_device:
                t = t.to(home_device)
            elif dev_kind == 1 and t.device.type == "cpu" and torch.cuda.is_available():
                t = t.to(home_device or torch.device("cuda", torch.cuda.current_device()))
            out.append(Partition(pid, t))
        elif kind == KIND_ARRAY:
            cls = ARRAY_CLASSES[tcode]
            t = raw.view(cls.dtype).clone() if nbytes else torch.empty(0, dtype=cls.dtype)
            out.append(Partition(pid, cls(t)))
        else:
            cls = writable_class(name)
            obj = cls()
            obj.read(DataInput(raw.cpu().numpy().tobytes()))
            out.append(Partition(pid, obj))
    return out


def pack_message(meta: bytes, payload: torch.Tensor, device: torch.device) -> torch.Tensor:
    """One contiguous uint8 message: [int64 meta_len][meta][pad][payload]."""
    head = struct.pack("<q", len(meta)) + meta
    hb = torch.frombuffer(bytearray(head + b"\0" * (_align(len(head)) - len(head))), dtype=torch.uint8)
    return torch.cat([hb.to(device), payload]) if payload.numel() else hb.to(device)


def unpack_message(msg: torch.Tensor, home_device: torch.device | None = None) -> List[Partition]:
    if msg.numel() == 0:
        return []
    head8 = msg[:8].cpu().numpy().tobytes()
    (mlen,) = struct.unpack("<q", head8)
    meta = msg[8:8 + mlen].cpu().numpy().tobytes()
    start = _align(8 + mlen)
    return decode_partitions(meta, msg[start:], home_device)
