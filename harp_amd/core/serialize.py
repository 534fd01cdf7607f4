"""Harp-compatible wire format (big-endian), for interop and the reference's tests.

Reference: io/Data.java:504-614 (head ``[byte bodyType][UTF ctx][int workerID][int
bodySize]([UTF opName])([int partitionID])``, for PARTITION_LIST the partition-id field
carries the number of partitions), io/DataUtil.java:288-465 (SIMPLE_LIST /
PARTITION_LIST bodies; an empty list encodes as a single UNKNOWN byte), typed arrays
``[type byte][int size][elements BE]`` (resource/DoubleArray.java:43-59), Writables
``[WRITABLE][UTF class][payload]`` (resource/Writable.java:36-51), partitions = payload
then int id (partition/Partition.java:66-78).

The collectives never use this element-wise format on the device path (they move raw
device bytes, :mod:`harp_amd.parallel.codec`); it exists so tables can be exchanged with
Harp-format producers/consumers and so the reference's encode/decode semantics are
testable. Array bodies are converted with numpy's big-endian dtypes (vectorised).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Union

import numpy as np
import torch

from .arrays import (ARRAY_CLASSES, BYTE_ARRAY, DOUBLE_ARRAY, FLOAT_ARRAY, INT_ARRAY, LONG_ARRAY, PARTITION_LIST,
                     SHORT_ARRAY, SIMPLE_LIST, UNKNOWN_DATA_TYPE, WRITABLE, Array)
from .partition import Partition
from .writable import DataInput, DataOutput, Writable, class_name, writable_class

_BE = {BYTE_ARRAY: ">i1", SHORT_ARRAY: ">i2", INT_ARRAY: ">i4", FLOAT_ARRAY: ">f4", LONG_ARRAY: ">i8",
       DOUBLE_ARRAY: ">f8"}
_TORCH2CODE = {torch.int8: BYTE_ARRAY, torch.uint8: BYTE_ARRAY, torch.int16: SHORT_ARRAY, torch.int32: INT_ARRAY,
               torch.float32: FLOAT_ARRAY, torch.int64: LONG_ARRAY, torch.float64: DOUBLE_ARRAY}


def encode_simple(obj, out: DataOutput) -> None:
    if isinstance(obj, Array):
        t, code = obj.tensor, obj.type_code
    elif isinstance(obj, torch.Tensor):
        t, code = obj.reshape(-1), _TORCH2CODE[obj.dtype]
    else:
        out.write_ubyte(WRITABLE)
        out.write_utf(class_name(obj))
        obj.write(out)
        return
    out.write_ubyte(code)
    a = t.detach().cpu().numpy()
    out.write_int(a.size)
    out.write_bytes(a.astype(_BE[code]).tobytes())


def decode_simple(inp: DataInput):
    code = inp.read_ubyte()
    if code == WRITABLE:
        obj = writable_class(inp.read_utf())()
        obj.read(inp)
        return obj
    if code not in _BE:
        raise ValueError(f"unknown data type {code}")
    n = inp.read_int()
    dt = np.dtype(_BE[code])
    a = np.frombuffer(inp.read_bytes(n * dt.itemsize), dtype=dt).astype(dt.newbyteorder("="))
    return ARRAY_CLASSES[code](torch.from_numpy(a.copy()))


def encode_partition_list(parts: Sequence[Partition]) -> bytes:
    out = DataOutput()
    if not parts:
        out.write_ubyte(UNKNOWN_DATA_TYPE)
        return out.getvalue()
    for p in parts:
        encode_simple(p.get(), out)
        out.write_int(p.id())
    return out.getvalue()


def decode_partition_list(b: bytes, count: int) -> List[Partition]:
    inp = DataInput(b)
    if count == 0:
        return []
    parts = []
    for _ in range(count):
        data = decode_simple(inp)
        parts.append(Partition(inp.read_int(), data))
    return parts


@dataclass
class Data:
    """A Harp message: head fields + decoded body (io/Data.java)."""

    body_type: int
    context_name: str
    worker_id: int
    body: list
    operation_name: Optional[str] = None
    partition_id: Optional[int] = None

    def is_operation_data(self) -> bool:
        return self.operation_name is not None

    def is_partition_data(self) -> bool:
        return self.body_type == PARTITION_LIST

    def encode(self) -> bytes:
        if self.body_type == PARTITION_LIST:
            body = encode_partition_list(self.body)
            pid = len(self.body)
        else:
            o = DataOutput()
            if not self.body:
                o.write_ubyte(UNKNOWN_DATA_TYPE)
            for x in self.body:
                encode_simple(x, o)
            body = o.getvalue()
            pid = self.partition_id
        head = DataOutput()
        head.write_ubyte(self.body_type)
        head.write_utf(self.context_name)
        head.write_int(self.worker_id)
        head.write_int(len(body))
        if self.operation_name is not None:
            head.write_utf(self.operation_name)
            if pid is not None:
                head.write_int(pid)
        h = head.getvalue()
        return len(h).to_bytes(4, "big") + h + body

    @classmethod
    def decode(cls, raw: bytes) -> "Data":
        hl = int.from_bytes(raw[:4], "big")
        inp = DataInput(raw[4:4 + hl])
        bt = inp.read_ubyte()
        ctx = inp.read_utf()
        wid = inp.read_int()
        blen = inp.read_int()
        op = inp.read_utf() if inp.remaining() else None
        pid = inp.read_int() if inp.remaining() else None
        body_raw = raw[4 + hl:4 + hl + blen]
        if bt == PARTITION_LIST:
            body = decode_partition_list(body_raw, pid or 0)
        else:
            body = []
            bi = DataInput(body_raw)
            if not (len(body_raw) == 1 and body_raw[0] == UNKNOWN_DATA_TYPE):
                while bi.remaining():
                    body.append(decode_simple(bi))
        return cls(bt, ctx, wid, body, op, pid)
