"""Partition-table checkpoint / resume (the ``.hpt`` format).

The reference has no checkpoint/resume — only final model dumps (K-means centroids as
text, KMUtil.java:213-252; SGD ``W-<worker>``/``H-<worker>``, SGDCollectiveMapper.java:
737-818; LDA periodic word-model dumps). Its only self-describing binary format is the
Table wire encoding. This module adds a per-rank binary checkpoint of any table plus a
JSON manifest tying ranks together:

``table-<name>-r<rank>.hpt``::

    header  (little-endian): magic b"HPT1", u32 version=1, i32 table_id, u8 kind
            (0 generic / 1 packed), 32-byte combiner op name, i32 world, i32 rank,
            i64 num_partitions, i64 index_offset
    payload 256-byte-aligned raw partition buffers (tensors copied device->host once)
            or Harp-format Writable bytes
    index   per partition: i32 id, u8 kind (0 tensor, 1 writable), u8 dtype code,
            u8 ndim, i64 shape[ndim], i64 offset, i64 nbytes, u32 crc32; writables add
            u16 len + class name

``manifest-<name>.json``: iteration, world size, per-rank files, RNG state, user extras.

Resume loads a rank's partitions back (onto any device); loading with a different world
size returns all partitions of the listed files, which the caller re-shards with a
regroup under the table's partitioner.
"""
from __future__ import annotations

import json
import os
import struct
import zlib
from typing import Dict, List, Optional

import torch

from ..core.combiner import ArrCombiner, Operation
from ..core.partition import Partition
from ..core.table import PackedTable, Table
from ..core.writable import DataInput, DataOutput, class_name, writable_class

MAGIC = b"HPT1"
VERSION = 1
ALIGN = 256
_DT = [torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int8, torch.uint8, torch.int16,
       torch.int32, torch.int64, torch.bool]
_DTC = {d: i for i, d in enumerate(_DT)}
_HDR = struct.Struct("<4sIiB32siiqq")


def _op_name(table: Table) -> str:
    op = getattr(table.combiner, "operation", None)
    return op.value if op is not None else type(table.combiner).__name__


def save_table(table: Table, path: str, rank: int = 0, world: int = 1) -> None:
    tmp = path + ".tmp"
    entries = []
    with open(tmp, "wb") as f:
        f.write(b"\0" * _HDR.size)
        off = _HDR.size
        parts = table.get_partitions()
        packed = isinstance(table, PackedTable)
        host_buf = table.buffer.detach().cpu() if packed else None  # one D2H copy for packed tables
        for idx, p in enumerate(parts):
            d = p.get()
            pad = (-off) % ALIGN
            f.write(b"\0" * pad)
            off += pad
            if packed:
                t = host_buf[table.row_of(p.id())]
            else:
                t = d if isinstance(d, torch.Tensor) else getattr(d, "tensor", None)
            if isinstance(t, torch.Tensor):
                t = t.detach().cpu().contiguous()
                raw = t.reshape(-1).view(torch.uint8).numpy().tobytes() if t.numel() else b""
                entries.append((p.id(), 0, _DTC[t.dtype], tuple(t.shape), off, len(raw), zlib.crc32(raw), None))
            else:
                o = DataOutput()
                d.write(o)
                raw = o.getvalue()
                entries.append((p.id(), 1, 0, (), off, len(raw), zlib.crc32(raw), class_name(d)))
            f.write(raw)
            off += len(raw)
        index_off = off
        for pid, kind, dt, shape, o, n, crc, cname in entries:
            f.write(struct.pack("<iBBB", pid, kind, dt, len(shape)))
            f.write(struct.pack(f"<{len(shape)}q", *shape))
            f.write(struct.pack("<qqI", o, n, crc))
            if kind == 1:
                nb = cname.encode()
                f.write(struct.pack("<H", len(nb)) + nb)
        f.seek(0)
        f.write(_HDR.pack(MAGIC, VERSION, table.table_id, 1 if packed else 0, _op_name(table).encode()[:32],
                          world, rank, len(entries), index_off))
    os.replace(tmp, path)


def load_table(path: str, device: str | torch.device = "cpu", combiner=None, verify: bool = True) -> Table:
    with open(path, "rb") as f:
        raw = f.read()
    magic, ver, tid, kind, opname, world, rank, n, index_off = _HDR.unpack_from(raw, 0)
    if magic != MAGIC or ver != VERSION:
        raise ValueError(f"{path}: not a harp .hpt v{VERSION} file")
    opname = opname.rstrip(b"\0").decode()
    if combiner is None:
        try:
            combiner = ArrCombiner(Operation(opname))
        except ValueError:
            combiner = ArrCombiner(Operation.SUM)
    pos = index_off
    parts: List[Partition] = []
    for _ in range(n):
        pid, k, dt, nd = struct.unpack_from("<iBBB", raw, pos)
        pos += 7
        shape = struct.unpack_from(f"<{nd}q", raw, pos)
        pos += 8 * nd
        o, nb, crc = struct.unpack_from("<qqI", raw, pos)
        pos += 20
        cname = None
        if k == 1:
            (ln,) = struct.unpack_from("<H", raw, pos)
            cname = raw[pos + 2:pos + 2 + ln].decode()
            pos += 2 + ln
        blob = raw[o:o + nb]
        if verify and zlib.crc32(blob) != crc:
            raise IOError(f"{path}: CRC mismatch in partition {pid}")
        if k == 0:
            t = (torch.frombuffer(bytearray(blob), dtype=torch.uint8).view(_DT[dt]).reshape(shape) if nb
                 else torch.empty(shape, dtype=_DT[dt]))
            parts.append(Partition(pid, t.to(device)))
        else:
            obj = writable_class(cname)()
            obj.read(DataInput(blob))
            parts.append(Partition(pid, obj))
    if kind == 1 and parts:
        ids = [p.id() for p in parts]
        return PackedTable(ids, torch.stack([p.get() for p in parts]), table_id=tid, combiner=combiner)
    t = Table(tid, combiner)
    for p in parts:
        t.insert_partition(p)
    return t


def save_checkpoint(directory: str, tables: Dict[str, Table], rank: int, world: int, iteration: int,
                    extra: Optional[dict] = None, comm=None) -> str:
    """Every rank writes its tables; rank 0 writes the manifest (after a barrier when a
    communicator is given, so the manifest only appears once all shards exist)."""
    os.makedirs(directory, exist_ok=True)
    for name, t in tables.items():
        save_table(t, os.path.join(directory, f"table-{name}-r{rank}.hpt"), rank, world)
    if comm is not None:
        comm.barrier()
    if rank == 0:
        man = {"version": VERSION, "iteration": iteration, "world": world,
               "tables": {n: [f"table-{n}-r{r}.hpt" for r in range(world)] for n in tables},
               "rng": {"torch": torch.random.get_rng_state().tolist()[:16]}, "extra": extra or {}}
        tmp = os.path.join(directory, "manifest.json.tmp")
        with open(tmp, "w") as f:
            json.dump(man, f)
        os.replace(tmp, os.path.join(directory, "manifest.json"))
    return directory


def load_checkpoint(directory: str, rank: int, world: int, device="cpu") -> tuple:
    with open(os.path.join(directory, "manifest.json")) as f:
        man = json.load(f)
    out = {}
    for name, files in man["tables"].items():
        if man["world"] == world:
            out[name] = load_table(os.path.join(directory, files[rank]), device)
        else:  # re-shard: every rank loads all shards; caller regroups with its partitioner
            merged = None
            for fn in files:
                t = load_table(os.path.join(directory, fn), device)
                if merged is None:
                    merged = Table(t.table_id, t.combiner)
                for p in t.get_partitions():
                    merged.add_partition(p)
            out[name] = merged
    return man, out
