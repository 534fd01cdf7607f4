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

``manifest.json``: iteration, world size, per-rank files (replicated tables: one file
written by rank 0), full CPU + GPU RNG state, user extras.

Resume loads a rank's partitions back (onto any device); loading with a different world
size returns all partitions of the listed files (first copy of an id wins, sorted by
id), from which the caller keeps the ids its partitioner assigns to it.
:class:`Checkpointer` adds the periodic ``it-<n>/`` + atomic ``LATEST`` protocol every
iterative app uses.
"""
from __future__ import annotations

import base64
import json
import os
import struct
import zlib
from typing import Dict, List, Optional, Sequence

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


def _rng_state() -> dict:
    st = {"torch": base64.b64encode(torch.random.get_rng_state().numpy().tobytes()).decode()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = [base64.b64encode(t.numpy().tobytes()).decode() for t in torch.cuda.get_rng_state_all()]
    return st


def restore_rng(man: dict) -> None:
    """Restore the CPU (and, when recorded and visible, per-device GPU) RNG state saved
    in a manifest, so a resumed randomized app continues the uninterrupted stream."""
    st = man.get("rng") or {}
    if isinstance(st.get("torch"), str):
        torch.random.set_rng_state(torch.frombuffer(bytearray(base64.b64decode(st["torch"])), dtype=torch.uint8))
    if st.get("cuda") and torch.cuda.is_available():
        states = [torch.frombuffer(bytearray(base64.b64decode(x)), dtype=torch.uint8) for x in st["cuda"]]
        if len(states) == torch.cuda.device_count():
            torch.cuda.set_rng_state_all(states)


def save_checkpoint(directory: str, tables: Dict[str, Table], rank: int, world: int, iteration: int,
                    extra: Optional[dict] = None, comm=None, replicated: Sequence[str] = ()) -> str:
    """Every rank writes its tables; rank 0 writes the manifest (after a barrier when a
    communicator is given, so the manifest only appears once all shards exist).

    Tables named in ``replicated`` hold the same partitions on every rank (e.g. the
    K-means centroids after an allreduce): only rank 0 writes them, and any world size
    loads that single file back unchanged."""
    os.makedirs(directory, exist_ok=True)
    rep = set(replicated)
    for name, t in tables.items():
        if name in rep and rank != 0:
            continue
        save_table(t, os.path.join(directory, f"table-{name}-r{rank}.hpt"), rank, world)
    if comm is not None:
        comm.barrier()
    if rank == 0:
        man = {"version": VERSION, "iteration": iteration, "world": world,
               "tables": {n: ([f"table-{n}-r0.hpt"] if n in rep else [f"table-{n}-r{r}.hpt" for r in range(world)])
                          for n in tables},
               "replicated": sorted(rep & set(tables)), "rng": _rng_state(), "extra": extra or {}}
        tmp = os.path.join(directory, "manifest.json.tmp")
        with open(tmp, "w") as f:
            json.dump(man, f)
        os.replace(tmp, os.path.join(directory, "manifest.json"))
    return directory


def load_checkpoint(directory: str, rank: int, world: int, device="cpu", rng: bool = False) -> tuple:
    """Load this rank's view of a checkpoint: its own shard when the world size matches;
    otherwise every shard, merged by partition id with the FIRST copy of a duplicated id
    kept (a checkpoint never holds two different values of one id, so nothing may be
    combined — combining would multiply replicated partitions), partitions sorted by id;
    the caller keeps the ids it owns under its partitioner. ``rng`` restores the saved RNG
    state."""
    with open(os.path.join(directory, "manifest.json")) as f:
        man = json.load(f)
    rep = set(man.get("replicated", []))
    out = {}
    for name, files in man["tables"].items():
        if name in rep:
            out[name] = load_table(os.path.join(directory, files[0]), device)
        elif man["world"] == world:
            out[name] = load_table(os.path.join(directory, files[rank]), device)
        else:  # re-shard: every rank loads all shards
            parts: Dict[int, Partition] = {}
            first = None
            for fn in files:
                t = load_table(os.path.join(directory, fn), device)
                first = first or t
                for p in t.get_partitions():
                    parts.setdefault(p.id(), p)
            ids = sorted(parts)
            if isinstance(first, PackedTable) and ids:
                out[name] = PackedTable(ids, torch.stack([parts[i].get() for i in ids]), table_id=first.table_id,
                                        combiner=first.combiner)
            else:
                merged = Table(first.table_id if first is not None else 0, first.combiner if first is not None else None)
                for i in ids:
                    merged.insert_partition(parts[i])
                out[name] = merged
    if rng:
        restore_rng(man)
    return man, out


class Checkpointer:
    """Periodic application checkpoints: ``<dir>/it-<iter>/`` (per-rank ``.hpt`` files +
    manifest) and a ``<dir>/LATEST`` pointer that rank 0 replaces atomically once every
    rank's shard is on disk, so a restart never sees a half-written step."""

    def __init__(self, directory: str, comm, every: int = 0):
        self.directory = directory
        self.comm = comm
        self.every = int(every or 0)

    @property
    def enabled(self) -> bool:
        return bool(self.directory)

    def due(self, it: int) -> bool:
        return self.enabled and self.every > 0 and (it + 1) % self.every == 0

    def save(self, it: int, tables: Dict[str, Table], extra: Optional[dict] = None,
             replicated: Sequence[str] = ()) -> str:
        sub = os.path.join(self.directory, f"it-{it:06d}")
        save_checkpoint(sub, tables, self.comm.rank, self.comm.world_size, it, extra=extra, comm=self.comm,
                        replicated=replicated)
        if self.comm.rank == 0:
            tmp = os.path.join(self.directory, "LATEST.tmp")
            with open(tmp, "w") as f:
                json.dump({"dir": os.path.basename(sub), "iteration": it}, f)
            os.replace(tmp, os.path.join(self.directory, "LATEST"))
        self.comm.barrier()  # no rank runs ahead of a LATEST that may still point back
        return sub

    def load_latest(self, device="cpu", rng: bool = False):
        """``(manifest, tables)`` of the newest complete checkpoint, or None."""
        if not self.enabled:
            return None
        latest = os.path.join(self.directory, "LATEST")
        if not os.path.exists(latest):
            return None
        with open(latest) as f:
            sub = os.path.join(self.directory, json.load(f)["dir"])
        return load_checkpoint(sub, self.comm.rank, self.comm.world_size, device=device, rng=rng)


def tensor_table(t: torch.Tensor, ids=None, table_id: int = 0) -> PackedTable:
    """Wrap a tensor as a packed table (row i = partition ``ids[i]``, default 0..n-1)."""
    if t.dim() == 0:
        t = t.reshape(1)
    ids = list(range(t.shape[0])) if ids is None else [int(i) for i in (ids.tolist() if torch.is_tensor(ids) else ids)]
    return PackedTable(ids, t, table_id=table_id, combiner=ArrCombiner(Operation.SUM))


def blob_table(t: torch.Tensor, table_id: int = 0) -> Table:
    """A whole tensor as ONE partition (id 0) — for per-rank state such as token topics."""
    tab = Table(table_id, ArrCombiner(Operation.SUM))
    tab.add(0, t)
    return tab
