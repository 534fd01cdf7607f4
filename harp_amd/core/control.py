"""Control writables (Harp ``util`` package): Ack, Barrier(status), PartitionCount,
PartitionSet, Join (util/Ack.java, Barrier.java:32-85, PartitionCount.java:33-106,
PartitionSet.java:35-133, Join.java:46-193). The collectives exchange this metadata as
device tensors; these classes keep the reference's message vocabulary available for
user protocols (events, custom exchanges) and for the Harp wire format."""
from __future__ import annotations

from typing import Dict, List

from .writable import DataInput, DataOutput, Writable


class Ack(Writable):
    def write(self, out: DataOutput) -> None:
        pass

    def read(self, inp: DataInput) -> None:
        pass


class Barrier(Writable):
    def __init__(self, status: bool = True):
        self.status = status

    def write(self, out: DataOutput) -> None:
        out.write_boolean(self.status)

    def read(self, inp: DataInput) -> None:
        self.status = inp.read_boolean()


class PartitionCount(Writable):
    def __init__(self, worker_id: int = 0, count: int = 0):
        self.worker_id, self.count = worker_id, count

    def write(self, out: DataOutput) -> None:
        out.write_int(self.worker_id)
        out.write_int(self.count)

    def read(self, inp: DataInput) -> None:
        self.worker_id = inp.read_int()
        self.count = inp.read_int()


class PartitionSet(Writable):
    def __init__(self, worker_id: int = 0, par_set: List[int] | None = None):
        self.worker_id = worker_id
        self.par_set = list(par_set or [])

    def write(self, out: DataOutput) -> None:
        out.write_int(self.worker_id)
        out.write_int(len(self.par_set))
        for p in self.par_set:
            out.write_int(p)

    def read(self, inp: DataInput) -> None:
        self.worker_id = inp.read_int()
        self.par_set = [inp.read_int() for _ in range(inp.read_int())]


class Join(Writable):
    def __init__(self, par_to_worker: Dict[int, List[int]] | None = None, worker_par_count: Dict[int, int] | None = None):
        self.par_to_worker_map = dict(par_to_worker or {})
        self.worker_par_count_map = dict(worker_par_count or {})

    def write(self, out: DataOutput) -> None:
        out.write_int(len(self.par_to_worker_map))
        for p, ws in self.par_to_worker_map.items():
            out.write_int(p)
            out.write_int(len(ws))
            for w in ws:
                out.write_int(w)
        out.write_int(len(self.worker_par_count_map))
        for w, c in self.worker_par_count_map.items():
            out.write_int(w)
            out.write_int(c)

    def read(self, inp: DataInput) -> None:
        self.par_to_worker_map = {}
        for _ in range(inp.read_int()):
            p = inp.read_int()
            self.par_to_worker_map[p] = [inp.read_int() for _ in range(inp.read_int())]
        self.worker_par_count_map = {}
        for _ in range(inp.read_int()):
            w = inp.read_int()
            self.worker_par_count_map[w] = inp.read_int()
