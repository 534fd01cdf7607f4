"""Communicator and worker topology.

Reference: the custom Java TCP transport (io/*, client/*, server/*: thread-per-connection
server, pooled sockets, big-endian serialization) plus ``Workers``
(worker/Workers.java:121-157: master = 0, min = 0, max = P-1, middle = max/2,
next = (self+1) mod P) and the bootstrap barrier ``start-worker``/``handshake``
(mapred/CollectiveMapper.java:253-310).

MI355X design: one process per GPU, ``torch.distributed`` process groups — backend
``nccl`` (= RCCL over xGMI) for device tensors, ``gloo`` on CPU-only hosts (the
reference's "2 workers on one host" test mode). Collectives move device
buffers straight to RCCL: there is no serialization, no socket pool and no receiver
thread. ``channel()`` creates an additional communicator over the same ranks with its
own RCCL stream, which is how concurrent collective streams (the reference's per-slice
rotation threads, MJ/dymoro/Rotator.java:43-50) keep a per-communicator issue order.
"""
from __future__ import annotations

import datetime
import os
import threading
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

# Reference timeouts (io/Constant.java:35-36): DATA_MAX_WAIT_TIME = 1800 s.
DATA_MAX_WAIT_TIME_S = float(os.environ.get("HARP_DATA_MAX_WAIT_TIME", "1800"))


def collective_timeout_s() -> float:
    """Collective watchdog: a collective that has not completed after this many seconds
    fails on every live rank (torch.distributed process-group timeout), the collective
    returns False and the job can restart from its last checkpoint. Read at call time from
    ``HARP_DATA_MAX_WAIT_TIME`` (default 1800 s, the reference's DATA_MAX_WAIT_TIME)."""
    return float(os.environ.get("HARP_DATA_MAX_WAIT_TIME", str(DATA_MAX_WAIT_TIME_S)))


class Workers:
    """Topology view (worker/Workers.java)."""

    def __init__(self, self_id: int, num_workers: int):
        self.self_id = int(self_id)
        self.num_workers = int(num_workers)

    master_id = 0
    min_id = 0

    @property
    def max_id(self) -> int:
        return self.num_workers - 1

    @property
    def middle_id(self) -> int:
        return self.max_id // 2

    @property
    def next_id(self) -> int:
        return (self.self_id + 1) % self.num_workers

    @property
    def prev_id(self) -> int:
        return (self.self_id - 1) % self.num_workers

    def is_master(self) -> bool:
        return self.self_id == self.master_id

    def is_the_only_worker(self) -> bool:
        return self.num_workers == 1

    def is_max(self) -> bool:
        return self.self_id == self.max_id

    def get_self_id(self) -> int:
        return self.self_id

    def get_num_workers(self) -> int:
        return self.num_workers

    def get_next_id(self) -> int:
        return self.next_id

    def get_master_id(self) -> int:
        return self.master_id

    def get_min_id(self) -> int:
        return self.min_id

    def get_max_id(self) -> int:
        return self.max_id

    def get_middle_id(self) -> int:
        return self.middle_id

    def __repr__(self) -> str:
        return f"Workers(self={self.self_id}, n={self.num_workers})"


def parse_nodes_file(text: str) -> List[List[str]]:
    """Harp nodes file: ``#<rack>`` lines start a rack, other lines are hostnames
    (worker/Nodes.java:89-118). Returns hosts grouped by rack in file order; worker
    ids are assigned sequentially across racks (Workers.java:130-144)."""
    racks: List[List[str]] = []
    cur: Optional[List[str]] = None
    for raw in text.splitlines():
        line = raw.strip()
        if not line:
            continue
        if line.startswith("#"):
            cur = []
            racks.append(cur)
        else:
            if cur is None:
                cur = []
                racks.append(cur)
            cur.append(line)
    return racks


# dtypes RCCL has no wire type for (ShortArray tables, reference ShortArray): data movement
# sends their bits as a same-width type; reductions run on an int32 / int64 copy
_NCCL_BITS = {torch.int16: torch.float16}
for _n, _w in (("uint16", torch.float16), ("uint32", torch.int32), ("uint64", torch.int64)):
    if hasattr(torch, _n):
        _NCCL_BITS[getattr(torch, _n)] = _w
_NCCL_WIDE = {torch.int16: torch.int32}


def nccl_wire(t: torch.Tensor) -> torch.Tensor:
    """``t`` itself, or a same-width view RCCL can move (bit-exact: no arithmetic)."""
    w = _NCCL_BITS.get(t.dtype)
    return t if w is None else t.view(w)


class Communicator:
    """A torch.distributed group plus the device its buffers live on."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None, device: torch.device | str | None = None,
                 name: str = "main"):
        self.group = group
        self.name = name
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world_size = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank, self.world_size, self.backend = 0, 1, "none"
        if device is None:
            if self.backend == "nccl" or (self.backend == "none" and torch.cuda.is_available()):
                device = torch.device("cuda", torch.cuda.current_device())
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        self.workers = Workers(self.rank, self.world_size)
        # gloo moves only host tensors for point-to-point / all-to-all: when gloo ranks keep
        # their buffers on a GPU (the multi-rank rehearsal on a one-GPU box, where RCCL
        # refuses two ranks per device), those ops stage through host memory
        self.stage = self.backend == "gloo" and self.device.type == "cuda" and self.world_size > 1
        # the reverse: RCCL moves only device tensors, so a host tensor handed to a primitive
        # under nccl runs on a device copy (a path the gloo tests would not catch)
        self.dev_stage = self.backend == "nccl" and self.world_size > 1
        self._channels: dict = {}
        self._lock = threading.Lock()
        # Optional fault injection hook (tests): called before every collective with the
        # op name; may raise or sleep to emulate a dropped/slow rank.
        self.fault_hook = None

    # -- identity -----------------------------------------------------------------
    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    def global_rank(self, group_rank: int) -> int:
        if self.group is None or not dist.is_initialized():
            return group_rank
        return dist.get_global_rank(self.group, group_rank)

    def channel(self, key: str) -> "Communicator":
        """Another communicator over the same ranks (own RCCL communicator/stream).

        Must be called collectively, in the same order, on every rank (torch's
        ``new_group`` contract)."""
        with self._lock:
            ch = self._channels.get(key)
            if ch is None:
                if self.world_size > 1:
                    ranks = [self.global_rank(r) for r in range(self.world_size)]
                    g = dist.new_group(ranks=ranks, backend=self.backend,
                                       timeout=datetime.timedelta(seconds=collective_timeout_s()))
                else:
                    g = None
                ch = Communicator(g, self.device, name=f"{self.name}/{key}")
                self._channels[key] = ch
            return ch

    def _hook(self, op: str) -> None:
        if self.fault_hook is not None:
            self.fault_hook(op)

    # -- primitives -------------------------------------------------------------------
    def barrier(self) -> None:
        self._hook("barrier")
        if self.world_size > 1:
            if self.backend == "nccl":
                t = torch.ones(1, device=self.device)
                dist.all_reduce(t, group=self.group)
            else:
                dist.barrier(group=self.group)

    def _host(self, t: torch.Tensor, fn) -> None:
        """Run a collective on a host copy of ``t`` and copy the result back (staging)."""
        h = t.detach().cpu().contiguous()
        fn(h)
        t.copy_(h)

    def _on_host(self, *ts: torch.Tensor) -> bool:
        """nccl with a host tensor among ``ts``: the op must run on device copies."""
        return self.dev_stage and any(t.device.type == "cpu" for t in ts)

    def _dev(self, t: torch.Tensor, fn) -> None:
        """Run a collective on a device copy of host tensor ``t``, copying the result back."""
        d = t.detach().to(self.device).contiguous()
        fn(d)
        t.copy_(d.cpu())

    def _wire(self, t: torch.Tensor) -> torch.Tensor:
        return nccl_wire(t) if self.dev_stage else t

    def _widened(self, t: torch.Tensor, fn) -> None:
        """A reduction of a dtype RCCL cannot reduce (int16) on a widened copy."""
        w = t.to(_NCCL_WIDE[t.dtype])
        fn(w)
        t.copy_(w)

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM, async_op: bool = False):
        self._hook("all_reduce")
        if self.world_size > 1:
            if self.stage and t.device.type != "cpu":
                return self._host(t, lambda h: dist.all_reduce(h, op=op, group=self.group))
            if self._on_host(t):
                return self._dev(t, lambda d: dist.all_reduce(d, op=op, group=self.group))
            if self.dev_stage and t.dtype in _NCCL_WIDE:
                return self._widened(t, lambda w: dist.all_reduce(w, op=op, group=self.group))
            return dist.all_reduce(t, op=op, group=self.group, async_op=async_op)
        return None

    def broadcast(self, t: torch.Tensor, root: int, async_op: bool = False):
        self._hook("broadcast")
        if self.world_size > 1:
            if self.stage and t.device.type != "cpu":
                return self._host(t, lambda h: dist.broadcast(h, src=self.global_rank(root), group=self.group))
            if self._on_host(t):
                return self._dev(t, lambda d: dist.broadcast(d, src=self.global_rank(root), group=self.group))
            return dist.broadcast(self._wire(t), src=self.global_rank(root), group=self.group, async_op=async_op)
        return None

    def reduce(self, t: torch.Tensor, root: int, op=dist.ReduceOp.SUM):
        self._hook("reduce")
        if self.world_size > 1:
            if self.stage and t.device.type != "cpu":
                return self._host(t, lambda h: dist.reduce(h, dst=self.global_rank(root), op=op, group=self.group))
            if self._on_host(t):
                return self._dev(t, lambda d: dist.reduce(d, dst=self.global_rank(root), op=op, group=self.group))
            if self.dev_stage and t.dtype in _NCCL_WIDE:
                return self._widened(t, lambda w: dist.reduce(w, dst=self.global_rank(root), op=op, group=self.group))
            dist.reduce(t, dst=self.global_rank(root), op=op, group=self.group)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        self._hook("all_gather")
        if self.world_size > 1:
            if self.stage and out.device.type != "cpu":
                ho = torch.empty(out.shape, dtype=out.dtype)
                dist.all_gather_into_tensor(ho, inp.cpu(), group=self.group)
                out.copy_(ho)
                return None
            if self._on_host(out, inp):
                do = torch.empty(out.shape, dtype=out.dtype, device=self.device)
                dist.all_gather_into_tensor(do, inp.to(self.device), group=self.group)
                out.copy_(do)
                return None
            return dist.all_gather_into_tensor(self._wire(out), self._wire(inp), group=self.group, async_op=async_op)
        out.copy_(inp.reshape(out.shape))
        return None

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op=dist.ReduceOp.SUM,
                       async_op: bool = False):
        self._hook("reduce_scatter")
        if self.world_size > 1:
            if self.stage and out.device.type != "cpu":
                ho = torch.empty(out.shape, dtype=out.dtype)
                dist.reduce_scatter_tensor(ho, inp.cpu(), op=op, group=self.group)
                out.copy_(ho)
                return None
            if self._on_host(out, inp):
                do = torch.empty(out.shape, dtype=out.dtype, device=self.device)
                dist.reduce_scatter_tensor(do, inp.to(self.device), op=op, group=self.group)
                out.copy_(do)
                return None
            if self.dev_stage and out.dtype in _NCCL_WIDE:
                w = torch.empty(out.shape, dtype=_NCCL_WIDE[out.dtype], device=out.device)
                dist.reduce_scatter_tensor(w, inp.to(w.dtype), op=op, group=self.group)
                out.copy_(w)
                return None
            return dist.reduce_scatter_tensor(out, inp, op=op, group=self.group, async_op=async_op)
        out.copy_(inp.reshape(out.shape))
        return None

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor,
                          out_splits: Sequence[int] | None = None, in_splits: Sequence[int] | None = None):
        self._hook("all_to_all")
        if self.world_size > 1:
            if self.stage and out.device.type != "cpu":
                ho = torch.empty(out.shape, dtype=out.dtype)
                dist.all_to_all_single(ho, inp.cpu(), out_splits, in_splits, group=self.group)
                out.copy_(ho)
                return
            if self._on_host(out, inp):
                do = torch.empty(out.shape, dtype=out.dtype, device=self.device)
                dist.all_to_all_single(do, inp.to(self.device), out_splits, in_splits, group=self.group)
                out.copy_(do)
                return
            dist.all_to_all_single(self._wire(out), self._wire(inp), out_splits, in_splits, group=self.group)
        else:
            out.copy_(inp)

    def sendrecv(self, sends: dict, recvs: dict, async_op: bool = False):
        """Grouped point-to-point: ``sends`` maps dest -> tensor, ``recvs`` src -> tensor."""
        self._hook("sendrecv")
        if self.stage:
            return self._staged_p2p({d: [t] for d, t in sends.items()}, {s: [t] for s, t in recvs.items()})
        if self._on_host(*sends.values(), *recvs.values()):
            return self._device_p2p({d: [t] for d, t in sends.items()}, {s: [t] for s, t in recvs.items()})
        ops = []
        for dst, t in sends.items():
            ops.append(dist.P2POp(dist.isend, self._wire(t), self.global_rank(dst), self.group))
        for src, t in recvs.items():
            ops.append(dist.P2POp(dist.irecv, self._wire(t), self.global_rank(src), self.group))
        if not ops:
            return []
        works = dist.batch_isend_irecv(ops)
        if async_op:
            return works
        for w in works:
            w.wait()
        return []

    def _staged_p2p(self, sends: dict, recvs: dict):
        """Host-staged grouped send/recv (gloo ranks with device buffers); completes before
        returning (no works to wait on)."""
        ops, host_recv = [], []
        for dst, ts in sends.items():
            for t in ts:
                ops.append(dist.P2POp(dist.isend, t.detach().cpu().contiguous(), self.global_rank(dst), self.group))
        for src, ts in recvs.items():
            for t in ts:
                h = torch.empty(t.shape, dtype=t.dtype)
                host_recv.append((t, h))
                ops.append(dist.P2POp(dist.irecv, h, self.global_rank(src), self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        for t, h in host_recv:
            t.copy_(h)
        return []

    def _device_p2p(self, sends: dict, recvs: dict):
        """Grouped send/recv of host tensors under nccl through device copies; completes
        before returning."""
        ops, dev_recv = [], []
        for dst, ts in sends.items():
            for t in ts:
                ops.append(dist.P2POp(dist.isend, t.detach().to(self.device).contiguous(), self.global_rank(dst),
                                      self.group))
        for src, ts in recvs.items():
            for t in ts:
                d = torch.empty(t.shape, dtype=t.dtype, device=self.device)
                dev_recv.append((t, d))
                ops.append(dist.P2POp(dist.irecv, d, self.global_rank(src), self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        for t, d in dev_recv:
            t.copy_(d)
        return []

    def sendrecv_multi(self, sends: dict, recvs: dict, async_op: bool = False):
        """Like :meth:`sendrecv` with a LIST of tensors per peer, all in one grouped call
        (per peer, the tensors are matched in list order)."""
        self._hook("sendrecv")
        if self.stage:
            return self._staged_p2p(sends, recvs)
        if self._on_host(*(t for ts in sends.values() for t in ts), *(t for ts in recvs.values() for t in ts)):
            return self._device_p2p(sends, recvs)
        ops = []
        for dst, ts in sends.items():
            for t in ts:
                ops.append(dist.P2POp(dist.isend, self._wire(t), self.global_rank(dst), self.group))
        for src, ts in recvs.items():
            for t in ts:
                ops.append(dist.P2POp(dist.irecv, self._wire(t), self.global_rank(src), self.group))
        if not ops:
            return []
        works = dist.batch_isend_irecv(ops)
        if async_op:
            return works
        for w in works:
            w.wait()
        return []

    # -- helpers built on the primitives ----------------------------------------------
    def all_gather_ints(self, values: Sequence[int]) -> torch.Tensor:
        """All-gather a small int64 vector; returns a CPU tensor [P, len(values)]."""
        v = torch.tensor(list(values), dtype=torch.int64, device=self.device)
        if self.world_size == 1:
            return v.cpu().reshape(1, -1)
        out = torch.empty(self.world_size * v.numel(), dtype=torch.int64, device=self.device)
        self.all_gather_into(out, v)
        return out.cpu().reshape(self.world_size, -1)

    def all_gather_bytes(self, msg: torch.Tensor) -> List[torch.Tensor]:
        """Variable-size uint8 all-gather: size exchange, then one padded all-gather."""
        if self.world_size == 1:
            return [msg]
        sizes = self.all_gather_ints([msg.numel()])[:, 0].tolist()
        mx = max(max(sizes), 1)
        buf = torch.zeros(mx, dtype=torch.uint8, device=self.device)
        buf[: msg.numel()] = msg
        out = torch.empty(mx * self.world_size, dtype=torch.uint8, device=self.device)
        self.all_gather_into(out, buf)
        return [out[r * mx: r * mx + sizes[r]] for r in range(self.world_size)]

    def all_to_all_bytes(self, msgs: List[torch.Tensor]) -> List[torch.Tensor]:
        """Variable-size uint8 all-to-all (alltoallv): msgs[r] goes to rank r."""
        P = self.world_size
        if P == 1:
            return [msgs[0]]
        send_sizes = torch.tensor([m.numel() for m in msgs], dtype=torch.int64, device=self.device)
        recv_sizes = torch.empty(P, dtype=torch.int64, device=self.device)
        self.all_to_all_single(recv_sizes, send_sizes)
        rs = recv_sizes.cpu().tolist()
        ss = [m.numel() for m in msgs]
        send = torch.cat(msgs) if sum(ss) else torch.empty(0, dtype=torch.uint8, device=self.device)
        recv = torch.empty(sum(rs), dtype=torch.uint8, device=self.device)
        if sum(ss) or sum(rs):
            self.all_to_all_single(recv, send, rs, ss)
        out, o = [], 0
        for n in rs:
            out.append(recv[o:o + n])
            o += n
        return out

    def broadcast_bytes(self, msg: Optional[torch.Tensor], root: int) -> torch.Tensor:
        if self.world_size == 1:
            return msg
        n = torch.tensor([msg.numel() if self.rank == root else 0], dtype=torch.int64, device=self.device)
        self.broadcast(n, root)
        size = int(n.item())
        buf = msg if self.rank == root else torch.empty(size, dtype=torch.uint8, device=self.device)
        if size:
            self.broadcast(buf, root)
        return buf

    def gather_bytes(self, msg: torch.Tensor, root: int) -> Optional[List[torch.Tensor]]:
        """Variable-size gather to ``root`` via grouped p2p (no padding)."""
        P = self.world_size
        if P == 1:
            return [msg]
        sizes = self.all_gather_ints([msg.numel()])[:, 0].tolist()
        if self.rank == root:
            bufs = {r: torch.empty(sizes[r], dtype=torch.uint8, device=self.device)
                    for r in range(P) if r != root and sizes[r] > 0}
            self.sendrecv({}, bufs)
            return [msg if r == root else bufs.get(r, torch.empty(0, dtype=torch.uint8, device=self.device))
                    for r in range(P)]
        if msg.numel():
            self.sendrecv({root: msg}, {})
        return None

    def __repr__(self) -> str:
        return f"Communicator({self.name}, rank={self.rank}/{self.world_size}, {self.backend}, {self.device})"
