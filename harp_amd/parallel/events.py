"""Asynchronous events outside the collective lockstep (Harp computation models A/D).

Reference: ``Event(type, ctx, sourceID, targetID, body)`` with types MESSAGE /
COLLECTIVE / LOCAL (client/Event.java:37-98, EventType.java:25-27); ``sendEvent``,
``getEvent`` (non-blocking) and ``waitEvent`` (blocking) on the mapper
(mapred/CollectiveMapper.java:623-663); delivery through per-(dest, ctx) batching queues
and an MST broadcast for collective events (client/SyncClient.java:95-200); the
receiver's ``EventQueue`` (io/EventQueue.java:28-74). Delivery is asynchronous with no
ordering guarantee across contexts.

MI355X design: small control messages ride the rendezvous key-value store that
``torch.distributed`` already runs (TCPStore on rank 0), not the RCCL data path — each
rank owns a mailbox ``harp/ev/<rank>`` with an atomically incremented sequence counter;
senders ``add`` to the counter and ``set`` the payload key, receivers consume in sequence
order. Device payloads are copied to host for transport (events are control-plane).
"""
from __future__ import annotations

import enum
import queue
import struct
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Optional

import torch
import torch.distributed as dist

from ..core.partition import Partition
from .codec import decode_partitions, encode_partitions


class EventType(enum.Enum):
    MESSAGE = 0
    COLLECTIVE = 1
    LOCAL = 2


@dataclass
class Event:
    event_type: EventType
    context_name: str
    source_id: int
    target_id: int
    body: Any = None

    # Harp-style accessors
    def get_event_type(self):
        return self.event_type

    def get_context_name(self):
        return self.context_name

    def get_source_id(self):
        return self.source_id

    def get_target_id(self):
        return self.target_id

    def get_body(self):
        return self.body


class EventQueue:
    """Thread-safe blocking queue of events (io/EventQueue.java)."""

    def __init__(self):
        self._q: "queue.Queue[Event]" = queue.Queue()

    def add_event(self, ev: Event) -> None:
        self._q.put(ev)

    def get_event(self) -> Optional[Event]:
        try:
            return self._q.get_nowait()
        except queue.Empty:
            return None

    def wait_event(self, timeout: Optional[float] = None) -> Optional[Event]:
        try:
            return self._q.get(timeout=timeout)
        except queue.Empty:
            return None

    def size(self) -> int:
        return self._q.qsize()


def _encode_event(ev: Event) -> bytes:
    body = ev.body
    if body is None:
        meta, payload = b"", b""
    else:
        meta, pt = encode_partitions([Partition(0, body)], torch.device("cpu"))
        payload = pt.numpy().tobytes()
    ctx = ev.context_name.encode("utf-8")
    head = struct.pack("<iiiHII", ev.event_type.value, ev.source_id, ev.target_id, len(ctx), len(meta), len(payload))
    return head + ctx + meta + payload


def _decode_event(b: bytes) -> Event:
    et, src, tgt, lc, lm, lp = struct.unpack_from("<iiiHII", b, 0)
    pos = struct.calcsize("<iiiHII")
    ctx = b[pos:pos + lc].decode("utf-8")
    pos += lc
    body = None
    if lm:
        meta = b[pos:pos + lm]
        pos += lm
        payload = torch.frombuffer(bytearray(b[pos:pos + lp]), dtype=torch.uint8) if lp else torch.empty(0, dtype=torch.uint8)
        body = decode_partitions(meta, payload, torch.device("cpu"))[0].get()
    return Event(EventType(et), ctx, src, tgt, body)


class EventChannel:
    """Per-rank event endpoint over the distributed store."""

    PREFIX = "harp/ev"

    def __init__(self, rank: int, world_size: int, store=None):
        self.rank = rank
        self.world_size = world_size
        if store is None and dist.is_available() and dist.is_initialized():
            try:
                store = dist.distributed_c10d._get_default_store()
            except Exception:
                store = None
        self.store = store
        self.queue = EventQueue()
        self._consumed = 0
        self._lock = threading.Lock()

    def _counter_key(self, r: int) -> str:
        return f"{self.PREFIX}/{r}/n"

    def _post(self, target: int, data: bytes) -> None:
        seq = self.store.add(self._counter_key(target), 1)
        self.store.set(f"{self.PREFIX}/{target}/{seq}", data)

    def send_event(self, ev: Event) -> bool:
        if ev.event_type is EventType.LOCAL or self.store is None and ev.target_id == self.rank:
            self.queue.add_event(ev)
            return True
        if self.store is None:
            return False
        data = _encode_event(ev)
        if ev.event_type is EventType.MESSAGE:
            if not (0 <= ev.target_id < self.world_size):
                return False
            if ev.target_id == self.rank:
                self.queue.add_event(_decode_event(data))
            else:
                self._post(ev.target_id, data)
            return True
        for r in range(self.world_size):  # COLLECTIVE: every other worker
            if r != self.rank:
                self._post(r, data)
        return True

    def _poll(self) -> None:
        if self.store is None:
            return
        with self._lock:
            n = self.store.add(self._counter_key(self.rank), 0)
            while self._consumed < n:
                self._consumed += 1
                key = f"{self.PREFIX}/{self.rank}/{self._consumed}"
                data = self.store.get(key)
                try:
                    self.store.delete_key(key)
                except Exception:
                    pass
                self.queue.add_event(_decode_event(data))

    def get_event(self) -> Optional[Event]:
        ev = self.queue.get_event()
        if ev is None:
            self._poll()
            ev = self.queue.get_event()
        return ev

    def wait_event(self, timeout: Optional[float] = None, poll_interval: float = 0.002) -> Optional[Event]:
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            ev = self.get_event()
            if ev is not None:
                return ev
            if deadline is not None and time.monotonic() > deadline:
                return None
            time.sleep(poll_interval)
