"""Metrics / tracing.

The reference logs ad-hoc wall-clock deltas (K-means ``Compute/Merge/Aggregate`` per
iteration at KMeansCollectiveMapper.java:191-193, SGD ``computeTime/waitTime`` at
SGDCollectiveMapper.java:294-298, rotation comm time at RotateTask.java:109-123,
regroup-vs-allgather time at RegroupCollective.java:274-295) plus JVM memory/GC logs
(CollectiveMapper.java:686-714).

Here:
  * per-phase timers backed by HIP events on the GPU (no host sync inside the timed
    region; resolved lazily);
  * per-collective records (kind, ctx, op, bytes moved, stream time from HIP events on
    the calling stream — the stream waits on RCCL's stream, so the event pair brackets
    the collective's device time — plus host time);
  * the xGMI link model: ideal time per collective kind over one ~153 GB/s link per
    direction (ring algorithms are per-link bound on a point-to-point mesh), so every
    record carries achieved GB/s and the ratio to that ideal;
  * per-iteration JSONL records (``Metrics.begin_iteration`` / ``end_iteration``):
    phase ms, collective ms / bytes / GB/s / efficiency, HBM use from ``hipMemGetInfo``;
  * optional roctx ranges so rocprofv3 traces show the same phase names.
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch


def _roctx():
    try:
        return torch.cuda.nvtx if torch.cuda.is_available() else None  # maps to roctx on ROCm
    except Exception:  # pragma: no cover
        return None


# pending HIP event pairs kept before the completed ones are folded in (without a device
# sync); past PENDING_HARD_CAP the rest are resolved with one sync. Long runs that never
# flush (no metrics path set) therefore hold a bounded number of events.
PENDING_SWEEP = 1024
PENDING_HARD_CAP = 8192


def _sweep_pending(pending: List[tuple], fold) -> None:
    """Fold every event pair whose end event has completed (``fold(item, seconds)``);
    keep the rest, in order. Synchronises only when the list is still over the hard cap."""
    if len(pending) < PENDING_SWEEP:
        return
    keep = []
    for item in pending:
        s, e = item[-2], item[-1]
        if e.query():
            fold(item, s.elapsed_time(e) / 1e3)
        else:
            keep.append(item)
    if len(keep) >= PENDING_HARD_CAP:
        torch.cuda.synchronize()
        for item in keep:
            fold(item, item[-2].elapsed_time(item[-1]) / 1e3)
        keep = []
    pending[:] = keep


class PhaseTimer:
    """Accumulates named phase times. On GPU uses hipEvents recorded on the current
    stream, resolved at :meth:`flush` (completed pairs are folded in as the list grows);
    on CPU uses perf_counter."""

    def __init__(self, use_events: Optional[bool] = None, annotate: bool = False):
        self.use_events = torch.cuda.is_available() if use_events is None else use_events
        self.annotate = annotate
        self._pending: List[tuple] = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        nvtx = _roctx() if self.annotate else None
        if nvtx is not None:
            nvtx.range_push(name)
        if self.use_events:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._pending.append((name, s, e))
                _sweep_pending(self._pending, self._fold)
                if nvtx is not None:
                    nvtx.range_pop()
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.totals[name] += time.perf_counter() - t0
                self.counts[name] += 1
                if nvtx is not None:
                    nvtx.range_pop()

    def _fold(self, item: tuple, seconds: float) -> None:
        self.totals[item[0]] += seconds
        self.counts[item[0]] += 1

    def flush(self) -> Dict[str, float]:
        if self._pending:
            torch.cuda.synchronize()
            for item in self._pending:
                self._fold(item, item[1].elapsed_time(item[2]) / 1e3)
            self._pending.clear()
        return dict(self.totals)

    def reset(self) -> None:
        self._pending.clear()
        self.totals.clear()
        self.counts.clear()


# dense bf16 MFMA peak of one MI355X at the 2.4 GHz boost clock (no sparsity); sustained
# clocks under MFMA load are lower (1.8-2.0 GHz measured), so ~0.8 is the practical ceiling
MFMA_BF16_PEAK_TFLOPS = 2500.0

# xGMI link model used to report achieved-vs-ideal collective bandwidth:
XGMI_LINK_GBPS = 153.0
XGMI_LINKS = 7


def ring_allreduce_ideal_s(nbytes: int, world: int, link_gbps: float = XGMI_LINK_GBPS) -> float:
    """Ideal single-ring allreduce time (2(P-1)/P * S over one link per direction)."""
    if world <= 1:
        return 0.0
    return 2 * (world - 1) / world * nbytes / (link_gbps * 1e9)


def ideal_collective_s(kind: str, nbytes: int, world: int, link_gbps: float = XGMI_LINK_GBPS) -> float:
    """Per-link-bound ideal time of one collective moving ``nbytes`` (the table's bytes on
    this rank) among ``world`` ranks: ring allreduce 2(P-1)/P*S; reduce-scatter (regroup)
    and allgather (P-1)/P*S of the full buffer; broadcast / reduce / rotate S (pipelined
    chain or one p2p hop); all-to-all-v (push/pull/join) (P-1)/P*S spread over P-1 links."""
    if world <= 1 or nbytes <= 0:
        return 0.0
    bw = link_gbps * 1e9
    P = world
    if kind == "allreduce":
        return ring_allreduce_ideal_s(nbytes, P, link_gbps)
    if kind in ("regroup", "regroup_aggregate", "allgather", "aggregate"):
        return (P - 1) / P * nbytes / bw
    if kind in ("broadcast", "reduce", "rotate"):
        return nbytes / bw
    if kind in ("push", "pull", "join"):
        return (P - 1) / P * nbytes / bw / max(1, min(P - 1, XGMI_LINKS))
    return 0.0


def table_nbytes(table) -> int:
    """Bytes of a table's payload: the packed buffer, or the sum of tensor payloads (plus
    the encoded size of non-tensor partitions) of a generic table."""
    if table is None:
        return 0
    buf = getattr(table, "buffer", None)
    if isinstance(buf, torch.Tensor):
        return buf.numel() * buf.element_size()
    n = 0
    try:
        parts = table.get_partitions()
    except Exception:
        return 0
    for p in parts:
        d = p.get()
        t = d if isinstance(d, torch.Tensor) else getattr(d, "tensor", None)
        if isinstance(t, torch.Tensor):
            n += t.numel() * t.element_size()
        elif hasattr(d, "get_num_write_bytes"):
            try:
                n += int(d.get_num_write_bytes())
            except Exception:
                pass
    return n


class Metrics:
    def __init__(self, rank: int = 0, path: Optional[str] = None, world: int = 1):
        self.rank = rank
        self.world = world
        self.path = path or os.environ.get("HARP_METRICS_JSONL")
        self.phases: Dict[str, float] = defaultdict(float)
        self.collectives: List[dict] = []
        self._pending: List[tuple] = []  # (record, start event, end event)
        self.timer = PhaseTimer()
        self._iter_mark: Optional[tuple] = None

    def record(self, name: str, seconds: float) -> None:
        self.phases[name] += seconds

    # -- collectives -----------------------------------------------------------------------
    def collective(self, kind: str, ctx: str, op: str, seconds: float, nbytes: int = 0,
                   events: Optional[tuple] = None) -> dict:
        """Record one collective. ``seconds`` is host time; with ``events`` (a recorded
        start/end pair on the calling stream) the stream time replaces it when resolved."""
        rec = {"kind": kind, "ctx": ctx, "op": op, "s": seconds, "host_s": seconds, "bytes": int(nbytes)}
        self.collectives.append(rec)
        if events is not None:
            self._pending.append((rec, events[0], events[1]))
            # completed pairs resolve in place, so the list stays bounded without metrics output
            _sweep_pending(self._pending, self._fold)
        if len(self.collectives) > 10000:
            del self.collectives[:5000]
        return rec

    @staticmethod
    def _fold(item: tuple, seconds: float) -> None:
        item[0]["s"] = seconds

    @contextlib.contextmanager
    def time_collective(self, kind: str, ctx: str, op: str, nbytes: int = 0, device: Optional[torch.device] = None):
        """Context manager timing one collective with HIP events on the current stream of
        ``device`` (host time on CPU devices)."""
        use_ev = device is not None and device.type == "cuda"
        if use_ev:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            host = time.perf_counter() - t0
            if use_ev:
                e.record()
                self.collective(kind, ctx, op, host, nbytes, events=(s, e))
            else:
                self.collective(kind, ctx, op, host, nbytes)

    def resolve(self) -> None:
        """Turn pending event pairs into stream times (one device sync)."""
        if self._pending:
            torch.cuda.synchronize()
            for rec, s, e in self._pending:
                rec["s"] = s.elapsed_time(e) / 1e3
            self._pending.clear()

    def memory(self) -> Dict[str, float]:
        if torch.cuda.is_available():
            free, total = torch.cuda.mem_get_info()
            return {
                "hbm_used_gb": (total - free) / 2**30,
                "hbm_total_gb": total / 2**30,
                "torch_alloc_gb": torch.cuda.memory_allocated() / 2**30,
                "torch_peak_gb": torch.cuda.max_memory_allocated() / 2**30,
            }
        try:
            import psutil

            rss = psutil.Process().memory_info().rss
        except Exception:  # pragma: no cover
            rss = 0
        return {"host_rss_gb": rss / 2**30}

    def emit(self, record: dict) -> dict:
        record = {"rank": self.rank, "t": time.time(), **record}
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(record) + "\n")
        return record

    def _annotate(self, c: dict) -> dict:
        ideal = ideal_collective_s(c["kind"], c["bytes"], self.world)
        out = {"kind": c["kind"], "op": c["op"], "ms": round(c["s"] * 1e3, 4), "bytes": c["bytes"]}
        if c["s"] > 0 and c["bytes"]:
            out["gbps"] = round(c["bytes"] / c["s"] / 1e9, 3)
        if ideal > 0:
            out["ideal_ms"] = float(f"{ideal * 1e3:.6g}")
            out["eff_vs_xgmi_model"] = round(ideal / c["s"], 4) if c["s"] > 0 else None
        return out

    # -- per-iteration records ------------------------------------------------------------
    @property
    def enabled(self) -> bool:
        return bool(self.path)

    def begin_iteration(self) -> None:
        if not self.path:
            return
        self.timer.flush()
        self.resolve()
        self._iter_mark = (dict(self.timer.totals), len(self.collectives))

    def end_iteration(self, app: str, it: int, flops: float = 0.0, peak_tflops: float = MFMA_BF16_PEAK_TFLOPS,
                      **extra) -> Optional[dict]:
        """Emit one JSONL record for the iteration since :meth:`begin_iteration` (no-op
        unless a metrics path is set: resolving the events costs a device sync).
        ``flops``: the iteration's useful matrix FLOPs on this rank; the record then carries
        the achieved TFLOP/s over the ``compute`` phase and its fraction of ``peak_tflops``."""
        if not self.path or self._iter_mark is None:
            return None
        totals0, c0 = self._iter_mark
        self._iter_mark = None
        totals = self.timer.flush()
        self.resolve()
        phases = {k: round((v - totals0.get(k, 0.0)) * 1e3, 4) for k, v in totals.items()
                  if v - totals0.get(k, 0.0) > 0}
        colls = [self._annotate(c) for c in self.collectives[c0:]]
        nbytes = sum(c["bytes"] for c in colls)
        coll_ms = sum(c["ms"] for c in colls)
        rec = {"event": "iteration", "app": app, "iter": it, "world": self.world, "phases_ms": phases,
               "collective_ms": round(coll_ms, 4), "collective_bytes": nbytes,
               "collective_gbps": round(nbytes / (coll_ms / 1e3) / 1e9, 3) if coll_ms > 0 else None,
               "collectives": colls, **self.memory(), **extra}
        comp_ms = phases.get("compute", 0.0)
        if flops > 0 and comp_ms > 0:
            tf = flops / (comp_ms / 1e3) / 1e12
            rec["compute_tflops"] = float(f"{tf:.6g}")
            rec["mfma_peak_frac"] = float(f"{tf / peak_tflops:.6g}") if peak_tflops > 0 else None
        return self.emit(rec)

    def summary(self) -> dict:
        self.resolve()
        agg: Dict[str, dict] = {}
        for c in self.collectives:
            a = agg.setdefault(c["kind"], {"calls": 0, "s": 0.0, "bytes": 0, "ideal_s": 0.0})
            a["calls"] += 1
            a["s"] += c["s"]
            a["bytes"] += c["bytes"]
            a["ideal_s"] += ideal_collective_s(c["kind"], c["bytes"], self.world)
        return {"phases": dict(self.phases), "collectives": agg, "memory": self.memory()}
