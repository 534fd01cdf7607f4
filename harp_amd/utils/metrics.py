"""Metrics / tracing.

The reference logs ad-hoc wall-clock deltas (K-means ``Compute/Merge/Aggregate`` per
iteration at KMeansCollectiveMapper.java:191-193, SGD ``computeTime/waitTime`` at
SGDCollectiveMapper.java:294-298, rotation comm time at RotateTask.java:109-123) plus
JVM memory/GC logs (CollectiveMapper.java:686-714).

Here: per-phase timers backed by HIP events on the GPU (no host sync inside the
timed region; resolved lazily), per-collective records (kind, ctx, op, seconds,
bytes), HBM usage from ``hipMemGetInfo`` and JSONL emission; optional roctx ranges so
rocprofv3 traces show the same phase names.
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


class PhaseTimer:
    """Accumulates named phase times. On GPU uses hipEvents recorded on the current
    stream, resolved at :meth:`flush`; on CPU uses perf_counter."""

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

    def flush(self) -> Dict[str, float]:
        if self._pending:
            torch.cuda.synchronize()
            for name, s, e in self._pending:
                self.totals[name] += s.elapsed_time(e) / 1e3
                self.counts[name] += 1
            self._pending.clear()
        return dict(self.totals)

    def reset(self) -> None:
        self._pending.clear()
        self.totals.clear()
        self.counts.clear()


class Metrics:
    def __init__(self, rank: int = 0, path: Optional[str] = None):
        self.rank = rank
        self.path = path or os.environ.get("HARP_METRICS_JSONL")
        self.phases: Dict[str, float] = defaultdict(float)
        self.collectives: List[dict] = []
        self.timer = PhaseTimer()

    def record(self, name: str, seconds: float) -> None:
        self.phases[name] += seconds

    def collective(self, kind: str, ctx: str, op: str, seconds: float, nbytes: int = 0) -> None:
        rec = {"kind": kind, "ctx": ctx, "op": op, "s": seconds, "bytes": nbytes}
        self.collectives.append(rec)
        if len(self.collectives) > 10000:
            del self.collectives[:5000]

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

    def emit(self, record: dict) -> None:
        record = {"rank": self.rank, "t": time.time(), **record}
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(record) + "\n")
        return record

    def summary(self) -> dict:
        agg: Dict[str, dict] = {}
        for c in self.collectives:
            a = agg.setdefault(c["kind"], {"calls": 0, "s": 0.0, "bytes": 0})
            a["calls"] += 1
            a["s"] += c["s"]
            a["bytes"] += c["bytes"]
        return {"phases": dict(self.phases), "collectives": agg, "memory": self.memory()}


# xGMI link model used to report achieved-vs-ideal collective bandwidth:
XGMI_LINK_GBPS = 153.0
XGMI_LINKS = 7


def ring_allreduce_ideal_s(nbytes: int, world: int, link_gbps: float = XGMI_LINK_GBPS) -> float:
    """Ideal single-ring allreduce time (2(P-1)/P * S over one link per direction)."""
    if world <= 1:
        return 0.0
    return 2 * (world - 1) / world * nbytes / (link_gbps * 1e9)
