"""Single-node launcher: one process per GPU (or per CPU worker under gloo).

Replaces the reference's Hadoop MapCollective job path (MapCollectiveRunner ->
MapCollectiveAppMaster -> container launcher writing ``nodes``/``tasks``/``lock`` to
HDFS) and the standalone ssh ``Driver`` (collective/Driver.java:
203-268). Gang semantics come from ``torch.distributed`` rendezvous: every rank joins
the group or the job fails (the reference disables speculation for the same reason,
MapCollectiveAppMaster.java:88-99).

Two entry points:
  * :func:`launch` — spawn ``num_workers`` local processes (``torch.multiprocessing``)
    that each build a :class:`CollectiveMapper`, used by tests (gloo, 127.0.0.1) and by
    single-node runs;
  * ``python -m torch.distributed.run --nproc-per-node N -m harp_amd.runtime.launcher
    --mapper pkg.mod:Class ...`` — the torchrun form (RANK/LOCAL_RANK/WORLD_SIZE env).
"""
from __future__ import annotations

import argparse
import datetime
import importlib
import json
import os
import pickle
import socket
import sys
import traceback
from typing import Any, Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..parallel.comm import Communicator, collective_timeout_s
from .inputformat import multi_file_splits
from .mapper import CollectiveMapper, Context, KeyValReader


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> Communicator:
    """Initialise torch.distributed from the environment (torchrun contract) and pin
    this process to GPU ``LOCAL_RANK``. Returns the world communicator. ``timeout_s``
    (default :func:`collective_timeout_s`) is the collective watchdog."""
    if timeout_s is None:
        timeout_s = collective_timeout_s()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    use_gpu = backend == "nccl" or (backend is None and torch.cuda.is_available())
    if use_gpu:
        torch.cuda.set_device(local_rank % max(torch.cuda.device_count(), 1))
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if world > 1 and not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    dev = torch.device("cuda", torch.cuda.current_device()) if use_gpu else torch.device("cpu")
    return Communicator(None, dev)


def shutdown() -> None:
    if dist.is_available() and dist.is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        t = [_to_cpu(v) for v in obj]
        return type(obj)(t) if not hasattr(obj, "_fields") else type(obj)(*t)
    return obj


def _worker(rank: int, world: int, port: int, backend: str, target: Callable, args: tuple,
            result_q, env: Optional[Dict[str, str]] = None) -> None:
    os.environ.update(env or {})
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    try:
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(world, 1)))
        comm = init_distributed(backend)
        res = target(comm, *args)
        # by-value pickle (not the shared-memory fd reducers of torch.multiprocessing):
        # the worker may exit before the parent reads, which would strand an fd handle
        result_q.put((rank, "ok", pickle.dumps(_to_cpu(res))))
    except BaseException as e:  # report to parent, then fail
        result_q.put((rank, "error", f"{e!r}\n{traceback.format_exc()}"))
        raise
    finally:
        shutdown()


def launch(target: Callable, num_workers: int, args: tuple = (), backend: str = "gloo",
           timeout: float = 600.0, retries: int = 0, env: Optional[Dict[str, str]] = None,
           grace_s: float = 10.0) -> List[Any]:
    """Run ``target(comm, *args)`` on ``num_workers`` local ranks; return results by rank.

    ``target`` must be importable (module-level) so it can be pickled to the workers.
    Failure handling: when a rank fails or dies, the others get ``grace_s``
    seconds to report (a dead peer makes their next collective fail, or the collective
    watchdog fires), then the gang is terminated; with ``retries`` the whole job is started
    again (``HARP_ATTEMPT`` = 1, 2, ... in the workers' environment) — the reference's
    whole-job resubmission (contrib KmeansMapCollective jobRetryCount); applications resume
    from their last checkpoint."""
    for attempt in range(retries + 1):
        e = dict(env or {}, HARP_ATTEMPT=str(attempt))
        try:
            return _launch_once(target, num_workers, args, backend, timeout, e, grace_s)
        except Exception:
            if attempt == retries:
                raise
    raise AssertionError("unreachable")


def _launch_once(target, num_workers, args, backend, timeout, env, grace_s) -> List[Any]:
    import torch.multiprocessing as mp

    if num_workers == 1:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            return [target(Communicator(None, torch.device("cpu") if backend == "gloo" else None), *args)]
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, num_workers, port, backend, target, args, q, env), daemon=False)
             for r in range(num_workers)]
    for p in procs:
        p.start()
    results: Dict[int, Any] = {}
    errors = []
    import time as _t

    deadline = _t.monotonic() + timeout
    while len(results) + len(errors) < num_workers:
        if _t.monotonic() > deadline:
            break
        if not q.empty():
            rank, status, val = q.get()
            (results.__setitem__(rank, pickle.loads(val)) if status == "ok" else errors.append((rank, val)))
            if errors:  # a failed gang: the rest get a grace period, then are stopped
                deadline = min(deadline, _t.monotonic() + grace_s)
        elif all(not p.is_alive() for p in procs) and q.empty():
            break
        elif any(p.exitcode not in (None, 0) for p in procs):  # died without reporting
            deadline = min(deadline, _t.monotonic() + grace_s)
            _t.sleep(0.01)
        else:
            _t.sleep(0.01)
    for p in procs:
        p.join(timeout=max(0.5, deadline - _t.monotonic()))
        if p.is_alive():
            p.terminate()
            p.join(5)
    if errors:
        raise RuntimeError(f"worker(s) failed: {errors}")
    if len(results) != num_workers:
        codes = [p.exitcode for p in procs]
        raise RuntimeError(f"only {len(results)}/{num_workers} workers reported (timeout or crash; exit codes {codes})")
    return [results[r] for r in range(num_workers)]


def run_mapper(comm: Communicator, mapper_cls, records: Sequence = (), conf: Optional[dict] = None):
    """Build and run one mapper on this rank (used as a :func:`launch` target)."""
    mapper = mapper_cls(comm)
    return mapper.run(KeyValReader(records), Context(conf))


def _load(spec: str):
    mod, _, name = spec.partition(":")
    return getattr(importlib.import_module(mod), name)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="harp_amd collective job (run under torchrun)")
    ap.add_argument("--mapper", required=True, help="module:Class of a CollectiveMapper subclass")
    ap.add_argument("--input", nargs="*", default=[], help="input files (split across workers)")
    ap.add_argument("--conf", default="{}", help="JSON job configuration")
    ap.add_argument("--backend", default=None)
    a = ap.parse_args(argv)
    comm = init_distributed(a.backend)
    splits = multi_file_splits(a.input, comm.world_size, seed=0)
    records = [(i, f) for i, f in enumerate(splits[comm.rank])]
    res = run_mapper(comm, _load(a.mapper), records, json.loads(a.conf))
    if comm.rank == 0 and res is not None:
        print(json.dumps(res, default=str))
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
