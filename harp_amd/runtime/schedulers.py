"""Intra-worker host task schedulers (Harp L0).

Reference: core/harp-collective/.../schdynamic/DynamicScheduler.java:33-287 (shared input
queue feeding one TaskMonitor thread per Task object, output queue, pause/pauseNow/stop
via sentinels, waitForOutput/hasOutput comparing input and output counts) and
schstatic/StaticScheduler.java:42-162 (one input queue per task = task-affine,
``submit(taskID, input)``, ``waitForOutput(taskID)``, a ``Submitter`` that lets tasks feed
other tasks for pipelines).

On MI355X the data-parallel inner loops run as HIP kernels; these schedulers drive the
host-side work around them (file loading/parsing, CPU fallbacks, I/O pipelines). Native
calls made through ctypes release the GIL, so task threads run truly in parallel.
"""
from __future__ import annotations

import queue
import threading
from typing import Any, Callable, Dict, Generic, List, Optional, Sequence, TypeVar

I = TypeVar("I")
O = TypeVar("O")

_STOP = object()
_PAUSE = object()


class Task(Generic[I, O]):
    """A unit of host work: ``run(input) -> output`` (schdynamic/Task.java)."""

    def run(self, inp: I) -> O:  # pragma: no cover - abstract
        raise NotImplementedError


class _FnTask(Task):
    def __init__(self, fn: Callable):
        self.fn = fn

    def run(self, inp):
        return self.fn(inp)


def _as_task(t) -> Task:
    return t if isinstance(t, Task) else _FnTask(t)


class DynamicScheduler(Generic[I, O]):
    """Work-sharing scheduler: any free task thread takes the next input."""

    def __init__(self, tasks: Sequence[Task | Callable]):
        self.tasks = [_as_task(t) for t in tasks]
        self._in: "queue.Queue" = queue.Queue()
        self._out: "queue.Queue" = queue.Queue()
        self._threads: List[threading.Thread] = []
        self._running = False
        self._n_in = 0
        self._n_out = 0
        self._lock = threading.Lock()
        self._paused = threading.Semaphore(0)
        self.errors: List[BaseException] = []

    def submit(self, inp: I) -> None:
        with self._lock:
            self._n_in += 1
        self._in.put(inp)

    def submit_all(self, inputs) -> None:
        for x in inputs:
            self.submit(x)

    def _monitor(self, task: Task) -> None:
        while True:
            item = self._in.get()
            if item is _STOP:
                return
            if item is _PAUSE:
                self._paused.release()
                return
            try:
                out = task.run(item)
            except BaseException as e:  # surface worker errors to the caller
                self.errors.append(e)
                out = None
            self._out.put(out)
            with self._lock:
                self._n_out += 1

    def start(self) -> None:
        if self._running:
            return
        self._running = True
        self._threads = [threading.Thread(target=self._monitor, args=(t,), daemon=True) for t in self.tasks]
        for th in self._threads:
            th.start()

    def _halt(self, sentinel, front: bool) -> None:
        if not self._running:
            return
        if front:  # pauseNow: sentinels go ahead of queued inputs
            with self._in.mutex:
                for _ in self._threads:
                    self._in.queue.appendleft(sentinel)
                self._in.not_empty.notify_all()
        else:
            for _ in self._threads:
                self._in.put(sentinel)
        if sentinel is _PAUSE:
            for _ in self._threads:
                self._paused.acquire()
        for th in self._threads:
            th.join()
        self._running = False

    def pause(self) -> None:
        """Finish everything submitted so far, then park the task threads."""
        self._halt(_PAUSE, front=False)

    def pause_now(self) -> None:
        """Stop after the inputs currently being processed; queued inputs stay queued."""
        self._halt(_PAUSE, front=True)

    def stop(self) -> None:
        self._halt(_STOP, front=False)

    def has_output(self) -> bool:
        with self._lock:
            return self._n_out > 0 or not self._out.empty()

    def wait_for_output(self, timeout: Optional[float] = None) -> O:
        out = self._out.get(timeout=timeout)
        with self._lock:
            self._n_out -= 1
            self._n_in -= 1
        return out

    def drain(self) -> List[O]:
        outs = []
        while True:
            with self._lock:
                pending = self._n_in
            if pending == 0:
                return outs
            outs.append(self.wait_for_output())

    def get_tasks(self) -> List[Task]:
        return self.tasks


class StaticScheduler(Generic[I, O]):
    """Task-affine scheduler: input ``i`` is processed by task ``task_id``."""

    def __init__(self, tasks: Sequence[Task | Callable]):
        self.tasks = [_as_task(t) for t in tasks]
        n = len(self.tasks)
        self._in = [queue.Queue() for _ in range(n)]
        self._out = [queue.Queue() for _ in range(n)]
        self._threads: List[threading.Thread] = []
        self._running = False
        self.submitter = Submitter(self)
        for t in self.tasks:
            setattr(t, "submitter", self.submitter)
        self.errors: List[BaseException] = []

    def submit(self, task_id: int, inp: I) -> None:
        self._in[task_id].put(inp)

    def _monitor(self, i: int) -> None:
        while True:
            item = self._in[i].get()
            if item is _STOP:
                return
            try:
                out = self.tasks[i].run(item)
            except BaseException as e:
                self.errors.append(e)
                out = None
            self._out[i].put(out)

    def start(self) -> None:
        if self._running:
            return
        self._running = True
        self._threads = [threading.Thread(target=self._monitor, args=(i,), daemon=True) for i in range(len(self.tasks))]
        for th in self._threads:
            th.start()

    def stop(self) -> None:
        if not self._running:
            return
        for q in self._in:
            q.put(_STOP)
        for th in self._threads:
            th.join()
        self._running = False

    pause = stop

    def wait_for_output(self, task_id: int, timeout: Optional[float] = None) -> O:
        return self._out[task_id].get(timeout=timeout)

    def has_output(self, task_id: int) -> bool:
        return not self._out[task_id].empty()


class Submitter:
    """Lets a task of a StaticScheduler submit work to another task (pipelines)."""

    def __init__(self, sched: StaticScheduler):
        self._sched = sched

    def submit(self, task_id: int, inp) -> None:
        self._sched.submit(task_id, inp)
