"""Dynamic model rotation ("dymoro", Harp computation model B).

Reference (ml/java/.../dymoro/):
  * ``Rotator`` wraps K model slices (tables), one ``RotateTask`` per slice on its own
    thread, so slice k rotates while compute runs on slice k+-1; ``getSplitMap(k)`` blocks
    until slice k's rotation finished (Rotator.java:30-86);
  * ``RotateTask.run``: compute the next rotation map, ``mapper.rotate(ctx,
    "rotate-<table>-<opID>", table, map)``, re-split the received table into column
    blocks (RotateTask.java:107-150); ``updateRotationMap`` follows a random order table
    (:158-210);
  * ``RotationUtil``: the master builds a (2P-1)*iters order table (per iteration a
    random placement permutation then P-1 distinct random shifts) and broadcasts it
    (RotationUtil.java:34-90);
  * ``Scheduler``: 2-D (row-split x col-split) conflict-free block scheduler with a timer
    budget (Scheduler.java:54-237); ``MPTask.doRun(cData, rData)`` (MPTask.java:56).

MI355X design: a rotation is a grouped ``ncclSend/ncclRecv`` of a device slab; the
:class:`DeviceRotator` keeps a spare receive buffer per slice and issues each slice's
rotation on its OWN communicator (its own RCCL stream) asynchronously, so the comm stream
overlaps the compute kernels on the current stream; completion is a device-side stream
wait, never a host sync (slice shapes are static, slice ids are derived from the order
table on the host). :class:`Rotator` provides the reference's table-level API on top of
the generic ``rotate`` collective for non-dense models.
"""
from __future__ import annotations

import math
import random
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from ..core.combiner import ArrCombiner, Operation
from ..core.table import PackedTable, Table
from ..parallel import collectives as C
from ..parallel.comm import Communicator


# ---------------------------------------------------------------- rotation orders
def create_rotation_order(rng: random.Random, num_iterations: int, num_workers: int) -> List[int]:
    """Order table of length (2P-1)*iters: per iteration a placement permutation of the P
    data blocks (identity in iteration 0), then the P-1 shifts 1..P-1 in random order."""
    P = num_workers
    orders: List[int] = []
    for it in range(num_iterations):
        if it == 0:
            orders += list(range(P))
        else:
            ids = list(range(P))
            while ids:
                orders.append(ids.pop(rng.randrange(len(ids))))
        ids = list(range(1, P))
        while ids:
            orders.append(ids.pop(rng.randrange(len(ids))))
    return orders


def get_rotation_sequences(mapper, num_iterations: int, seed: int = 0, ctx: str = "sgd") -> List[int]:
    """Master creates the order table and broadcasts it (RotationUtil.getRotationSequences)."""
    P = mapper.get_num_workers()
    n = (2 * P - 1) * num_iterations
    if mapper.is_master():
        orders = create_rotation_order(random.Random(seed), num_iterations, P)
        t = PackedTable([0], torch.tensor([orders], dtype=torch.int64, device=mapper.device),
                        combiner=ArrCombiner(Operation.SUM))
    else:
        t = PackedTable([], torch.zeros((0, n), dtype=torch.int64, device=mapper.device),
                        combiner=ArrCombiner(Operation.SUM))
    if not mapper.broadcast(ctx, "bcast-rotate-orders", t, mapper.get_master_id(), False):
        raise IOError("broadcast of rotation orders failed")
    return t.buffer[0].cpu().tolist()


def ring_strides(P: int, S: int) -> List[int]:
    """Ring strides for S concurrently rotating slices on P fully connected GPUs: slice k
    moves from worker w to w + stride_k, every stride coprime with P (so each slice still
    visits every worker once per iteration), alternating directions (1, P-1, 3, P-3, ...).
    On MI355X every GPU pair has its own xGMI link, so slices on different strides move
    over different links instead of sharing the one to the next rank (two slices: twice the
    rotation bandwidth)."""
    if P <= 2:
        return [1] * S
    cand: List[int] = []
    for a in range(1, P):
        if math.gcd(a, P) == 1:
            for st in (a, P - a):
                if st not in cand:
                    cand.append(st)
    return [cand[k % len(cand)] for k in range(S)]


class RotationSchedule:
    """Placement of P data blocks over P workers for every (iteration, step).

    ``placement(it, s)[i]`` = worker holding data block i at step s of iteration it. With
    ``orders=None`` the schedule is a ring of the given ``stride`` (coprime with P): block i
    sits on (i + stride*s) mod P, and every rotation sends to self + stride. Random
    ``orders`` (the reference's RotationUtil) ignore the stride."""

    def __init__(self, num_workers: int, orders: Optional[Sequence[int]] = None, stride: int = 1):
        self.P = num_workers
        self.orders = list(orders) if orders is not None else None
        self.stride = stride % max(num_workers, 1) if num_workers > 1 else 0
        if num_workers > 1 and math.gcd(self.stride, num_workers) != 1:
            raise ValueError(f"ring stride {stride} must be coprime with {num_workers} workers")

    def placement(self, it: int, s: int) -> List[int]:
        P = self.P
        if self.orders is None:
            return [(i + self.stride * s) % P for i in range(P)]
        row = self.orders[(2 * P - 1) * it:(2 * P - 1) * (it + 1)]
        if len(row) < 2 * P - 1:
            raise IndexError("rotation order table exhausted")
        base = row[:P]
        shift = 0 if s == 0 else row[P + s - 1]
        return [(base[i] + shift) % P for i in range(P)]

    def block_at(self, worker: int, it: int, s: int) -> int:
        return self.placement(it, s).index(worker)

    def rotation_map(self, it: int, s: int) -> List[int]:
        """Worker->worker map moving step (it, s) to the next step."""
        cur = self.placement(it, s)
        nxt = self.placement(it, s + 1) if s + 1 < self.P else self.placement(it + 1, 0)
        m = [0] * self.P
        for i in range(self.P):
            m[cur[i]] = nxt[i]
        return m


# ---------------------------------------------------------------- device rotation engine
class DeviceRotator:
    """Asynchronous rotation of equally-shaped device slabs (one per model slice).

    ``start(k, rmap)`` sends slab k to ``rmap[self]`` and receives the slab of the worker
    mapping to self into a spare buffer, on slice k's private communicator; ``get(k)``
    makes the current stream wait for it (no host sync) and returns the new slab."""

    def __init__(self, comm: Communicator, slabs: Sequence[torch.Tensor], name: str = "rot", metrics=None,
                 codec=None):
        self.comm = comm
        self.name = name
        self.slabs = list(slabs)
        # ``codec`` (ops.slabcodec.SlabCodec, optional): slabs travel as fixed-size sparse
        # payloads, encoded on the compute stream after the slab's last use and decoded in
        # place on arrival (no spare dense slab; the send buffer outlives the send)
        self.codec = codec if comm.world_size > 1 else None
        if self.codec is None:
            self.spare = [torch.empty_like(s) for s in self.slabs]
        else:
            self.sendbuf = [self.codec.empty_payload() for _ in self.slabs]
            self.recvbuf = [self.codec.empty_payload() for _ in self.slabs]
        self.channels = [comm.channel(f"{name}-{k}") for k in range(len(self.slabs))]
        self._work: Dict[int, list] = {}
        self._nops = 0
        self.comm_time = 0.0
        self.metrics = metrics  # records bytes per rotation + the exposed wait (see get)

    def start(self, k: int, rmap: Sequence[int]) -> None:
        me = self.comm.rank
        dst = rmap[me]
        src = list(rmap).index(me)
        if dst == me:
            return
        ch = self.channels[k]
        if self.codec is not None:
            self.codec.encode(self.slabs[k], self.sendbuf[k])
            self._work[k] = ch.sendrecv({dst: self.sendbuf[k]}, {src: self.recvbuf[k]}, async_op=True)
            return
        self._work[k] = ch.sendrecv({dst: self.slabs[k]}, {src: self.spare[k]}, async_op=True)

    def get(self, k: int) -> torch.Tensor:
        works = self._work.pop(k, None)
        if works is not None:
            if self.metrics is not None:
                # the wait makes the compute stream depend on the rotation; events around it
                # time only the part of the transfer NOT hidden behind compute
                slab = self.slabs[k]
                nbytes = self.codec.nbytes if self.codec is not None else slab.numel() * slab.element_size()
                with self.metrics.time_collective("rotate_wait", self.name, f"slice-{k}-{self._nops}",
                                                  nbytes, self.comm.device):
                    for w in works:
                        w.wait()
                self._nops += 1
            else:
                for w in works:
                    w.wait()  # stream-level wait on GPU (RCCL), blocking on gloo
            if self.codec is not None:
                self.codec.decode(self.recvbuf[k], self.slabs[k])
            else:
                self.slabs[k], self.spare[k] = self.spare[k], self.slabs[k]
        return self.slabs[k]

    def wait_all(self) -> None:
        for k in list(self._work):
            self.get(k)


# ---------------------------------------------------------------- table-level Rotator
class Rotator:
    """Reference-style rotator over generic tables (one rotation thread per slice).

    Each slice's rotations are issued from its own thread on its own communicator
    channel, so concurrent rotations of different slices keep a per-communicator issue
    order (the RCCL requirement; SURVEY §2.0 concurrency contract).

    ``static_rows``: the slices keep their row counts between rotations (the reference's
    fixed model slices), so PackedTable slices are flagged ``ring_rows`` and rotate with
    no per-hop header round trip after the first (``collectives._ring_rows``). Their ids
    change every hop, so they are NOT ``static_layout`` (that flag promises a fixed id
    layout to the cached push / pull / join plans)."""

    def __init__(self, tables: Sequence[Table], mapper, orders: Optional[Sequence[int]] = None, ctx: str = "rotate",
                 static_rows: bool = False):
        self.tables = list(tables)
        if static_rows:
            for t in self.tables:
                if isinstance(t, PackedTable):
                    t.ring_rows = True
        self.mapper = mapper
        P = mapper.get_num_workers()
        self.schedule = RotationSchedule(P, orders)
        self.channels = [mapper.comm.channel(f"{ctx}-table-{k}") for k in range(len(tables))]
        self._pool = ThreadPoolExecutor(max_workers=max(1, len(tables)))
        self._fut: Dict[int, Future] = {}
        self._step = [0] * len(tables)
        self.comm_time = 0.0

    def get_split_map(self, k: int) -> Table:
        f = self._fut.pop(k, None)
        if f is not None:
            f.result()
        return self.tables[k]

    def rotate(self, k: int) -> None:
        step = self._step[k]
        P = self.schedule.P
        it, s = divmod(step, P)
        rmap = self.schedule.rotation_map(it, s) if self.schedule.orders is not None else None
        self._step[k] += 1

        def work():
            t0 = time.perf_counter()
            ok = C.rotate(self.channels[k], self.tables[k], rmap)
            self.comm_time += time.perf_counter() - t0
            if not ok:
                raise IOError(f"rotate of slice {k} failed")

        self._fut[k] = self._pool.submit(work)

    def start(self) -> None:
        pass

    def pause(self) -> None:
        for k in list(self._fut):
            self.get_split_map(k)

    def stop(self) -> None:
        self.pause()
        self._pool.shutdown(wait=True)


# ---------------------------------------------------------------- time-bounded steps
class StepBudget:
    """Time-bounded rotation step on the GPU (the reference's Scheduler timer,
    Scheduler.java:118-137: blocks are submitted until a TimerTask fires, so every worker
    rotates after ``time`` ms whatever its share of work).

    A step's work is cut into ``pieces`` (kernel launches over successive windows of the
    data, so the cut falls on kernel boundaries); pieces are issued one ahead of the
    device: before issuing piece i+1 the host waits for piece i-1's completion event,
    then stops issuing once ``budget_s`` has elapsed since the step began. The device
    never idles between pieces, and at most one piece runs past the budget. On the CPU
    the pieces run synchronously and the clock is checked after each one."""

    def __init__(self, budget_s: float, device: torch.device):
        self.budget_s = float(budget_s)
        self.device = device
        self.compute_s = 0.0  # accumulated step time (for the tuner)

    def run(self, pieces) -> Tuple[int, int]:
        """``pieces``: iterable of zero-arg callables returning items trained. Returns
        (items, pieces run)."""
        gpu = self.device.type == "cuda"
        t0 = time.perf_counter()
        items, n, prev = 0, 0, None
        for piece in pieces:
            if n and time.perf_counter() - t0 >= self.budget_s:
                break
            items += int(piece())
            n += 1
            if gpu:
                ev = torch.cuda.Event()
                ev.record()
                if prev is not None:
                    prev.synchronize()  # piece n-1 done; piece n is running: the device stays busy
                prev = ev
        if prev is not None:
            prev.synchronize()
        self.compute_s += time.perf_counter() - t0
        return items, n


def tune_budget(mapper, compute_s: float, items: int, total_items: int, steps: int, ratio: float,
                ctx: str = "sgd", it: int = 0) -> float:
    """Reference adjustMiniBatch (SGDCollectiveMapper.java:623-668): all-gather every
    worker's (compute time, items trained) of the first iteration, then size the per-step
    budget so one iteration trains ``ratio`` of all items:
    budget = ratio / (trained fraction) * (mean per-step compute time)."""
    P = mapper.get_num_workers()
    t = PackedTable([mapper.get_self_id()], torch.tensor([[compute_s, float(items)]], dtype=torch.float64,
                                                         device=mapper.device), combiner=ArrCombiner(Operation.SUM))
    if not mapper.allgather(ctx, f"allgather-compute-status-{it}", t):
        raise IOError("allgather of compute status failed")
    tot = t.buffer.sum(0).cpu().tolist()
    frac = tot[1] / max(float(total_items), 1.0)
    avg_step = tot[0] / P / max(steps, 1)
    return ratio / max(frac, 1e-12) * avg_step


class BudgetTuner:
    """Per-iteration retuning of the rotation-step time budget so the share of all items
    trained per iteration lands in ``[min_bound, max_bound]`` percent (the reference's LDA
    ``adjustMiniBatch``, LDAMPCollectiveMapper.java:295-314, 477-557).

    Each iteration every worker's (compute time, items trained) is all-gathered. Over
    ``max_bound``: halve the budget. Under ``min_bound``: double it (and keep doubling
    while the projection stays under); an under-train after an over-train starts a
    ``break_period`` (1, 2, 4, ... iterations) during which the budget is left alone,
    which damps oscillation.

    Deviation, measured on MI355X: the reference decides on the trained percentage scaled
    by (predicted / actual) compute time, predicted = budget x P x slices x P, which
    divides out steps that overran their timer. On the GPU a step's pieces are issued one
    ahead (:class:`StepBudget`), so every step overruns by up to two pieces and that
    projection stayed inside the band while 87 % of the tokens were trained. The
    halve / double rule here therefore uses the TRAINED percentage; the projection is
    used once, for the first tuning (``proportional_first``), which sets the budget in one
    proportional step toward the band's midpoint (the SGD ``adjustMiniBatch`` rule,
    SGDCollectiveMapper.java:623-668): the reference starts LDA at a 1 s CPU step, and a
    GPU step is milliseconds, so plain halving would need ~10 iterations to get there.
    Returns the new budget in seconds. Bounds outside (0, 100] fall back to 50/50 and
    ``max_bound == 100`` disables tuning, as in the reference (:98-118)."""

    def __init__(self, min_bound: int, max_bound: int, proportional_first: bool = True):
        lo = min_bound if 0 < min_bound <= 100 else 50
        hi = max_bound if 0 < max_bound <= 100 else 50
        hi = max(hi, lo)
        self.enabled = hi != 100
        self.min_bound, self.max_bound = (100, 100) if not self.enabled else (lo, hi)
        self.proportional_first = proportional_first
        self.has_over_trained = False
        self.last_under_train = 0
        self.break_period = 0
        self.tuned = 0
        self.history: List[dict] = []

    def __call__(self, mapper, budget_s: float, compute_s: float, items: int, total_items: int, steps: int,
                 it: int, ctx: str = "lda") -> float:
        if not self.enabled:
            return budget_s
        P = mapper.get_num_workers()
        t = PackedTable([mapper.get_self_id()], torch.tensor([[compute_s, float(items)]], dtype=torch.float64,
                                                             device=mapper.device), combiner=ArrCombiner(Operation.SUM))
        if not mapper.allgather(ctx, f"allgather-compute-status-{it}", t):
            raise IOError("allgather of compute status failed")
        tot_time, tot_items = t.buffer.sum(0).cpu().tolist()
        real = 100.0 * tot_items / max(float(total_items), 1.0)
        predicted = budget_s * P * steps
        proj = real * predicted / max(tot_time, 1e-12)
        new = budget_s
        rec = {"iter": it, "trained_pct": round(real, 3), "projected_pct": round(proj, 3), "budget_s": budget_s}
        if self.tuned == 0 and self.proportional_first:
            if proj > self.max_bound or proj < self.min_bound:
                target = 0.5 * (self.min_bound + self.max_bound)
                new = budget_s * target / max(proj, 1e-9)
        elif self.last_under_train == 0 or it - self.last_under_train >= self.break_period:
            if real > self.max_bound:
                self.has_over_trained = True
                new = budget_s / 2
            elif real < self.min_bound:
                if self.has_over_trained:
                    self.last_under_train = it
                    self.break_period = 1 if self.break_period == 0 else 2 * self.break_period
                new = budget_s * 2
                potential = 2 * real
                while potential < self.min_bound and potential > 0:
                    potential *= 2
                    new *= 2
        self.tuned += 1
        rec["new_budget_s"] = new
        self.history.append(rec)
        return new


# ---------------------------------------------------------------- 2-D block scheduler
class BlockScheduler:
    """Conflict-free 2-D (row split x column split) block scheduler.

    Never runs two blocks sharing a row split or a column split at the same time
    (Scheduler.java:104-116,150-213), refills as blocks finish, and optionally stops
    submitting when ``time_budget`` seconds have elapsed (the reference's timer that keeps
    all workers rotating in lockstep, :118-137). ``task(row, col) -> items`` runs on a
    host thread pool; native (ctypes) tasks release the GIL and run in parallel."""

    def __init__(self, num_rows: int, num_cols: int, task: Callable[[int, int], int], num_threads: int = 4):
        self.R, self.C = num_rows, num_cols
        self.task = task
        self.num_threads = max(1, num_threads)

    def schedule(self, time_budget: Optional[float] = None, blocks: Optional[Sequence[Tuple[int, int]]] = None) -> dict:
        todo = set(blocks) if blocks is not None else {(r, c) for r in range(self.R) for c in range(self.C)}
        busy_r, busy_c = set(), set()
        lock = threading.Condition()
        done_items = [0]
        done_blocks = []
        t0 = time.perf_counter()
        inflight = [0]

        def run(r, c):
            try:
                n = self.task(r, c)
            finally:
                with lock:
                    busy_r.discard(r)
                    busy_c.discard(c)
                    done_items[0] += int(n or 0)
                    done_blocks.append((r, c))
                    inflight[0] -= 1
                    lock.notify_all()

        with ThreadPoolExecutor(max_workers=self.num_threads) as ex:
            with lock:
                first = True  # the first round of conflict-free blocks is submitted before the
                while todo or inflight[0]:  # timer counts (Scheduler.java:104-117 then :118-137)
                    timed_out = (not first and time_budget is not None
                                 and time.perf_counter() - t0 > time_budget)
                    launched = False
                    if not timed_out:
                        for (r, c) in sorted(todo):
                            if inflight[0] >= self.num_threads:
                                break
                            if r not in busy_r and c not in busy_c:
                                todo.discard((r, c))
                                busy_r.add(r)
                                busy_c.add(c)
                                inflight[0] += 1
                                ex.submit(run, r, c)
                                launched = True
                    first = False
                    if timed_out and not inflight[0]:
                        break
                    if not launched:
                        lock.wait(timeout=0.05)
        return {"items": done_items[0], "blocks": done_blocks, "remaining": sorted(todo),
                "seconds": time.perf_counter() - t0}


class MPTask:
    """Base of a model-parallel task: ``do_run(col_data, row_data) -> items`` with timing
    records (MPTask.java:27-80)."""

    def __init__(self):
        self.items = 0
        self.seconds = 0.0

    def do_run(self, col_data, row_data) -> int:  # pragma: no cover - abstract
        raise NotImplementedError

    def __call__(self, col_data, row_data) -> int:
        t0 = time.perf_counter()
        n = self.do_run(col_data, row_data)
        self.seconds += time.perf_counter() - t0
        self.items += int(n or 0)
        return n
