"""Host schedulers (schdynamic/schstatic tests) and the 2-D block scheduler."""
import threading
import time

from harp_amd.runtime.dymoro import BlockScheduler, MPTask
from harp_amd.runtime.schedulers import DynamicScheduler, StaticScheduler, Task


class Square(Task):
    def run(self, x):
        return x * x


def test_dynamic_scheduler_lifecycle():
    s = DynamicScheduler([Square() for _ in range(4)])
    s.start()
    s.submit_all(range(20))
    outs = sorted(s.drain())
    assert outs == sorted(x * x for x in range(20))
    s.pause()
    s.submit(3)  # queued while paused
    s.start()
    assert s.wait_for_output(timeout=5) == 9
    s.stop()
    assert not s.errors


def test_static_scheduler_affinity_and_pipeline():
    seen = {}

    class T(Task):
        def __init__(self, i):
            self.i = i

        def run(self, x):
            seen.setdefault(self.i, []).append(x)
            if self.i == 0:
                self.submitter.submit(1, x + 100)  # pipeline into task 1
            return (self.i, x)

    s = StaticScheduler([T(0), T(1)])
    s.start()
    s.submit(0, 1)
    assert s.wait_for_output(0, timeout=5) == (0, 1)
    assert s.wait_for_output(1, timeout=5) == (1, 101)
    s.stop()
    assert seen == {0: [1], 1: [101]}


def test_block_scheduler_conflict_free():
    active_r, active_c = set(), set()
    lock = threading.Lock()
    violations = []

    def task(r, c):
        with lock:
            if r in active_r or c in active_c:
                violations.append((r, c))
            active_r.add(r)
            active_c.add(c)
        time.sleep(0.002)
        with lock:
            active_r.discard(r)
            active_c.discard(c)
        return 10

    res = BlockScheduler(4, 4, task, num_threads=4).schedule()
    assert not violations and res["items"] == 160 and len(res["blocks"]) == 16 and not res["remaining"]


def test_block_scheduler_timer():
    res = BlockScheduler(8, 8, lambda r, c: time.sleep(0.02) or 1, num_threads=2).schedule(time_budget=0.05)
    assert 0 < len(res["blocks"]) < 64 and len(res["remaining"]) == 64 - len(res["blocks"])


def test_mptask_records():
    class T(MPTask):
        def do_run(self, c, r):
            return len(c) * len(r)

    t = T()
    t([1, 2], [1, 2, 3])
    assert t.items == 6 and t.seconds >= 0
