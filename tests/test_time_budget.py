"""Time-bounded rotation steps (reference dymoro Scheduler timer, Scheduler.java:118-137)
and first-iteration retuning (SGDCollectiveMapper.java:623-668 adjustMiniBatch), for
MF-SGD and LDA, on 1 and 2 gloo ranks. The deterministic full-pass mode stays the
default; with an unbounded budget the budgeted path trains exactly what it would."""
import math

import pytest
import torch

from harp_amd.models.sgd_mf import SGDConfig, SGDCollectiveMapper, synthetic_ratings
from harp_amd.parallel.comm import Communicator
from harp_amd.runtime.dymoro import StepBudget
from harp_amd.runtime.launcher import launch
from harp_amd.runtime.mapper import KeyValReader


def _sgd(comm, **kw):
    tr = synthetic_ratings(600, 120, 9000, seed=6)
    cfg = SGDConfig(rank=8, epochs=3, test_every=0, xcd_blocks=False, **kw)
    m = SGDCollectiveMapper(comm, cfg, 600, 120, tr, None)
    m.run(KeyValReader([]))
    return {"W": m.W.cpu(), "trained": m.trained, "budget": list(getattr(m, "budget_history", [])),
            "n_local": m.train.n}


def _cpu():
    return Communicator(None, torch.device("cpu"))


def test_unbounded_budget_equals_full_passes():
    full = _sgd(_cpu())
    bud = _sgd(_cpu(), time_budget_ms=1e9, budget_pieces=4)
    assert bud["trained"] == full["trained"] == 3 * 9000
    assert torch.allclose(bud["W"], full["W"], atol=1e-6)


def test_tiny_budget_cuts_each_step_to_one_piece_and_cursors_advance():
    res = _sgd(_cpu(), time_budget_ms=1e-6, budget_pieces=4)
    # one piece (ceil(m/4) ratings of the slice) per visit: about a quarter per epoch
    assert 0.2 * 3 * 9000 < res["trained"] < 0.3 * 3 * 9000


def test_budget_retuned_after_first_epoch_two_workers():
    res = launch(_sgd_tuned, 2, timeout=300)
    for r in res:
        b = r["budget"]
        assert len(b) == 2 and b[1] > 0 and b[1] != b[0]
    assert res[0]["budget"][1] == pytest.approx(res[1]["budget"][1])  # one all-gathered decision


def _sgd_tuned(comm):
    return _sgd(comm, time_budget_ms=0.05, budget_pieces=8, tune_ratio=0.5)


def test_step_budget_counts_and_stops():
    b = StepBudget(0.0, torch.device("cpu"))
    calls = []
    items, n = b.run((lambda i=i: calls.append(i) or 10) for i in range(5))
    assert (items, n, calls) == (10, 1, [0])  # the first piece always runs
    b = StepBudget(10.0, torch.device("cpu"))
    items, n = b.run((lambda: 3) for _ in range(4))
    assert (items, n) == (12, 4)


def _lda(comm, budget):
    from harp_amd.models.lda import LDACollectiveMapper, LDAConfig, synthetic_corpus

    doc, word = synthetic_corpus(150, 400, 6, 40, seed=2)
    cfg = LDAConfig(num_topics=8, iterations=4, print_interval=1, time_budget_ms=budget, budget_pieces=4)
    m = LDACollectiveMapper(comm, cfg, 150, 400, (doc, word))
    m.init_model(KeyValReader([]))
    toks = [m.iterate(it) for it in range(4)]
    m.rot.wait_all()
    return {"tokens": toks, "total": int(m.tz.numel()), "loglik": m.log_likelihood(3),
            "nk": int(m.nk.sum())}


@pytest.mark.parametrize("P", [1, 2])
def test_lda_budget(P):
    full = launch(_lda, P, args=(0.0,), timeout=300)
    unb = launch(_lda, P, args=(1e9,), timeout=300)
    tiny = launch(_lda, P, args=(1e-6,), timeout=300)
    for f, u, t in zip(full, unb, tiny):
        assert f["tokens"] == u["tokens"] == [f["total"]] * 4
        assert all(x < f["total"] for x in t["tokens"])
        assert f["nk"] == u["nk"] == t["nk"]  # topic counts stay consistent under any cut
    assert unb[0]["loglik"] == pytest.approx(full[0]["loglik"], rel=0.02)


def test_cpu_threaded_block_scheduler_path():
    """CPU workers run the 8 x 8 cells through the conflict-free 2-D BlockScheduler (the
    reference's Scheduler); unbounded it trains every rating, a tiny timer stops early."""
    tr = synthetic_ratings(600, 120, 9000, seed=6)
    out = {}
    for name, b in (("all", 0.0), ("timer", 1e-6)):
        cfg = SGDConfig(rank=8, epochs=2, test_every=0, xcd_blocks=True, cpu_threads=4, time_budget_ms=b)
        m = SGDCollectiveMapper(_cpu(), cfg, 600, 120, tr, None)
        m.run(KeyValReader([]))
        out[name] = m.trained
    assert out["all"] == 2 * 9000
    assert 0 < out["timer"] < 2 * 9000


def _lda_tuned(comm, lo, hi, iters=5):
    from harp_amd.models.lda import LDACollectiveMapper, LDAConfig, synthetic_corpus

    doc, word = synthetic_corpus(4000, 3000, 20, 60, seed=5)
    cfg = LDAConfig(num_topics=64, iterations=iters, print_interval=0, time_budget_ms=1000.0, budget_pieces=8,
                    min_bound=lo, max_bound=hi)
    m = LDACollectiveMapper(comm, cfg, 4000, 3000, (doc, word))
    m.init_model(KeyValReader([]))
    toks = [m.iterate(it) for it in range(iters)]
    m.rot.wait_all()
    return {"tokens": toks, "total": m.total_tokens, "budget": list(m.budget_history), "hist": m.tuner.history,
            "nk": int(m.nk.sum())}


def test_lda_budget_tuner_converges_into_band_two_workers():
    """LDA timer auto-tuning (LDAMPCollectiveMapper.java:295-314, 477-557): starting at the
    reference's 1 s step (a full sweep here), the all-gathered trained percentage lands in
    [40, 80] within 3 iterations, and every worker takes the same budget decisions."""
    res = launch(_lda_tuned, 2, args=(40, 80), timeout=600)
    for r in res:
        assert r["budget"][0] == pytest.approx(1.0)
        assert r["hist"][0]["trained_pct"] == pytest.approx(100.0)  # iteration 0: everything
        assert r["budget"][1] < 0.5  # one proportional step down
        tot = [sum(x) for x in zip(*[q["tokens"] for q in res])]
        pct = [100.0 * t / r["total"] for t in tot]
        assert any(40 <= p <= 80 for p in pct[1:4]), (pct, r["hist"])
        assert r["nk"] == r["total"]
    assert res[0]["budget"] == pytest.approx(res[1]["budget"])  # one all-gathered decision


def test_budget_tuner_state_machine():
    """Halve over the band, double under it, and a break period after an under-train that
    followed an over-train (the reference's hasOverTrained / lastUnderTrainIte / breakPeriod)."""
    from harp_amd.runtime.dymoro import BudgetTuner

    class _M:  # one worker: the all-gather returns its own (time, items)
        device = torch.device("cpu")

        def get_num_workers(self):
            return 1

        def get_self_id(self):
            return 0

        def allgather(self, ctx, op, t):
            return True

    t = BudgetTuner(40, 80, proportional_first=False)
    m = _M()
    # full budget used, 100 % trained: over -> halve
    assert t(m, 1.0, 4.0, 100, 100, 4, it=1) == pytest.approx(0.5)
    # 10 % trained with the budget fully used: under after an over -> double twice (10->20->40),
    # and a break period of 1 starts at iteration 2
    assert t(m, 0.5, 2.0, 10, 100, 4, it=2) == pytest.approx(2.0)
    assert t.break_period == 1 and t.last_under_train == 2
    # at iteration 3 (3 - 2 >= 1) tuning resumes; 60 % is inside the band -> unchanged
    assert t(m, 2.0, 8.0, 60, 100, 4, it=3) == pytest.approx(2.0)
    assert BudgetTuner(0, 100).enabled is False and BudgetTuner(0, 0).max_bound == 50


def test_threaded_cpu_path_with_tuning():
    """the threaded CPU BlockScheduler path with a budget and tune_ratio used to
    raise AttributeError after epoch 0 (no StepBudget on that path)."""
    tr = synthetic_ratings(600, 120, 9000, seed=6)
    cfg = SGDConfig(rank=8, epochs=2, test_every=0, xcd_blocks=True, cpu_threads=4, time_budget_ms=5.0,
                    tune_ratio=0.5)
    m = SGDCollectiveMapper(_cpu(), cfg, 600, 120, tr, None)
    m.run(KeyValReader([]))
    assert len(m.budget_history) == 2 and m.budget_history[1] > 0 and m.budget.compute_s > 0
