"""Checkpoint / resume and model output for every iterative app.

Each app runs on 2 gloo ranks with a checkpoint every iteration; rank 1 is killed
(``HARP_FAULT kind=exit``) part-way, the launcher restarts the gang (``retries=1``), the
app resumes from ``LATEST`` and must end with the model of an uninterrupted run. Re-shard
cases save with 2 ranks and resume with 1. Model dumps follow the reference formats
(SGDCollectiveMapper.java:737-818 ``id : v1 .. vr``; LDAMPCollectiveMapper.java:593-628
``word topic:count ..``)."""
import os

import pytest
import torch

from harp_amd.runtime.launcher import launch
from harp_amd.utils.model_io import read_factor_rows, read_topic_counts

FAULT = {"HARP_FAULT": "rank=1,iter=2,kind=exit"}


# ------------------------------------------------------------------------------ MF-SGD
def _ratings():
    from harp_amd.models.sgd_mf import synthetic_ratings

    return synthetic_ratings(400, 90, 6000, seed=4)


def _sgd_job(comm, d, model_dir=""):
    from harp_amd.models.sgd_mf import SGDConfig, SGDCollectiveMapper
    from harp_amd.runtime.mapper import KeyValReader

    cfg = SGDConfig(rank=8, epochs=5, test_every=1, xcd_blocks=False, random_order=True,
                    checkpoint_dir=str(d), checkpoint_every=1, model_dir=model_dir)
    tr = _ratings()
    m = SGDCollectiveMapper(comm, cfg, 400, 90, tr, tr)
    m.run(KeyValReader([]))
    return {"rmse": m.rmse_history, "W": m.W.cpu(), "users": m.users.cpu(), "start": m.start_iteration}


def test_sgd_kill_and_resume(tmp_path):
    ref = launch(_sgd_job, 2, args=(tmp_path / "ref",), timeout=300)
    res = launch(_sgd_job, 2, args=(tmp_path / "ft", str(tmp_path / "model")), timeout=300, retries=1, env=FAULT)
    assert [x["start"] for x in res] == [2, 2]  # died before the it-2 checkpoint: resume at 2
    for a, b in zip(ref, res):
        assert torch.allclose(a["W"], b["W"], atol=1e-6)
        assert [x[0] for x in a["rmse"]] == [x[0] for x in b["rmse"]] == [1, 2, 3, 4, 5]
        assert a["rmse"][-1][1] == pytest.approx(b["rmse"][-1][1], rel=1e-6)
    # model dump: W rows of both workers cover every user exactly once; H covers every item
    ids, rows = [], []
    for r in range(2):
        i, w = read_factor_rows(str(tmp_path / "model" / f"W-{r}"))
        ids.append(i)
        assert w.shape[1] == 8
    allu = torch.cat(ids)
    assert allu.unique().numel() == allu.numel()
    hid = torch.cat([read_factor_rows(str(tmp_path / "model" / f"H-{r}"))[0] for r in range(2)])
    assert sorted(hid.tolist()) == list(range(90))
    assert float(open(tmp_path / "model" / "evaluation").read()) == pytest.approx(res[0]["rmse"][-1][2])


def _sgd_one(comm, d):
    return _sgd_job(comm, d)


def test_sgd_reshard_two_to_one(tmp_path):
    from harp_amd.models.sgd_mf import SGDConfig, SGDCollectiveMapper
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    two = launch(_sgd_job, 2, args=(tmp_path,), timeout=300)
    # resume the finished 2-rank checkpoint on 1 rank for 2 more epochs
    cfg = SGDConfig(rank=8, epochs=7, test_every=1, xcd_blocks=False, random_order=True,
                    checkpoint_dir=str(tmp_path), checkpoint_every=0)
    tr = _ratings()
    m = SGDCollectiveMapper(Communicator(None, torch.device("cpu")), cfg, 400, 90, tr, tr)
    m.init_model(KeyValReader([]))
    start = m.resume()
    assert start == 5
    W = torch.zeros(400, 8)
    for x in two:
        W[x["users"]] = x["W"]
    assert torch.allclose(m.W, W[m.users], atol=1e-7)
    tr_rmse, _ = m._eval_ring(start - 1)
    assert tr_rmse == pytest.approx(two[0]["rmse"][-1][1], rel=1e-6)  # same model, any world


# ------------------------------------------------------------------------------ LDA
def _corpus():
    from harp_amd.models.lda import synthetic_corpus

    return synthetic_corpus(120, 300, 5, 30, seed=3)


def _lda_job(comm, d, push_pull=False, model_dir=""):
    from harp_amd.models.lda import LDACollectiveMapper, LDAConfig, LDAPushPullMapper
    from harp_amd.runtime.mapper import KeyValReader

    cfg = LDAConfig(num_topics=8, iterations=5, print_interval=1, checkpoint_dir=str(d), checkpoint_every=1,
                    block_words=64, model_dir=model_dir)
    cls = LDAPushPullMapper if push_pull else LDACollectiveMapper
    m = cls(comm, cfg, 120, 300, _corpus())
    m.run(KeyValReader([]))
    return {"loglik": m.loglik, "tz": m.tz.cpu(), "nk": m.nk.cpu(), "start": m.start_iteration}


@pytest.mark.parametrize("push_pull", [False, True])
def test_lda_kill_and_resume(tmp_path, push_pull):
    ref = launch(_lda_job, 2, args=(tmp_path / "ref", push_pull), timeout=300)
    res = launch(_lda_job, 2, args=(tmp_path / "ft", push_pull, str(tmp_path / "model")), timeout=300, retries=1,
                 env=FAULT)
    assert [x["start"] for x in res] == [2, 2]
    for a, b in zip(ref, res):
        assert torch.equal(a["tz"], b["tz"]) and torch.equal(a["nk"], b["nk"])
        assert [x[0] for x in b["loglik"]] == [1, 2, 3, 4, 5]
        assert a["loglik"][-1][1] == pytest.approx(b["loglik"][-1][1], rel=1e-12)
    # word model dump (printed at the last iteration): every word id once, counts sum to the
    # token count
    folder = tmp_path / "model" / "tmp_word_model" / "5"
    words = {}
    for r in range(2):
        words.update(read_topic_counts(str(folder / str(r))))
    doc, word = _corpus()
    tot = sum(sum(v.values()) for v in words.values())
    assert tot == doc.numel()
    assert set(int(w) for w in word.unique()) <= set(words)
    assert float(open(tmp_path / "model" / "evaluation").read()) == pytest.approx(res[0]["loglik"][-1][1])


# ------------------------------------------------------------------------------ CCD / ALS
def _mf_tr():
    g = torch.Generator().manual_seed(5)
    n = 3000
    u = torch.randint(0, 200, (n,), generator=g)
    i = torch.randint(0, 70, (n,), generator=g)
    v = (torch.rand(n, generator=g) * 4 + 1)
    return u, i, v


def _ccd_job(comm, d, model_dir=""):
    from harp_amd.models.ccd import CCDConfig, train_ccd

    u, i, v = _mf_tr()
    P, r = comm.world_size, comm.rank
    sl = slice(r * u.numel() // P, (r + 1) * u.numel() // P)
    res = train_ccd(comm, u[sl], i[sl], v[sl], 200, 70,
                    CCDConfig(rank=6, iterations=5, checkpoint_dir=str(d), checkpoint_every=1, model_dir=model_dir))
    return {"W": res["W"].cpu(), "H": res["H"].cpu(), "uid": res["user_ids"].cpu(), "hist": res["history"],
            "start": res["start_iteration"]}


def _als_job(comm, d, model_dir=""):
    from harp_amd.models.als import ALSConfig, train_als

    u, i, v = _mf_tr()
    P, r = comm.world_size, comm.rank
    sl = slice(r * u.numel() // P, (r + 1) * u.numel() // P)
    res = train_als(comm, u[sl], i[sl], v[sl], 200, 70,
                    ALSConfig(factors=5, iterations=5, checkpoint_dir=str(d), checkpoint_every=1, model_dir=model_dir))
    return {"W": res["X"].cpu(), "H": res["Y"].cpu(), "uid": res["user_ids"].cpu(), "hist": res["history"],
            "start": res["start_iteration"]}


@pytest.mark.parametrize("job", [_ccd_job, _als_job], ids=["ccd", "als"])
def test_factor_apps_kill_and_resume(tmp_path, job):
    ref = launch(job, 2, args=(tmp_path / "ref",), timeout=300)
    res = launch(job, 2, args=(tmp_path / "ft", str(tmp_path / "model")), timeout=300, retries=1, env=FAULT)
    assert [x["start"] for x in res] == [2, 2]
    for a, b in zip(ref, res):
        assert torch.allclose(a["W"], b["W"], atol=1e-9) and torch.allclose(a["H"], b["H"], atol=1e-9)
        assert [h["iter"] for h in b["hist"]] == [1, 2, 3, 4, 5]
    ids = torch.cat([read_factor_rows(str(tmp_path / "model" / f"W-{r}"))[0] for r in range(2)])
    assert sorted(ids.tolist()) == list(range(200))


@pytest.mark.parametrize("job", [_ccd_job, _als_job], ids=["ccd", "als"])
def test_factor_apps_reshard_two_to_one(tmp_path, job):
    two = launch(job, 2, args=(tmp_path,), timeout=300)
    from harp_amd.parallel.comm import Communicator

    # a 1-rank job over the finished checkpoint starts at iteration 5 == cfg.iterations: no
    # work left, the returned factors are the re-sharded checkpoint
    one = job(Communicator(None, torch.device("cpu")), tmp_path)
    W = torch.zeros_like(one["W"])
    for x in two:
        W[x["uid"]] = x["W"]
    assert torch.allclose(one["W"], W, atol=1e-12)
    assert len(one["hist"]) == 5


def test_gather_factors_ids_above_2_24():
    from harp_amd.models.mf_common import gather_factors

    res = launch(_big_ids_job, 2, timeout=120)
    n, f = res[0]
    assert n == 2 and f


def _big_ids_job(comm):
    from harp_amd.models.mf_common import gather_factors

    base = (1 << 24) + 1  # odd ids above 2^24 are not representable in fp32
    ids = torch.tensor([base + 2 * comm.rank + 1], dtype=torch.int64)
    F = torch.full((1, 3), float(comm.rank + 1))
    full = gather_factors(comm, ids, F, base + 8)
    ok = bool(full[base + 1, 0] == 1.0) and bool(full[base + 3, 0] == 2.0)
    return (int((full[:, 0] != 0).sum()), ok)


# ------------------------------------------------------------------------------ K-means
def _km_job(comm, d, strategy):
    from harp_amd.models.kmeans import KMeansConfig, run_kmeans

    g = torch.Generator().manual_seed(8)
    x = torch.rand((900, 6), generator=g) * 10
    c0 = torch.rand((10, 6), generator=g) * 10
    P, r = comm.world_size, comm.rank
    cfg = KMeansConfig(num_points=900 // P, num_centroids=10, dim=6, iterations=6, strategy=strategy,
                       checkpoint_dir=str(d), checkpoint_every=1)
    return run_kmeans(comm, cfg, points=x[r * 900 // P:(r + 1) * 900 // P], init_centroids=c0)


def test_rotation_kmeans_kill_and_resume(tmp_path):
    ref = launch(_km_job, 2, args=(tmp_path / "ref", "rotation"), timeout=300)
    res = launch(_km_job, 2, args=(tmp_path / "ft", "rotation"), timeout=300, retries=1, env=FAULT)
    assert [x["start_iteration"] for x in res] == [2, 2]
    assert torch.allclose(ref[0]["centroids"], res[0]["centroids"], atol=1e-6)
    assert res[0]["objective"] == pytest.approx(ref[0]["objective"], rel=1e-9)


@pytest.mark.parametrize("strategy", ["allreduce", "rotation"])
def test_kmeans_resume_on_other_world_size(tmp_path, strategy):
    """a replicated centroid table saved by 2 ranks must not be summed twice
    when 1 rank resumes it."""
    from harp_amd.models.kmeans import KMeansConfig, KMeansCollectiveMapper
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    two = launch(_km_job, 2, args=(tmp_path, strategy), timeout=300)
    m = KMeansCollectiveMapper(Communicator(None, torch.device("cpu")),
                               KMeansConfig(num_points=900, num_centroids=10, dim=6, iterations=6,
                                            strategy=strategy, checkpoint_dir=str(tmp_path)))
    m.init_model(KeyValReader([]))
    assert m.resume() == 6
    assert torch.allclose(m.c[:10], two[0]["centroids"], atol=1e-6)


def _ccd_rot_job(comm, d):
    from harp_amd.models.ccd import CCDConfig, train_ccd

    u, i, v = _mf_tr()
    P, r = comm.world_size, comm.rank
    sl = slice(r * u.numel() // P, (r + 1) * u.numel() // P)
    res = train_ccd(comm, u[sl], i[sl], v[sl], 200, 70,
                    CCDConfig(rank=6, iterations=5, mode="rotation", checkpoint_dir=str(d), checkpoint_every=1))
    return {"W": res["W"].cpu(), "H": res["H"].cpu(), "start": res["start_iteration"], "hist": res["history"]}


def test_ccd_rotation_mode_kill_and_resume(tmp_path):
    ref = launch(_ccd_rot_job, 2, args=(tmp_path / "ref",), timeout=300)
    res = launch(_ccd_rot_job, 2, args=(tmp_path / "ft",), timeout=300, retries=1, env=FAULT)
    assert [x["start"] for x in res] == [2, 2]
    for a, b in zip(ref, res):
        assert torch.allclose(a["W"], b["W"], atol=1e-9) and torch.allclose(a["H"], b["H"], atol=1e-9)
        assert len(b["hist"]) == 5


def _mds_job(comm, d, model_dir=""):
    from harp_amd.models import mds as MD
    from tests.test_mds import _problem

    D, W = _problem(30, seed=4)
    P, r = comm.world_size, comm.rank
    a, b = r * 30 // P, (r + 1) * 30 // P
    cfg = MD.MDSConfig(d=3, alpha=0.8, threshold=1e-6, checkpoint_dir=str(d), checkpoint_every=1, model_dir=model_dir)
    out = MD.wda_mds(comm, D[a:b], W[a:b], a, 30, cfg)
    return {"X": out["X"].cpu(), "stress": out["stress"], "start": out["start_stage"], "hist": out["history"]}


def test_mds_kill_and_resume_and_x_file(tmp_path):
    """Annealing-stage checkpoints of the replicated embedding: a rank killed in stage 2
    (before its checkpoint) restarts at stage 2 and ends bit-identical to the uninterrupted run; rank 0 writes X in
    the reference's storeXOnMaster format."""
    from harp_amd.utils.model_io import read_mds_points

    ref = launch(_mds_job, 2, args=(tmp_path / "ref",), timeout=300)
    res = launch(_mds_job, 2, args=(tmp_path / "ft", str(tmp_path / "model")), timeout=300, retries=1, env=FAULT)
    assert [x["start"] for x in res] == [2, 2]
    for a, b in zip(ref, res):
        assert torch.equal(a["X"], b["X"]) and a["hist"] == b["hist"]
    ids, X, labels = read_mds_points(str(tmp_path / "model" / "X"))
    assert ids.tolist() == list(range(30)) and labels == [1] * 30
    assert torch.allclose(X, res[0]["X"], atol=1e-9)
    # the replicated X resumes on a different world size
    one = launch(_mds_job, 1, args=(tmp_path / "ft",), timeout=300)[0]
    assert one["start"] == len(ref[0]["hist"]) - 1  # every annealing stage was checkpointed
