"""The K-means tutorial of the reference (website/content/docs/examples/kmeans.md), written
as user code against the harp_amd mapper API (examples/kmeans_tutorial.py): the four
synchronisation strategies give the same centroids, and the km.sh accuracy gate's mean
distance band (contrib/test_scripts/km.sh:47,58: 2 workers, 1000 points, K=10, d=10,
U[0,10), 100 iterations -> (7.0, 7.8)) holds."""
import pytest
import torch

from examples.kmeans_tutorial import _job
from harp_amd.runtime.launcher import launch


@pytest.fixture(scope="module")
def runs():
    out = {}
    for s in ("allreduce", "broadcast-reduce", "push-pull", "regroup-allgather"):
        conf = {"n": 500, "k": 10, "d": 10, "iterations": 100, "strategy": s}
        out[s] = launch(_job, 2, args=(conf,), timeout=300)
    return out


def test_strategies_agree(runs):
    ref = runs["allreduce"][0]["centroids"]
    for s, res in runs.items():
        for r in res:
            assert torch.allclose(r["centroids"], ref, atol=1e-9), s


def test_km_sh_accuracy_band(runs):
    for s, res in runs.items():
        tot = sum(r["mean_distance"] for r in res) / len(res)  # equal point counts per worker
        assert 7.0 < tot < 7.8, (s, tot)
