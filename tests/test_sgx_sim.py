"""SGX-simulated K-means (experimental kmeans/sgxsimu): the enclave cost model reproduces
the reference's arithmetic and the wrapped K-means still matches plain Lloyd."""
import math

import torch

from harp_amd.models.kmeans import KMeansConfig, run_kmeans
from harp_amd.models.sgx_sim import SGXConfig, SGXCostModel, run_sgx_kmeans
from harp_amd.runtime.launcher import launch


def test_cost_model_matches_reference_formulas():
    m = SGXCostModel()
    # creation: (221000 + 96*1024*22.677) kcycles * 0.0002941 ms/kcycle per enclave
    per = (221000.0 + 96 * 1024 * 22.677) * 0.0002941
    assert m.enclave_creation_ms(96, 4) == int(per * 4)
    # attestation: (C(4,2) + (2-1)*4) pairs * 80 kcycles
    assert m.local_attestation_ms(4, 2) == int((math.comb(4, 2) + 4) * 80 * 0.0002941)
    # 10k centroids x 101 doubles -> 7890 KB
    assert m.double_kb(10000 * 101) == 10000 * 101 * 8 // 1024
    kb = 7890
    assert m.regroup_ms(kb, 4) == int(3 * (9.0 + 8.5) * 0.0002941 + (kb // 4) * 6 * 1.4 * 0.0002941)
    assert m.allgather_ms(kb, 4) == int((9.0 + 8.5 * 3) * 0.0002941 + kb * 1.4 * 0.0002941)
    # paging fit at an 8 MB shard: s = 8192/10/1024 = 0.8
    s = 0.8
    r = -0.000592887941 * s ** 3 + 0.03776145898 * s ** 2 - 0.172624736 * s + 0.08813241271
    assert abs(m.mem_ratio(8192) - r) < 1e-12
    sh = m.shard_ms(8192, 1000.0)
    assert sh["ecall"] == int((8.5 + 8192 * 1.4) * 0.0002941)
    assert sh["mem"] == max(0, int(1000.0 * r) - sh["ecall"])


def _job(comm, fn, cfg, x, c0, *extra):
    P, r = comm.world_size, comm.rank
    lo, hi = r * x.shape[0] // P, (r + 1) * x.shape[0] // P
    return fn(comm, cfg, *extra, points=x[lo:hi], init_centroids=c0)


def test_sgx_kmeans_same_model_plus_accounted_overhead():
    g = torch.Generator().manual_seed(4)
    x = torch.rand((800, 16), generator=g) * 10
    c0 = torch.rand((8, 16), generator=g) * 10
    cfg = KMeansConfig(num_points=400, num_centroids=8, dim=16, iterations=6, strategy="regroup_allgather")
    plain = launch(_job, 2, args=(run_kmeans, cfg, x, c0), timeout=300)
    sgx = launch(_job, 2, args=(run_sgx_kmeans, cfg, x, c0, SGXConfig(threads=2, enclave_task_mb=1)), timeout=300)
    assert torch.allclose(plain[0]["centroids"], sgx[0]["centroids"], atol=1e-5)
    rec = sgx[0]["sgx"]
    assert len(rec["iterations"]) == 6
    assert rec["totals_ms"]["init"] > 0  # enclave creation + attestation
    for it in rec["iterations"]:
        assert it["sgx_ms"] == it["ecall"] + it["ocall"] + it["mem"] + it["comm"]
        assert it["gpu_ms"] > 0
