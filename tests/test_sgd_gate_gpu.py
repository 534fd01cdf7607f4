"""The reference's MF-SGD accuracy gate on the GPU path at FULL concurrency,
and plain vs lossless write-back on the bench's Netflix-shape distribution.

Gate: ml/java/test_scripts/mfsgd.sh:63,73-75 -- r = 40, lambda = 0.05, epsilon = 0.002, 200
iterations, 2 workers, test RMSE in (0.80, 0.84); the reference run gave 0.8345 and this
framework's sequential CPU path 0.8344 (tests/test_sgd_mf.py). The GPU runs every XCD's 128
blocks (2,048 concurrent update streams per cell); on ML-10M's skewed items that many streams
collide on hot H rows, and the rows whose collisions would lose updates take atomic write-back
(SGDConfig.conflict_mode = "hot", ops.mf.hot_items; the default "cap" mode instead lowers the
blocks per XCD: 0.8377 on this gate, profiles/r5_sgd_gpu)."""
import pytest
import torch

from harp_amd.runtime.launcher import launch

pytestmark = pytest.mark.gpu


def _gate_job(comm, cfg, nu, ni, train, test):
    from harp_amd.models.sgd_mf import SGDCollectiveMapper
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    comm = Communicator(None, torch.device("cuda", 0))  # the two gloo ranks share the GPU
    m = SGDCollectiveMapper(comm, cfg, nu, ni, train, test)
    m.run(KeyValReader([]))
    return {"rmse": m.result["rmse"], "bpx": m.bpx, "hot": m.hot_items, "atomic": m.atomic,
            "placement": m.placement_events}


def test_ml10m_gate_at_full_concurrency(cuda):
    from harp_amd.models.sgd_mf import SGDConfig
    from harp_amd.utils.datasets import load_ml10m

    data = load_ml10m()
    if data is None:
        pytest.skip("ML-10M split not available")
    train, test, nu, ni = data
    cfg = SGDConfig(rank=40, lam=0.05, lr=0.002, epochs=200, num_slices=2, test_every=50, init="reference",
                    conflict_mode="hot")
    res = launch(_gate_job, 2, args=(cfg, nu, ni, train, test), timeout=900)
    r0 = res[0]
    test_rmse = r0["rmse"][-1][2]
    print({"test_rmse": test_rmse, "blocks_per_xcd": r0["bpx"], "hot_items": r0["hot"], "atomic": r0["atomic"]})
    assert r0["bpx"] == cfg.blocks_per_xcd == 128  # no concurrency cap
    assert r0["hot"] > 0
    assert 0.80 < test_rmse < 0.84
    assert test_rmse <= 0.8365  # within 0.002 of the sequential CPU run (0.8344)


def test_plain_vs_lossless_writeback_on_bench_shape(cuda):
    """On the bench's own Netflix-shape synthetic (480,189 x 17,770, 100M ratings, skew 2:
    per-cell sum p^2 ~ 0.0015; rank 128, 10 epochs as the bench's record) plain H stores and
    fully lossless atomic write-back reach the same train RMSE within 0.1 %: the bench
    number is accuracy-safe at its distribution, and the hot-item rule flags nothing there.
    (Scaled down to 10M ratings the gap is 0.4 %: fewer updates per item per epoch, a less
    converged model -- the check is made at the size the bench runs.)"""
    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings
    from harp_amd.ops import mf as MF
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    users, items, n = 480_189, 17_770, 100_480_507
    u, i, v = synthetic_ratings(users, items, n, seed=7, device=cuda)
    out = {}
    for atomic in (0, MF.ATOMIC_W | MF.ATOMIC_H):
        cfg = SGDConfig(rank=128, epochs=10, test_every=10, num_slices=1, atomic=atomic)
        m = SGDCollectiveMapper(Communicator(None, cuda), cfg, users, items, (u, i, v), None)
        m.run(KeyValReader([]))
        out[atomic] = (m.rmse_history[-1][1], m.hot_items, m.bpx)
    plain, lossless = out[0][0], out[3][0]
    print(out)
    assert out[0][1] == 0 and out[0][2] == 128
    assert abs(plain - lossless) / lossless < 1e-3, out
