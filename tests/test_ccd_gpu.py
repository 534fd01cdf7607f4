"""MF-CCD HIP kernels (csrc/ccd.hip) vs the torch fp64 formulation of the same update
order: residual recompute and a full coordinate phase, short (register) and long rows."""
import pytest
import torch

from harp_amd.ops import ccd as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [8, 37, 120])
def test_ccd_phase_and_residual(cuda, k):
    g = torch.Generator().manual_seed(k)
    n_rows, n_cols = 300, 500
    # rows 7 / 13 / 17 (257-8192 nonzeros): workgroup-per-row kernel; row 11 (8193-12288): its
    # wide form (column ids in LDS); row 19 (> 12288): lockstep
    rows = torch.cat([torch.randint(0, n_rows, (20000,), generator=g), torch.full((700,), 7),
                      torch.full((9000,), 11), torch.full((5000,), 13), torch.full((200,), 17),
                      torch.full((13000,), 19)])
    cols = torch.randint(0, n_cols, (rows.numel(),), generator=g)
    vals = torch.rand(rows.numel(), generator=g, dtype=torch.float64) * 4 + 1
    o = torch.argsort(rows, stable=True)
    rows, cols, vals = rows[o], cols[o], vals[o]
    W = torch.rand(n_rows, k, generator=g, dtype=torch.float64) * 0.3
    H = torch.rand(n_cols, k, generator=g, dtype=torch.float64) * 0.3
    ptr = C.row_ptr_of(rows, n_rows)
    # CPU fp64 reference
    res_c = C.residual(rows.int(), cols.int(), vals, W, H)
    Wc = W.clone()
    C.phase(rows.int(), ptr, cols.int(), res_c, Wc, H, 0.05)
    # GPU fp32
    d = lambda x, dt=torch.float32: x.to(cuda, dt).contiguous()
    rg, cg = d(rows, torch.int32), d(cols, torch.int32)
    res_g = C.residual(rg, cg, d(vals), d(W), d(H))
    torch.cuda.synchronize()
    r0 = C.residual(rows.int(), cols.int(), vals, W, H)
    assert torch.allclose(res_g.double().cpu(), r0, atol=1e-4)
    Wg = d(W)
    C.phase(rg, ptr.to(cuda), cg, res_g, Wg, d(H), 0.05)
    torch.cuda.synchronize()
    assert torch.allclose(Wg.double().cpu(), Wc, atol=2e-3, rtol=2e-3), (Wg.double().cpu() - Wc).abs().max()
    assert torch.allclose(res_g.double().cpu(), res_c, atol=5e-3)


def test_ccd_model_gpu_matches_cpu(cuda):
    from harp_amd.models.ccd import CCDConfig, train_ccd
    from harp_amd.models.sgd_mf import synthetic_ratings
    from harp_amd.parallel.comm import Communicator

    u, i, v = synthetic_ratings(400, 300, 20000, seed=1, true_rank=4)
    key = torch.unique(u * 300 + i)
    u, i = key // 300, key % 300
    v = (1 + (u * 7 + i * 3) % 5).double()
    cfg = CCDConfig(rank=16, lam=0.1, iterations=4)
    a = train_ccd(Communicator(device="cpu"), u, i, v, 400, 300, cfg)
    b = train_ccd(Communicator(device=cuda), u, i, v, 400, 300, cfg)
    ra, rb = a["history"][-1]["train_rmse"], b["history"][-1]["train_rmse"]
    assert abs(ra - rb) < 1e-3 * max(1.0, ra), (ra, rb)


def test_ccd_rotation_mode_matches_allgather_on_gpu(cuda):
    """Rotation mode (dimension slices rotated, csrc/ccd.hip phase kernels on slices) on
    one GPU follows the same per-row update order as the allgather mode."""
    from harp_amd.models.ccd import CCDConfig, train_ccd
    from harp_amd.parallel.comm import Communicator

    g = torch.Generator().manual_seed(2)
    n = 200_000
    u = torch.randint(0, 5000, (n,), generator=g)
    i = torch.randint(0, 800, (n,), generator=g)
    v = torch.rand(n, generator=g) * 4 + 1
    c = Communicator(None, cuda)
    a = train_ccd(c, u, i, v, 5000, 800, CCDConfig(rank=24, iterations=3))
    b = train_ccd(c, u, i, v, 5000, 800, CCDConfig(rank=24, iterations=3, mode="rotation", slices_per_rank=2))
    assert torch.allclose(a["W"], b["W"], rtol=1e-3, atol=1e-4)
    assert a["history"][-1]["train_rmse"] == pytest.approx(b["history"][-1]["train_rmse"], rel=1e-4)


def test_ccd_residual_carry_gpu(cuda):
    """fp32 residuals carried by permutation between phases (one GPU) stay within rounding
    of the per-phase recompute over 6 iterations."""
    from harp_amd.models.ccd import CCDConfig, train_ccd
    from harp_amd.parallel.comm import Communicator

    g = torch.Generator().manual_seed(3)
    n = 300_000
    u = torch.randint(0, 6000, (n,), generator=g)
    i = (torch.rand(n, generator=g) ** 2 * 900).long()  # skewed items: long rows take the lockstep path
    v = torch.rand(n, generator=g) * 4 + 1
    c = Communicator(None, cuda)
    a = train_ccd(c, u, i, v, 6000, 900, CCDConfig(rank=24, iterations=6, residual_resync=1))
    b = train_ccd(c, u, i, v, 6000, 900, CCDConfig(rank=24, iterations=6))
    for ha, hb in zip(a["history"], b["history"]):
        assert hb["train_rmse"] == pytest.approx(ha["train_rmse"], rel=1e-5)
    assert torch.allclose(a["W"], b["W"], rtol=1e-3, atol=1e-4)
