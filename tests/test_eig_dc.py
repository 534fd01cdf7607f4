"""Divide-and-conquer tridiagonal eigensolver (host reference of csrc/tridiag_dc.hip) and the
compact-WY back-transform of harp_amd.ops.eig, on the CPU against numpy/LAPACK."""
import numpy as np
import pytest
import torch

from harp_amd.ops import eig as EIG
from harp_amd.ops.tridiag_dc import eigh_tridiag, tree_levels


def _cases():
    rng = np.random.default_rng(0)
    n = 120
    yield "randn", rng.standard_normal(n), rng.standard_normal(n - 1)
    yield "cluster", 1 + 1e-6 * rng.standard_normal(n), 1e-6 * rng.standard_normal(n - 1)
    yield "wilkinson", np.abs(np.arange(n) - n // 2).astype(float), np.ones(n - 1)
    e = np.ones(n - 1)
    e[::15] = 1e-15
    yield "glued", np.tile(np.abs(np.arange(15) - 7.0), 8), e
    d = np.ones(n)
    d[::2] = 2.0
    yield "decoupled", d, np.zeros(n - 1)
    for m in (1, 2, 3, 5, 17):
        yield f"n{m}", rng.standard_normal(m), rng.standard_normal(m - 1)


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_dc_reference_matches_lapack(case):
    _, d, e = case
    n = d.size
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    w, V = eigh_tridiag(d, e)
    nt = max(np.linalg.norm(T, 2), 1e-300)
    assert np.abs(V.T @ V - np.eye(n)).max() <= 1e-13
    assert np.abs(T @ V - V * w).max() <= 1e-13 * nt
    assert np.abs(w - np.linalg.eigvalsh(T)).max() <= 1e-13 * nt


def test_tree_covers_every_split_once():
    # csrc/tridiag_dc.hip dc_setup_kernel takes |e| off both sides of EVERY position 1 .. n - 1
    for n in (1, 2, 3, 7, 64, 1000):
        mids = [m[1] for lev in tree_levels(n) for m in lev]
        assert sorted(mids) == list(range(1, n))


def test_tree_level_metadata():
    """ops.eig._tree's host arrays for harp_dc_tridiag: level offsets, largest block, and the
    "covers all n rows" flags that let a level swap the two Q buffers (no copy-back)."""
    import torch

    from harp_amd.ops.eig import _tree

    for n in (2, 17, 64, 65, 1000, 4096):
        levels = tree_levels(n)
        merges, off, smax, nlev, _, full = _tree(n, torch.device("cpu"))
        assert nlev == len(levels) and merges.numel() == 3 * sum(len(lev) for lev in levels)
        for li, lev in enumerate(levels):
            assert off[li + 1] - off[li] == len(lev)
            assert smax[li] == max(hi - lo for lo, _, hi in lev)
            assert full[li] == int(sum(hi - lo for lo, _, hi in lev) == n)
            # merges of one level are disjoint row blocks
            spans = sorted((lo, hi) for lo, _, hi in lev)
            assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
        assert full[nlev - 1] == 1  # the top merge covers everything


def _householder_tridiag(A):
    """dsytd2-style reduction with the v[0] = 1 convention the HIP kernel stores."""
    A = A.copy()
    n = A.shape[0]
    Vt = np.zeros((n, n))
    tau = np.zeros(n)
    for k in range(n - 2):
        x = A[k + 1:, k].copy()
        alpha, sig = x[0], float(x[1:] @ x[1:])
        if sig == 0.0:
            continue
        beta = -np.copysign(np.sqrt(alpha * alpha + sig), alpha)
        t = (beta - alpha) / beta
        v = x / (alpha - beta)
        v[0] = 1.0
        H = np.eye(n)
        H[k + 1:, k + 1:] -= t * np.outer(v, v)
        A = H @ A @ H
        Vt[k, k + 1:] = v
        tau[k] = t
    return np.diag(A).copy(), np.diag(A, 1).copy(), Vt, tau


def test_back_transform_recovers_eigenvectors():
    rng = np.random.default_rng(1)
    n = 60
    X = rng.standard_normal((n, n))
    A = X + X.T
    d, e, Vt, tau = _householder_tridiag(A)
    w, Z = eigh_tridiag(d, e)
    Xv = EIG.back_transform(torch.from_numpy(Vt), torch.from_numpy(tau), torch.from_numpy(Z)).numpy()
    assert np.abs(Xv.T @ Xv - np.eye(n)).max() <= 1e-12
    assert np.abs(A @ Xv - Xv * w).max() <= 1e-12 * np.linalg.norm(A, 2)


def test_wy_factor_matches_back_transform():
    """The side-stream split (M = V T formed before the D&C, then two GEMMs) equals the
    one-shot compact-WY back-transform, including a tau = 0 (identity) reflector."""
    rng = np.random.default_rng(2)
    n = 48
    X = rng.standard_normal((n, n))
    A = X + X.T
    d, e, Vt, tau = _householder_tridiag(A)
    tau[5] = 0.0
    Vt[5] = rng.standard_normal(n)  # ignored: tau = 0
    w, Z = eigh_tridiag(d, e)
    Vt_t, tau_t, Z_t = (torch.from_numpy(a) for a in (Vt, tau, Z))
    ref = EIG.back_transform(Vt_t, tau_t, Z_t)
    Vm, Mt = EIG.wy_factor(Vt_t, tau_t)
    got = EIG.apply_wy(Vm, Mt, Z_t)
    assert torch.allclose(got, ref, rtol=0, atol=1e-13)
    assert EIG.wy_factor(Vt_t[:2, :2], tau_t[:2]) is None
