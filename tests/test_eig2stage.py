"""Two-stage tridiagonalisation host reference (harp_amd/ops/eig2stage.py): band form,
bulge chasing, back-transform, and the minimal safe lag between pipelined sweeps."""
import numpy as np
import pytest

from harp_amd.ops import eig2stage as E


@pytest.mark.parametrize("n,b", [(3, 2), (10, 3), (37, 4), (100, 8), (64, 16)])
def test_two_stage_matches_lapack(n, b):
    rng = np.random.default_rng(n * 10 + b)
    M = rng.standard_normal((n, n))
    A = (M + M.T) / 2
    B, _ = E.sy2sb(A, b)
    i, j = np.indices(B.shape)
    assert np.abs(B[np.abs(i - j) > b]).max(initial=0.0) == 0.0  # band form
    d, e, _, Bt = E.sb2st(B, b)
    assert np.abs(np.tril(Bt, -2)).max(initial=0.0) == 0.0  # tridiagonal
    w, Z = E.eigh_two_stage(A, b)
    assert np.abs(w - np.linalg.eigvalsh(A)).max() <= 1e-12 * n
    assert np.abs(Z.T @ Z - np.eye(n)).max() <= 1e-13 * n
    assert np.abs(A @ Z - Z * w).max() <= 1e-12 * n


def _steps(n, b, s):
    out, lo, hi, col = [], s + 1, min(s + b, n - 1), s
    while lo <= n - 1 and hi - lo >= 1:
        out.append((col, lo, hi))
        col, lo, hi = lo, hi + 1, min(hi + b, n - 1)
    return out


def _chase_step(B, n, b, col, lo, hi):
    v, tau, beta = E.householder(B[lo:hi + 1, col].copy())
    if tau != 0.0:
        rows = slice(lo, hi + 1)
        cend = min(hi + b, n - 1)
        D = B[rows, rows].copy()
        p = tau * (D @ v)
        w = p - 0.5 * tau * (p @ v) * v
        B[rows, rows] = D - np.outer(v, w) - np.outer(w, v)
        for c_lo, c_hi in ((col, lo - 1), (hi + 1, cend)):
            if c_hi >= c_lo:
                blk = B[rows, c_lo:c_hi + 1].copy()
                blk -= tau * np.outer(v, v @ blk)
                B[rows, c_lo:c_hi + 1] = blk
                B[c_lo:c_hi + 1, rows] = blk.T
    B[lo, col] = B[col, lo] = beta
    B[lo + 1:hi + 1, col] = 0.0
    B[col, lo + 1:hi + 1] = 0.0


def test_pipelined_sweeps_need_lag_three():
    """Sweep s may take step k once sweep s - 1 finished step k + 2: interleaving at lag 3
    reproduces the sequential chase exactly, lag 2 does not (the schedule a parallel
    bulge-chasing kernel must respect)."""
    n, b = 97, 8
    rng = np.random.default_rng(2)
    M = rng.standard_normal((n, n))
    B, _ = E.sy2sb((M + M.T) / 2, b)
    ref = B.copy()
    S = [_steps(n, b, s) for s in range(n - 2)]
    for s in range(n - 2):
        for st in S[s]:
            _chase_step(ref, n, b, *st)
    diffs = {}
    for lag in (2, 3):
        Bt = B.copy()
        T = max(lag * s + len(S[s]) for s in range(n - 2))
        for t in range(T):
            for s in reversed(range(n - 2)):  # later sweeps first: the hazardous order
                k = t - lag * s
                if 0 <= k < len(S[s]):
                    _chase_step(Bt, n, b, *S[s][k])
        diffs[lag] = np.abs(Bt - ref).max()
    assert diffs[3] == 0.0 and diffs[2] > 1e-6, diffs
