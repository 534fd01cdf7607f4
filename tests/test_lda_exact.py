"""The exact one-sweep distribution behind the GPU sampler's distribution test
(harp_amd/ops/lda_check.py) checked on the CPU against a direct Monte Carlo of the same
sequential collapsed-Gibbs sweep (numpy, vectorised over replicas): the enumeration that
gates the production kernel must itself be right."""
import itertools

import numpy as np
import pytest

from harp_amd.ops import lda_check as C


def _simulate(order, R, alpha, beta, vbeta, rng):
    T, n = len(C.ACTIVE), len(C.DOC_PAT)
    z0 = np.array(C.Z0_IDX)
    cur = np.tile(z0, (R, 1))
    eye = np.eye(T)
    snap = np.array(C.WORD_BG, dtype=np.float64)
    for j in range(n):
        snap[C.WORD_PAT[j], z0[j]] += 1
    inv = 1.0 / (np.array(C.NK_ACTIVE, dtype=np.float64) + vbeta)
    done = []
    for i in order:
        d, w, c = C.DOC_PAT[i], C.WORD_PAT[i], C.CHUNK_OF[i]
        nd = sum(eye[cur[:, j]] for j in range(n) if j != i and C.DOC_PAT[j] == d)
        nw = np.tile(snap[w], (R, 1)) - eye[z0[i]]
        for j in done:
            if C.CHUNK_OF[j] == c:
                nw += eye[cur[:, j]] - eye[z0[j]]
        p = (nd + alpha) * (nw + beta) * inv
        cdf = np.cumsum(p / p.sum(1, keepdims=True), 1)
        cur[:, i] = (rng.random((R, 1)) > cdf).sum(1).clip(max=T - 1)
        done.append(i)
    return (cur * (4 ** np.arange(n - 1, -1, -1))).sum(1)


@pytest.mark.parametrize("order", [(0, 1, 2, 3, 4, 5, 6), (3, 4, 5, 0, 1, 2, 6)])
def test_enumerated_sweep_distribution_matches_monte_carlo(order):
    alpha, beta, vbeta = 0.3, 0.05, 1.0
    prob = C.exact_sweep_distribution(order, alpha, beta, vbeta)
    assert abs(prob.sum() - 1.0) < 1e-12
    codes = _simulate(order, 200_000, alpha, beta, vbeta, np.random.default_rng(7))
    hist = np.bincount(codes, minlength=prob.size).astype(np.float64)
    chi2, df = C._chi2(hist, prob)
    assert chi2 < df + 6 * (2 * df) ** 0.5 + 10, (chi2, df)


def test_token_order_matters():
    """The two chunk orders give different distributions (so the GPU test must, and does,
    pair each replica with the order its descriptors produced)."""
    a = C.exact_sweep_distribution((0, 1, 2, 3, 4, 5, 6), 0.3, 0.05, 1.0)
    b = C.exact_sweep_distribution((3, 4, 5, 0, 1, 2, 6), 0.3, 0.05, 1.0)
    assert np.abs(a - b).max() > 1e-3
