"""Host model of the chip-wide tridiagonalisation of csrc/eig_ll.hip, step for step: the
column x' is the only per-column state, v = scl x' + gam e_{k+1} is affine in it so the
Householder norm, the panel dots and the row dots all come from ONE reduction over x', p is
formed per block of RW rows from the panel-start matrix plus the deferred corrections, and the
panel-start matrix is only updated every NBP columns. Checked against LAPACK (numpy) so the
formulas the kernel implements are pinned on the CPU."""
import numpy as np
import pytest


def sytrd_ll_model(A, nbp=4, rw=8):
    n = A.shape[0]
    Aps = A.copy()
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 1))
    Vt = np.zeros((n, n))
    tau_out = np.zeros(n)
    Vp = np.zeros((n, nbp))
    Wp = np.zeros((n, nbp))
    x = np.zeros(n)
    x[1:] = A[1:, 0]
    d[0] = A[0, 0]
    for k in range(n - 2):
        j = k % nbp
        k1 = k + 1
        alpha = x[k1]
        sigma = float(np.dot(x[k1 + 1:], x[k1 + 1:]))
        # the one reduction: row dots A_ps[r] . x', panel dots W_l . x', V_l . x'
        Q = Aps @ x
        Dw = Wp[:, :j].T @ x
        Dv = Vp[:, :j].T @ x
        if sigma != 0.0:
            beta = -np.copysign(np.sqrt(alpha * alpha + sigma), alpha)
            tau = (beta - alpha) / beta
            scl = 1.0 / (alpha - beta)
            gam = -beta * scl
        else:
            beta, tau, scl, gam = alpha, 0.0, 0.0, 1.0
        v = np.zeros(n)
        v[k1 + 1:] = scl * x[k1 + 1:]
        v[k1] = 1.0
        gW = scl * Dw + gam * Wp[k1, :j]
        gV = scl * Dv + gam * Vp[k1, :j]
        p = np.zeros(n)
        for r0 in range(0, n, rw):  # one workgroup's rows
            for r in range(r0, min(r0 + rw, n)):
                q = scl * Q[r] + gam * Aps[r, k1]
                q -= Vp[r, :j] @ gW + Wp[r, :j] @ gV
                p[r] = tau * q
        p[:k1] = 0.0
        c = 0.5 * tau * float(np.dot(p, v))
        w = p - c * v
        Vp[:, j] = v
        Wp[:, j] = w
        Vt[k] = v
        tau_out[k] = tau
        e[k] = beta
        xn = Aps[:, k1] - Vp[:, :j + 1] @ Wp[k1, :j + 1] - Wp[:, :j + 1] @ Vp[k1, :j + 1]
        d[k1] = xn[k1]
        if k + 3 >= n:
            e[n - 2] = xn[n - 1]
            d[n - 1] = Aps[n - 1, n - 1] - 2.0 * float(Vp[n - 1, :j + 1] @ Wp[n - 1, :j + 1])
            break
        x = np.zeros(n)
        x[k1 + 1:] = xn[k1 + 1:]
        if j == nbp - 1:
            Aps -= Vp @ Wp.T + Wp @ Vp.T
            Vp[:] = 0.0
            Wp[:] = 0.0
    if n == 2:
        e[0] = A[1, 0]
        d[1] = A[1, 1]
    return d, e[:max(n - 1, 0)], Vt, tau_out


def _q_from_reflectors(Vt, tau):
    n = Vt.shape[0]
    Q = np.eye(n)
    for k in range(n - 2):
        v = Vt[k]
        Q = Q @ (np.eye(n) - tau[k] * np.outer(v, v))
    return Q


@pytest.mark.parametrize("n,nbp", [(3, 4), (4, 4), (5, 2), (9, 4), (17, 4), (40, 4), (64, 3), (71, 4)])
def test_model_reproduces_the_matrix(n, nbp):
    rng = np.random.default_rng(n)
    M = rng.standard_normal((n, n))
    A = (M + M.T) / 2
    d, e, Vt, tau = sytrd_ll_model(A, nbp=nbp)
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    Q = _q_from_reflectors(Vt, tau)
    assert np.abs(Q.T @ Q - np.eye(n)).max() < 1e-13
    assert np.abs(Q @ T @ Q.T - A).max() < 1e-12 * max(1.0, np.abs(A).max()) * n
    assert np.abs(np.linalg.eigvalsh(T) - np.linalg.eigvalsh(A)).max() < 1e-12 * n


def test_model_degenerate_columns():
    """Already-tridiagonal and diagonal inputs take the tau = 0 path."""
    n = 30
    T0 = np.diag(np.arange(n, dtype=float)) + np.diag(np.ones(n - 1), 1) + np.diag(np.ones(n - 1), -1)
    for A in (T0, np.diag(np.arange(n, dtype=float)), 3.0 * np.eye(n)):
        d, e, Vt, tau = sytrd_ll_model(A)
        T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
        assert np.abs(np.linalg.eigvalsh(T) - np.linalg.eigvalsh(A)).max() < 1e-12
