"""Two-stage symmetric tridiagonalisation: host (numpy) reference.

Stage 1 (sy2sb): dense -> band of half-bandwidth ``b`` by panel QR + two-sided compact-WY
updates (one panel of b columns per step instead of one column). Stage 2 (sb2st): band ->
tridiagonal by bulge chasing, one Householder reflector of length <= b per step. The
eigenvector back-transform applies the stage-2 reflectors (in reverse order) and then the
stage-1 reflectors. This module is the numerical reference for the GPU kernels and the
test oracle; see SURVEY.md §2.8.2 (PCA step 2: eigenvalues and eigenvectors of the
correlation matrix, PCADaalCollectiveMapper.java:136-154).

Status: measured, not the library path. A one-CU HIP bulge chase (band of half-width 8 plus
its bulge resident in LDS, one wave per sweep, 16 sweeps in flight at the minimal safe lag
of 3 steps -- the lag this module's interleaving test establishes) reproduced this
reference (eigenvalue error 3.4e-13 at n = 1000) but took 6.25 ms at n = 1000: ~3n
dependent steps of ~1.6 us each, more than half of the one-stage reduction it was to
replace (profiles/r4_eigh/sb2st_probe.log). The library keeps the one-stage form
(ops.eig.eigh).
"""
from __future__ import annotations

import numpy as np


def householder(x: np.ndarray):
    """v (v[0] = 1), tau, beta with (I - tau v v^T) x = beta e_0 (LAPACK dlarfg)."""
    alpha = float(x[0])
    sig = float(x[1:] @ x[1:]) if x.size > 1 else 0.0
    v = np.zeros_like(x)
    v[0] = 1.0
    if sig == 0.0:
        return v, 0.0, alpha
    beta = -np.copysign(np.sqrt(alpha * alpha + sig), alpha)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def sy2sb(A: np.ndarray, b: int):
    """Band form B = Q1^T A Q1 (half-bandwidth b) and the stage-1 reflectors as a list of
    (row0, v, tau): H = I - tau v v^T acting on rows row0 .. row0 + len(v) - 1, in the order
    applied (Q1 = H_0 H_1 ...)."""
    A = np.array(A, dtype=np.float64, copy=True)
    n = A.shape[0]
    refl = []
    c0 = 0
    while c0 + b < n - 1:
        r0 = c0 + b
        m = n - r0
        P = A[r0:, c0:c0 + b].copy()
        k = min(m, b)
        V = np.zeros((m, k))
        taus = np.zeros(k)
        for i in range(k):
            v, tau, beta = householder(P[i:, i])
            V[i:, i] = v
            taus[i] = tau
            if tau != 0.0:
                P[i:, i:] -= tau * np.outer(v, v @ P[i:, i:])
            P[i, i] = beta
            P[i + 1:, i] = 0.0
        # compact WY: Q = I - V T V^T, T upper (T^-1 = diag(1/tau) + striu(V^T V))
        T = np.zeros((k, k))
        for i in range(k):
            T[i, i] = taus[i]
            if i:
                T[:i, i] = -taus[i] * T[:i, :i] @ (V[:, :i].T @ V[:, i])
        A[r0:, c0:c0 + b] = P
        A[c0:c0 + b, r0:] = P.T
        A22 = A[r0:, r0:]
        X = A22 @ V @ T
        Y = X - 0.5 * V @ (T.T @ (V.T @ X))
        A[r0:, r0:] = A22 - V @ Y.T - Y @ V.T
        for i in range(k):
            refl.append((r0 + i, V[i:, i].copy(), float(taus[i])))
        c0 += b
    return A, refl


def sb2st(B: np.ndarray, b: int):
    """Tridiagonal (d, e) of the band matrix B by bulge chasing, and the stage-2 reflectors
    as (row0, v, tau) in the order applied (B = Q2 T Q2^T, Q2 = H_0 H_1 ...)."""
    B = np.array(B, dtype=np.float64, copy=True)
    n = B.shape[0]
    refl = []
    for s in range(n - 2):
        # step 0: annihilate column s below the subdiagonal
        lo, hi = s + 1, min(s + b, n - 1)
        col = s
        while lo <= n - 1 and hi - lo >= 1:
            v, tau, beta = householder(B[lo:hi + 1, col])
            if tau != 0.0:
                rows = slice(lo, hi + 1)
                cend = min(hi + b, n - 1)
                # B <- H B H with H acting on rows / columns lo..hi: the diagonal block two-sided,
                # the coupled blocks (columns col..lo-1 and hi+1..cend) from the left, mirrored
                D = B[rows, rows]
                p_ = tau * (D @ v)
                w = p_ - 0.5 * tau * (p_ @ v) * v
                B[rows, rows] = D - np.outer(v, w) - np.outer(w, v)
                for c_lo, c_hi in ((col, lo - 1), (hi + 1, cend)):
                    if c_hi < c_lo:
                        continue
                    blk = B[rows, c_lo:c_hi + 1]
                    blk -= tau * np.outer(v, v @ blk)
                    B[c_lo:c_hi + 1, rows] = blk.T
            B[lo, col] = B[col, lo] = beta
            B[lo + 1:hi + 1, col] = 0.0
            B[col, lo + 1:hi + 1] = 0.0
            refl.append((lo, v, tau))
            # the bulge: rows hi+1 .. min(hi+b, n-1) of column lo
            col = lo
            lo, hi = hi + 1, min(hi + b, n - 1)
    d = np.diag(B).copy()
    e = np.diag(B, -1).copy()
    return d, e, refl, B


def apply_reflectors(refl, Z: np.ndarray, reverse: bool = True) -> np.ndarray:
    """Z <- H_0 H_1 ... H_k Z (reverse=True: the last reflector first)."""
    Z = np.array(Z, copy=True)
    seq = reversed(refl) if reverse else refl
    for r0, v, tau in seq:
        if tau == 0.0:
            continue
        rows = slice(r0, r0 + v.size)
        Z[rows] -= tau * np.outer(v, v @ Z[rows])
    return Z


def eigh_two_stage(A: np.ndarray, b: int = 8):
    """Eigenvalues (ascending) and eigenvectors through sy2sb -> sb2st -> tridiagonal eig."""
    B, r1 = sy2sb(A, b)
    d, e, r2, _ = sb2st(B, b)
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    w, Z = np.linalg.eigh(T)
    Z = apply_reflectors(r2, Z)
    Z = apply_reflectors(r1, Z)
    return w, Z

