"""Symmetric tridiagonal eigen-decomposition by divide and conquer -- the host reference
of the device kernels in ``csrc/eig.hip`` (same tree, deflation, root finder and Loewner
vectors, step for step), used as their oracle in the tests.

Tree: the index range [0, n) is split at its midpoint recursively down to 1 x 1 leaves;
split point m of a range couples T1 = T[lo:m] and T2 = T[m:hi] through beta = e[m - 1]:

    T = diag(T1 - |beta| e_last e_last^T, T2 - |beta| e_1 e_1^T) + |beta| u u^T,
    u = [e_last; sign(beta) e_1]

so every split subtracts |beta| from d[m - 1] and d[m] once, leaves are the modified
diagonal, and a merge of solved halves (Q1, D1), (Q2, D2) is the rank-one problem
D + rho z z^T with z = Q^T u / |Q^T u|, rho = |beta| |Q^T u|^2 (Cuppen). Merges of one
tree level are independent.

Merge (LAPACK dlaed2 / dlaed3 / dlaed4 semantics, re-derived):
 * sort the 2 halves' eigenvalues (rank by counting; ties by index);
 * deflation with tol = 8 eps max(max|d|, rho max|z|): rho |z_j| <= tol keeps (d_j, q_j);
   two surviving neighbours whose rotation (c, s) zeroing z_pj has |(d_j - d_pj) c s| <= tol
   are rotated (columns of Q too) and pj is kept with d_pj c^2 + d_j s^2;
 * the k surviving (d, z): root i of 1/rho + sum z_j^2 / (d_j - lambda) = 0 in
   (d_i, d_{i+1}) (the last in (d_{k-1}, d_{k-1} + rho |z|^2]) is found in coordinates
   shifted to its nearer pole (lambda = d_o + tau), by a two-pole rational model step
   (Bunch-Nielsen-Sorensen fixed weight) safeguarded by a bisection bracket;
 * z is recomputed from the roots (Gu-Eisenstat / Loewner), so the vectors
   u_i[j] = zhat_j / (d_j - lambda_i) are orthogonal to working precision whatever the
   root error; Q_new = Q_perm[:, :k] U.

Reference: the DAAL PCA correlation step (eigenvalues AND eigenvectors),
ml/daal/src/main/java/edu/iu/daal_pca/cordensedistr/PCADaalCollectiveMapper.java:136-154.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np

EPS = 2.220446049250313e-16


def tree_levels(n: int) -> List[List[Tuple[int, int, int]]]:
    """Merges per level, bottom level first: (lo, mid, hi) with halves [lo, mid), [mid, hi)."""
    levels: List[List[Tuple[int, int, int]]] = []

    def rec(lo: int, hi: int, depth: int) -> None:
        if hi - lo <= 1:
            return
        mid = (lo + hi) // 2
        rec(lo, mid, depth + 1)
        rec(mid, hi, depth + 1)
        while len(levels) <= depth:
            levels.append([])
        levels[depth].append((lo, mid, hi))

    rec(0, n, 0)
    return levels[::-1]


def secular_root(i: int, dd: np.ndarray, z: np.ndarray, rho: float, max_iter: int = 64) -> Tuple[int, float, int]:
    """Root i (0-based) of 1/rho + sum z_j^2 / (d_j - lambda) for ascending dd, rho > 0.
    Returns (origin index o, tau, iterations) with lambda = dd[o] + tau."""
    k = dd.size
    zz = z * z
    if i < k - 1:
        gap = dd[i + 1] - dd[i]
        mid = 0.5 * gap
        f = 1.0 / rho + np.sum(zz / ((dd - dd[i]) - mid))
        if f >= 0.0:
            o, lo, hi = i, 0.0, mid
        else:
            o, lo, hi = i + 1, -mid, 0.0
    else:
        o = i
        lo, hi = 0.0, rho * float(np.sum(zz))
    delta = dd - dd[o]
    tau = 0.5 * (lo + hi)
    it = 0
    for it in range(1, max_iter + 1):
        D = delta - tau
        t = zz / D
        left = t[: i + 1]
        right = t[i + 1:]
        psi, phi = left.sum(), right.sum()
        dpsi = (left / D[: i + 1]).sum()
        dphi = (right / D[i + 1:]).sum() if right.size else 0.0
        f = 1.0 / rho + psi + phi
        erretm = 2.0 * EPS * (1.0 / rho + abs(psi) + abs(phi))
        if abs(f) <= erretm or hi - lo <= 2.0 * EPS * max(abs(lo), abs(hi)):
            break
        if f < 0.0:
            lo = tau
        else:
            hi = tau
        D1 = D[i]
        b1 = dpsi * D1 * D1
        c = 1.0 / rho + (psi - b1 / D1)
        if i < k - 1:
            D2 = D[i + 1]
            b2 = dphi * D2 * D2
            c += phi - b2 / D2
            # c eta^2 - B eta + D1 D2 f = 0
            B = c * (D1 + D2) + b1 + b2
            C = D1 * D2 * f
            disc = max(B * B - 4.0 * c * C, 0.0)
            sq = math.sqrt(disc)
            cands = []
            if c != 0.0:
                q = 0.5 * (B + math.copysign(sq, B))
                if q != 0.0:
                    cands = [q / c, C / q]
            elif B != 0.0:
                cands = [C / B]
        else:
            c += phi
            cands = [D1 + b1 / c] if c != 0.0 else []
        eta = None
        for cand in cands:
            nt = tau + cand
            if math.isfinite(nt) and lo < nt < hi:
                if eta is None or abs(cand) < abs(eta):
                    eta = cand
        if eta is None:
            tau = 0.5 * (lo + hi)
        else:
            tau = tau + eta
            if abs(eta) <= 2.0 * EPS * abs(tau):
                break
    return o, tau, it


def merge(d: np.ndarray, Q: np.ndarray, lo: int, mid: int, hi: int, beta: float) -> dict:
    """Merge the solved halves of [lo, hi) in place (d[lo:hi] eigenvalues, Q[lo:hi, lo:hi]
    block); returns diagnostics."""
    s = hi - lo
    blk = Q[lo:hi, lo:hi]
    dv = d[lo:hi].copy()
    zr = np.concatenate([blk[mid - lo - 1, : mid - lo], math.copysign(1.0, beta) * blk[mid - lo, mid - lo:]])
    # rank by counting (ties by index): the merged ascending order
    key = np.lexsort((np.arange(s), dv))
    dv, zr = dv[key], zr[key]
    cols = blk[:, key].copy()
    nz = float(np.sqrt(np.sum(zr * zr)))
    rho = abs(beta) * nz * nz
    if rho == 0.0:
        blk[:, :] = cols
        d[lo:hi] = dv
        return {"k": 0}
    z = zr / nz
    tol = 8.0 * EPS * max(float(np.max(np.abs(dv))), rho * float(np.max(np.abs(z))))
    keep = []  # surviving positions (ascending)
    defl = []
    pj = -1
    for j in range(s):
        if rho * abs(z[j]) <= tol:
            defl.append(j)
            continue
        if pj < 0:
            pj = j
            continue
        ss, cc = z[pj], z[j]
        tau = math.hypot(cc, ss)
        t = dv[j] - dv[pj]
        cc, ss = cc / tau, -ss / tau
        if abs(t * cc * ss) <= tol:
            z[j], z[pj] = tau, 0.0
            x, y = cols[:, pj].copy(), cols[:, j].copy()
            cols[:, pj] = cc * x + ss * y
            cols[:, j] = cc * y - ss * x
            tt = dv[pj] * cc * cc + dv[j] * ss * ss
            dv[j] = dv[pj] * ss * ss + dv[j] * cc * cc
            dv[pj] = tt
            defl.append(pj)
            pj = j
        else:
            keep.append(pj)
            pj = j
    if pj >= 0:
        keep.append(pj)
    k = len(keep)
    dd, zz = dv[keep], z[keep]
    org = np.zeros(k, dtype=np.int64)
    taus = np.zeros(k)
    iters = 0
    for i in range(k):
        o, t_, it = secular_root(i, dd, zz, rho)
        org[i], taus[i] = o, t_
        iters = max(iters, it)
    # Loewner: zhat_j^2 = (lambda_j - d_j)/rho * prod_{i != j} (lambda_i - d_j) / (d_i - d_j)
    zh = np.zeros(k)
    for j in range(k):
        p = ((dd[org[j]] - dd[j]) + taus[j]) / rho
        for i in range(k):
            if i != j:
                p *= ((dd[org[i]] - dd[j]) + taus[i]) / (dd[i] - dd[j])
        zh[j] = math.copysign(math.sqrt(max(p, 0.0)), zz[j])
    U = np.zeros((k, k))
    for i in range(k):
        u = zh / ((dd - dd[org[i]]) - taus[i])
        U[:, i] = u / np.linalg.norm(u)
    newcols = np.empty_like(cols)
    newcols[:, :k] = cols[:, keep] @ U
    newcols[:, k:] = cols[:, sorted(defl)]
    lam = np.concatenate([dd[org] + taus, dv[sorted(defl)]])
    blk[:, :] = newcols
    d[lo:hi] = lam
    return {"k": k, "iters": iters}


def eigh_tridiag(d: np.ndarray, e: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Eigenvalues (ascending) and eigenvectors of the symmetric tridiagonal (d, e)."""
    d = np.asarray(d, dtype=np.float64).copy()
    e = np.asarray(e, dtype=np.float64)
    n = d.size
    levels = tree_levels(n)
    for lev in levels:
        for (lo, mid, hi) in lev:
            b = abs(e[mid - 1])
            d[mid - 1] -= b
            d[mid] -= b
    Q = np.eye(n)
    for lev in levels:
        for (lo, mid, hi) in lev:
            merge(d, Q, lo, mid, hi, float(e[mid - 1]))
    order = np.argsort(d, kind="stable")
    return d[order], Q[:, order]
