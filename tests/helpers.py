"""Shared test helpers: instances, dense reconstructions of the constraint matrices, metrics."""
import math

import numpy as np


def dense_A(cl, bi, j, t_idx):
    """Dense block-diagonal (list over l) constraint matrix A_{j,(r,s,k)} (MPMP.jl:385-386)."""
    m, N = bi.m[j], bi.n_samples[j]
    loc = t_idx
    k = loc % N
    rs = loc // N
    r = 0
    while (r + 1) * (r + 2) // 2 <= rs:
        r += 1
    s = rs - r * (r + 1) // 2
    E = np.zeros((m, m))
    if r == s:
        E[r, r] = 1.0
    else:
        E[r, s] = E[s, r] = 0.5
    out = []
    for l in range(bi.L[j]):
        d = bi.Y_blocksizes[j][l] // m
        W = np.zeros((d, d))
        for v, lam in zip(cl.A[l][k], cl.H[l][k]):
            v = np.asarray(v, dtype=float)
            W += float(lam) * np.outer(v, v)
        out.append(np.kron(E, W))
    return out


def rand_spd(n, rng, shift=1.0):
    G = rng.standard_normal((n, n))
    return G @ G.T / n + shift * np.eye(n)


def rel_err(a, b, scale=0.0):
    """max|a-b| / max(max|b|, scale); exact (mpmath) when either side holds mpf objects."""
    a = np.asarray(a).ravel()
    b = np.asarray(b).ravel()
    if a.size == 0:
        return 0.0
    if a.dtype == object or b.dtype == object:
        import mpmath
        num = max(abs(mpmath.mpf(x) - mpmath.mpf(y)) for x, y in zip(a, b))
        den = max([abs(mpmath.mpf(y)) for y in b] + [mpmath.mpf(scale), mpmath.mpf(1e-300)])
        return float(num / den)
    a = a.astype(float)
    b = b.astype(float)
    return float(np.max(np.abs(a - b)) / max(1e-300, float(np.max(np.abs(b))), scale))


def poly_min_instance(pk, coef=(2.0, 1.0, -3.0, 0.0, 1.0)):
    """max y s.t. p(x) - y is a sum of squares (univariate): optimum = min_x p(x).
    One cluster, m = 1, v_k = (1, x_k, x_k^2), lambda = 1, B = 1, c_k = p(x_k), b = 1."""
    N = len(coef)
    deg = (len(coef) - 1) // 2
    xs = np.cos(np.pi * (2 * np.arange(N) + 1) / (2 * N)) * 2.0
    A = [[[np.array([x ** i for i in range(deg + 1)])] for x in xs]]
    H = [[[1.0] for _ in xs]]
    B = np.ones((N, 1))
    c = np.array([np.polyval(list(coef)[::-1], x) for x in xs])
    dcoef = [i * coef[i] for i in range(1, len(coef))]
    r = np.roots(dcoef[::-1])
    r = r[np.abs(r.imag) < 1e-12].real
    pmin = float(min(np.polyval(list(coef)[::-1], r)))
    return [pk.Cluster(A, B, c, H)], np.array([1.0]), pmin


CONFIGS_SMALL = [
    dict(J=2, delta=4, rank=1, n_y=4),                    # C1
    dict(J=2, delta=3, rank=1, n_y=3, m=2, L=2),          # polynomial-matrix clusters, 2 blocks
    dict(J=3, delta=4, rank=2, n_y=5),                    # rank 2
    dict(J=3, delta=5, rank=1, n_y=4, m=3, L=2),          # m = 3
    dict(J=1, delta=6, rank=1, n_y=1),                    # single cluster, n_y = 1
]
