"""Problem data: the reference's constraint tuples, synthetic instances, and the flat C-ABI layout.

A cluster is the ``(A, B, c, H)`` tuple returned by ``prepareabc`` (MPMP.jl:385-406):

* ``A[l][k][rnk]`` -- vector v_{j,l,k,rnk} (length delta_jl),
* ``H[l][k][rnk]`` -- its eigenvalue lambda (``A_sign``),
* ``B`` -- dim_S x n_y matrix, ``c`` -- dim_S vector, tuples ordered (r, s<=r, k) (MPMP.jl:390-398).

Values are numpy float64 arrays, or (for multi-word runs) numpy object arrays of
``mpmath.mpf``; :func:`to_planes` splits them exactly into planar limbs for the C ABI.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np


@dataclass
class Cluster:
    A: list
    B: np.ndarray
    c: np.ndarray
    H: list

    # tuple-compatible access, as constraints[j][1..4] in MPMP.jl (0-based here)
    def __getitem__(self, i):
        return (self.A, self.B, self.c, self.H)[i]


# ---------------------------------------------------------------------------------------------
# deterministic counter-based RNG (splitmix64), so instances are identical everywhere
# ---------------------------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, stream: int, n: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """n uniforms in [lo, hi) from counter (seed, stream, i)."""
    with np.errstate(over="ignore"):
        base = _splitmix64(np.array([(seed * 0x100000001B3 + stream * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF],
                                    dtype=np.uint64))[0]
        z = _splitmix64(base + np.arange(n, dtype=np.uint64))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return lo + (hi - lo) * u


def synth(J: int, delta: int, rank: int, n_y: int, seed: int = 0, m: int = 1, L: int = 1,
          N: int | None = None, kind: str = "random", ranks=None) -> tuple:
    """Synthetic clustered low-rank SDP, strictly primal and dual feasible.

    m x m polynomial-matrix clusters, L blocks each, N = 2 delta - 1 samples (default), ``rank``
    vectors per sample (or an explicit ``ranks[l][k]`` list).  v ~ U[-1,1)/sqrt(delta) (``kind =
    "random"``) or Chebyshev polynomials at Chebyshev nodes (``"poly"``); lambda ~ U[0.5, 1.5);
    B ~ U[-1, 1).  With x0 = 1, X0 = sum_i A_i > 0 and b = B^T x0; with Y0 = I, y0 ~ U[-1,1),
    c = Tr(A_i) + B y0.  Returns ``(constraints, b)``.
    """
    if N is None:
        N = 2 * delta - 1
    cons = []
    xs = []
    for j in range(J):
        A, H = [], []
        for l in range(L):
            Al, Hl = [], []
            for k in range(N):
                rk = rank if ranks is None else ranks[l][k]
                st = ((j * 131 + l) * 65537 + k) * 17
                if kind == "poly":
                    xk = math.cos(math.pi * (2 * k + 1) / (2 * N))
                    vk = np.polynomial.chebyshev.chebvander(np.array([xk]), delta - 1)[0]
                    vs = [vk * (1.0 + 0.1 * uniform(seed, st + q, delta)) / math.sqrt(delta)
                          for q in range(rk)]
                else:
                    vs = [uniform(seed, st + q, delta) / math.sqrt(delta) for q in range(rk)]
                lam = list(uniform(seed, st + 7919, max(rk, 1), 0.5, 1.5)[:rk])
                Al.append(vs)
                Hl.append(lam)
            A.append(Al)
            H.append(Hl)
        D = m * (m + 1) // 2 * N
        B = uniform(seed, 10_000_019 + j, D * n_y).reshape(n_y, D).T.copy()
        # c = Tr(A_i Y0) + B y0 with Y0 = I:  Tr(E_rs (x) W) = delta_rs Tr(W)
        c = np.zeros(D)
        for r in range(m):
            s = r
            for k in range(N):
                t = k + (s + r * (r + 1) // 2) * N
                c[t] = sum(lam * float(v @ v) for l in range(L) for v, lam in zip(A[l][k], H[l][k]))
        cons.append(Cluster(A, B, c, H))
        xs.append(np.ones(D))
    y0 = uniform(seed, 77_777_777, n_y)
    b = np.zeros(n_y)
    for cl, x0 in zip(cons, xs):
        cl.c = cl.c + cl.B @ y0
        b = b + cl.B.T @ x0
    return cons, b


def synth_mixed(specs, n_y: int, seed: int = 0) -> tuple:
    """Synthetic instance with per-cluster shapes: ``specs[j] = dict(m=, deltas=[delta_l...],
    N=, ranks=None or ranks[l][k])``.  Same construction (and feasibility) as :func:`synth`.
    The sphere-packing shape of BASELINE config 5 is :data:`SPHERE_PACKING_SHAPE`."""
    cons, xs = [], []
    for j, sp in enumerate(specs):
        m, deltas, N = sp["m"], sp["deltas"], sp["N"]
        A, H = [], []
        for l, delta in enumerate(deltas):
            Al, Hl = [], []
            for k in range(N):
                rk = 1 if sp.get("ranks") is None else sp["ranks"][l][k]
                st = ((j * 131 + l) * 65537 + k) * 17 + 3
                Al.append([uniform(seed, st + q, delta) / math.sqrt(delta) for q in range(rk)])
                Hl.append(list(uniform(seed, st + 7919, max(rk, 1), 0.5, 1.5)[:rk]))
            A.append(Al)
            H.append(Hl)
        D = m * (m + 1) // 2 * N
        B = uniform(seed, 10_000_019 + j, D * n_y).reshape(n_y, D).T.copy()
        c = np.zeros(D)
        for r in range(m):
            for k in range(N):
                t = k + (r + r * (r + 1) // 2) * N
                c[t] = sum(lam * float(v @ v) for l in range(len(deltas))
                           for v, lam in zip(A[l][k], H[l][k]))
        cons.append(Cluster(A, B, c, H))
        xs.append(np.ones(D))
    y0 = uniform(seed, 77_777_777, n_y)
    b = np.zeros(n_y)
    for cl, x0 in zip(cons, xs):
        cl.c = cl.c + cl.B @ y0
        b = b + cl.B.T @ x0
    return cons, b


def synth_C(bi, seed: int, scale: float = 0.125) -> list:
    """A nonzero constant matrix C (the ``C`` keyword of solverank1sdp, MPMP.jl:599, 691-695) in
    the block structure of X: per (j,l) a symmetric matrix with entries scale * U[-1,1) (lower
    triangle drawn, mirrored, so C is exactly symmetric)."""
    out = []
    q = 0
    for j, bj in enumerate(bi.Y_blocksizes):
        row = []
        for n in bj:
            u = uniform(seed, 900_001 + q, n * n).reshape(n, n) * scale
            Cb = np.tril(u) + np.tril(u, -1).T
            row.append(Cb)
            q += 1
        out.append(row)
    return out


def synth_start(bi, seed: int) -> tuple:
    """A seeded interior start point (x, X, y, Y) for ``initial_solutions`` (MPMP.jl:613,
    687-689): X, Y = diagonal in [1, 3) plus a symmetric perturbation below 1/(4n) per entry
    (strictly diagonally dominant, so positive definite); x, y ~ U[-1/2, 1/2)."""
    def spd(stream, n):
        d = uniform(seed, stream, n, 1.0, 3.0)
        u = uniform(seed, stream + 1, n * n, -1.0, 1.0).reshape(n, n) / (4.0 * n)
        return np.diag(d) + np.tril(u, -1) + np.tril(u, -1).T
    nx = sum(bi.dim_S)
    x = uniform(seed, 810_001, nx, -0.5, 0.5)
    y = uniform(seed, 810_003, bi.n_y, -0.5, 0.5)
    X, Y = [], []
    q = 0
    for bj in bi.Y_blocksizes:
        X.append([spd(820_001 + 4 * (q + l), n) for l, n in enumerate(bj)])
        Y.append([spd(830_001 + 4 * (q + l), n) for l, n in enumerate(bj)])
        q += len(bj)
    return x, X, y, Y


# Block structure of the sphere-packing instance of examples/SpherePacking.jl (n = 3, d = 8,
# N = 2 radii; SP.jl:56-105): J = 7 clusters, blocks {2}, {18, 16}, {9, 8} x 3, {1} x 2,
# dim_S = {3, 51, 17, 17, 17, 1, 1}, n_y = 52 (SURVEY.md §8 "C5").
SPHERE_PACKING_SHAPE = dict(
    specs=[dict(m=2, deltas=[1], N=1), dict(m=2, deltas=[9, 8], N=17)]
    + [dict(m=1, deltas=[9, 8], N=17)] * 3 + [dict(m=1, deltas=[1], N=1)] * 2,
    n_y=52)


# ---------------------------------------------------------------------------------------------
# flat C-ABI layout (include/clrsdp.h)
# ---------------------------------------------------------------------------------------------
def to_planes(values, words: int) -> np.ndarray:
    """Split values (float64 array or object array of mpmath.mpf) into ``words`` planar limbs."""
    vals = np.asarray(values).reshape(-1)
    if words == 1 or vals.dtype != object:
        out = np.zeros(words * vals.size)
        out[:vals.size] = np.asarray(vals, dtype=np.float64) if vals.dtype != object else \
            np.array([float(v) for v in vals])
        return out
    import mpmath
    out = np.zeros((words, vals.size))
    for i, v in enumerate(vals):
        # exact remainders (independent of mpmath.mp.prec): limb w is the nearest double of
        # what the previous limbs leave over
        if isinstance(v, mpmath.mpf):
            r = v
        else:  # strings, lazy constants (mpmath.pi): convert well beyond 4 limbs
            with mpmath.workprec(1024):
                r = mpmath.mpf(v)
        for w in range(words):
            h = float(r)
            out[w, i] = h
            r = mpmath.fsub(r, h, exact=True)
    return out.reshape(-1)


def from_planes(planes: np.ndarray, n: int, words: int) -> np.ndarray:
    """Inverse of :func:`to_planes`: the exact sums of the limbs as ``mpmath.mpf``."""
    import mpmath
    P = np.asarray(planes).reshape(words, -1)
    out = np.empty(n, dtype=object)
    for i in range(n):
        s = mpmath.mpf(0)
        for q in range(words):
            s = mpmath.fadd(s, float(P[q, i]), exact=True)
        out[i] = s
    return out


@dataclass
class Flat:
    """Constraint data in the layout of clrsdp_upload_constraints."""

    J: int
    n_y: int
    m: np.ndarray
    L: np.ndarray
    n_samples: np.ndarray
    delta: np.ndarray
    ranks: np.ndarray
    V: list          # per (j,l) delta x K column-major (as values, possibly object)
    lam: list        # per (j,l) K values
    B: list          # per j D x n_y (column-major when flattened with order='F')
    c: list
    block_sizes: list  # per (j,l) n = m delta


def flatten(constraints: Sequence, bi) -> Flat:
    J = bi.J
    delta, ranks, V, lam, Bs, cs, nbs = [], [], [], [], [], [], []
    for j in range(J):
        cl = constraints[j]
        for l in range(bi.L[j]):
            nz = bi.nz_k[j][l]
            d = len(cl.A[l][nz][0])
            delta.append(d)
            cols, lv = [], []
            for k in range(bi.n_samples[j]):
                ranks.append(len(cl.A[l][k]))
                for rnk, v in enumerate(cl.A[l][k]):
                    cols.append(np.asarray(v))
                    lv.append(cl.H[l][k][rnk])
            Vm = np.stack(cols, axis=1)
            V.append(Vm)
            lam.append(np.array(lv, dtype=Vm.dtype))
            nbs.append(bi.m[j] * d)
        Bs.append(np.asarray(cl.B))
        cs.append(np.asarray(cl.c))
    return Flat(J, bi.n_y, np.array(bi.m, dtype=np.int64), np.array(bi.L, dtype=np.int64),
                np.array(bi.n_samples, dtype=np.int64), np.array(delta, dtype=np.int64),
                np.array(ranks, dtype=np.int64), V, lam, Bs, cs, nbs)


def concat_colmajor(mats) -> np.ndarray:
    parts = [np.asarray(M).reshape(-1, order="F") for M in mats]
    if not parts:
        return np.zeros(0)
    if any(p.dtype == object for p in parts):
        return np.concatenate([p.astype(object) for p in parts])
    return np.concatenate(parts)


def blocks_to_flat(blocks) -> np.ndarray:
    """[[X_jl]] -> concatenated column-major blocks (the CLRSDP_BUF_X layout)."""
    return concat_colmajor([b for bj in blocks for b in bj])


def flat_to_blocks(flat: np.ndarray, bi) -> list:
    out, off = [], 0
    for j in range(bi.J):
        bj = []
        for l in range(bi.L[j]):
            n = bi.Y_blocksizes[j][l]
            bj.append(np.asarray(flat[off:off + n * n]).reshape(n, n, order="F"))
            off += n * n
        out.append(bj)
    return out
