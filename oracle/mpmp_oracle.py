"""ORACLE -- CPU restatement of MPMP.jl's interior-point step (TEST INFRASTRUCTURE ONLY).

This module is the *checker* for the MI355X path.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product package never does (it fails
loudly when its HIP library is missing instead of falling back to anything here).

What it restates
----------------
``solverank1sdp`` (MPMP.jl:595-1025) and every L2 callee on the hot path, line by line in
meaning, 0-based instead of 1-based:

=====================================  ==========================================
function here                          reference
=====================================  ==========================================
``dot_blocks``                         ``dot(::BlockDiagonal, ...)`` MPMP.jl:205-220
``compute_residual_R``                 ``compute_residual_R!`` MPMP.jl:1189-1215
``xinv``                               X^-1 loop (``spd_inv!``) MPMP.jl:762-801
``compute_S_integrated``               MPMP.jl:1218-1414 (4-term formula 1373-1398)
``compute_T_decomposition``            MPMP.jl:1417-1514 (LU of S_j, LinvB, BTUinv, Q, LU(Q))
``trace_A`` / ``trace_A_AY``           MPMP.jl:1517-1584 / 1585-1618
``compute_weighted_A``                 MPMP.jl:1621-1678
``compute_residuals``                  MPMP.jl:1107-1144 (+ ``calculate_res_d`` 1095-1102)
``compute_search_direction``           MPMP.jl:1682-1824
``compute_step_length``                MPMP.jl:1829-1898
objectives / errors / gap / terminate  MPMP.jl:1026-1092, 1147-1185
``BlockInfo``                          MPMP.jl:467-513 (+ ``distribute_weights_swapping`` 425-465)
``solverank1sdp``                      MPMP.jl:595-1025 (loop 742-954, log columns 700-714/923-937)
=====================================  ==========================================

Arithmetic backends
-------------------
The reference computes with Arb balls at ``precision(BigFloat)`` bits and drops radii with
``get_mid!`` after every heavy product, i.e. it is prec-bit floating point.
``Fp64`` restates it in IEEE binary64 (numpy/scipy: partially pivoted LU for S_j and Q exactly
as ``approx_lu!``; a general eigen-solver on the non-symmetrised L^-1 dM L^-T as
``approx_eig_qr!``).  ``Mp(prec)`` restates it at ``prec`` bits with mpmath numbers in numpy
object arrays and hand-written LU / triangular solves / Cholesky, for the multi-word
(double-double, quad-double) tolerances.

Parity status: UNPINNED
-----------------------
The reference ships no tests, fixtures or golden vectors, and it cannot be run
in this container (no ``julia``, no Arb/FLINT).  This restatement is therefore
anchored only by (i) its line-by-line correspondence to MPMP.jl cited above, (ii) exact algebraic
identities checked in ``tests/test_oracle.py`` (KKT residuals of the block solve, symmetry of S,
S_ij = Tr(A_i X^-1 A_j Y) against a dense brute-force construction), and (iii) known-answer
SDPs whose optimum is known in closed form (``tests/test_oracle.py::test_known_answer_*``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

try:  # scipy is only needed by the fp64 backend
    import scipy.linalg as _sla
except Exception:  # pragma: no cover
    _sla = None

import mpmath


# --------------------------------------------------------------------------------------------
# arithmetic backends
# --------------------------------------------------------------------------------------------
class Fp64:
    """IEEE binary64 backend (numpy arrays of float64)."""

    name = "fp64"
    dtype = np.float64

    def num(self, v):
        return float(v)

    def zeros(self, *shape):
        return np.zeros(shape, dtype=np.float64)

    def eye(self, n):
        return np.eye(n, dtype=np.float64)

    def asarray(self, a):
        return np.asarray(a, dtype=np.float64)

    def lu(self, A):
        """approx_lu!: P A = L U with partial pivoting; returns (LU, perm) s.t. A[perm] = L U."""
        lu, piv = _sla.lu_factor(A, check_finite=False)
        perm = np.arange(A.shape[0])
        for i, p in enumerate(piv):  # LAPACK ipiv -> row permutation
            perm[i], perm[p] = perm[p], perm[i]
        return lu, perm

    def solve_tril(self, L, B, unit):
        return _sla.solve_triangular(L, B, lower=True, unit_diagonal=bool(unit), check_finite=False)

    def solve_triu(self, U, B):
        return _sla.solve_triangular(U, B, lower=False, check_finite=False)

    def inv_spd(self, A):
        c = _sla.cho_factor(A, lower=True, check_finite=False)
        return _sla.cho_solve(c, np.eye(A.shape[0]), check_finite=False)

    def cholesky(self, A):
        return np.linalg.cholesky(A)

    def eigvals_real(self, M):
        """approx_eig_qr! on the (non-symmetrised) matrix; real parts of all eigenvalues."""
        return np.real(np.linalg.eigvals(M))

    def to_float(self, v):
        return float(v)


class Mp:
    """``prec``-bit backend: numpy object arrays of ``mpmath.mpf`` (small instances only)."""

    dtype = object

    def __init__(self, prec: int):
        self.prec = int(prec)
        self.name = f"mp{prec}"
        mpmath.mp.prec = self.prec
        self.zero = mpmath.mpf(0)
        self.one = mpmath.mpf(1)

    def num(self, v):
        if isinstance(v, mpmath.mpf):
            return +v
        if isinstance(v, str):
            return mpmath.mpf(v)
        return mpmath.mpf(v)

    def zeros(self, *shape):
        a = np.empty(shape, dtype=object)
        a.fill(self.zero)
        return a

    def eye(self, n):
        a = self.zeros(n, n)
        for i in range(n):
            a[i, i] = self.one
        return a

    def asarray(self, a):
        a = np.asarray(a, dtype=object)
        out = np.empty(a.shape, dtype=object)
        for idx in np.ndindex(a.shape):
            out[idx] = self.num(a[idx])
        return out

    def lu(self, A):
        n = A.shape[0]
        lu = A.copy()
        perm = list(range(n))
        for k in range(n):
            p = max(range(k, n), key=lambda i: abs(lu[i, k]))
            if lu[p, k] == 0:
                raise np.linalg.LinAlgError("singular matrix in approx_lu")
            if p != k:
                lu[[k, p], :] = lu[[p, k], :]
                perm[k], perm[p] = perm[p], perm[k]
            piv = lu[k, k]
            for i in range(k + 1, n):
                lu[i, k] = lu[i, k] / piv
                f = lu[i, k]
                if f != 0:
                    lu[i, k + 1:] = lu[i, k + 1:] - f * lu[k, k + 1:]
        return lu, np.array(perm)

    def solve_tril(self, L, B, unit):
        B = B.copy()
        vec = B.ndim == 1
        if vec:
            B = B.reshape(-1, 1)
        n = L.shape[0]
        for i in range(n):
            if i:
                B[i, :] = B[i, :] - L[i, :i] @ B[:i, :]
            if not unit:
                B[i, :] = B[i, :] / L[i, i]
        return B.reshape(-1) if vec else B

    def solve_triu(self, U, B):
        B = B.copy()
        vec = B.ndim == 1
        if vec:
            B = B.reshape(-1, 1)
        n = U.shape[0]
        for i in range(n - 1, -1, -1):
            if i < n - 1:
                B[i, :] = B[i, :] - U[i, i + 1:] @ B[i + 1:, :]
            B[i, :] = B[i, :] / U[i, i]
        return B.reshape(-1) if vec else B

    def cholesky(self, A):
        n = A.shape[0]
        L = self.zeros(n, n)
        for j in range(n):
            s = A[j, j] - (L[j, :j] @ L[j, :j] if j else self.zero)
            if s <= 0:
                raise np.linalg.LinAlgError("matrix not positive definite")
            L[j, j] = mpmath.sqrt(s)
            for i in range(j + 1, n):
                t = A[i, j] - (L[i, :j] @ L[j, :j] if j else self.zero)
                L[i, j] = t / L[j, j]
        return L

    def inv_spd(self, A):
        L = self.cholesky(A)
        Linv = self.solve_tril(L, self.eye(A.shape[0]), unit=False)
        return Linv.T @ Linv

    def eigvals_real(self, M):
        # approx_eig_qr! on an AcbMatrix; here the (mathematically symmetric) matrix is
        # symmetrised first so that mpmath's symmetric solver can be used.
        n = M.shape[0]
        S = mpmath.matrix(n, n)
        for i in range(n):
            for j in range(n):
                S[i, j] = (M[i, j] + M[j, i]) / 2
        ev = mpmath.eigsy(S, eigvals_only=True)
        return np.array([ev[i] for i in range(n)], dtype=object)

    def to_float(self, v):
        return float(v)


# --------------------------------------------------------------------------------------------
# problem data and BlockInfo (MPMP.jl:385-406, 467-560)
# --------------------------------------------------------------------------------------------
@dataclass
class Cluster:
    """One polynomial-matrix constraint, the ``(A, B, c, H)`` tuple of ``prepareabc``.

    ``A[l][k][rnk]`` is the vector v_{j,l,k,rnk} (MPMP.jl:385), ``H[l][k][rnk]`` its eigenvalue
    lambda (``A_sign``, MPMP.jl:386), ``B`` the dim_S x n_y matrix and ``c`` the dim_S vector
    (MPMP.jl:387-400), tuples ordered (r, s<=r, k) as MPMP.jl:390-391.
    """

    A: list
    B: np.ndarray
    c: np.ndarray
    H: list


def distribute_weights_swapping(weights, n, nswaps=None):
    """MPMP.jl:425-465 (greedy balance of per-(j,l) weights over ``n`` workers)."""
    w = list(weights)
    if nswaps is None:
        nswaps = len(w) ** 2
    step = len(w) // n + 1
    nstep = n - (step * n - len(w))
    sets = [list(range(i * step, (i + 1) * step)) for i in range(nstep)]
    sets += [list(range(nstep * step + i * (step - 1), nstep * step + (i + 1) * (step - 1)))
             for i in range(n - nstep)]
    set_w = [sum(w[i] for i in s) for s in sets]
    index_set, index_el = 1, 1
    for _ in range(nswaps):
        order = sorted(((set_w[i], i) for i in range(len(set_w))), reverse=True)
        max_set = order[index_set - 1][1]
        els = sorted(((w[sets[max_set][i]], i) for i in range(len(sets[max_set]))), reverse=True)
        max_el = sets[max_set][els[index_el - 1][1]]
        min_set = int(np.argmin(set_w))
        min_el = sets[min_set][int(np.argmin([w[i] for i in sets[min_set]]))]
        if (set_w[min_set] + w[max_el] - w[min_el] < set_w[max_set]
                and set_w[max_set] - w[max_el] + w[min_el] < set_w[max_set]):
            sets[max_set] = [i for i in sets[max_set] if i != max_el] + [min_el]
            set_w[max_set] += w[min_el] - w[max_el]
            sets[min_set] = [i for i in sets[min_set] if i != min_el] + [max_el]
            set_w[min_set] += w[max_el] - w[min_el]
            index_el, index_set = 1, 1
        elif index_el < len(sets[index_set - 1]):
            index_el += 1
        elif index_el == step - 1 and index_set < n - 1:
            index_set += 1
            index_el = 1
        else:
            break
    return sets, set_w


@dataclass
class BlockInfo:
    """MPMP.jl:467-513, 0-based."""

    J: int
    n_y: int
    m: List[int]
    L: List[int]
    n_samples: List[int]
    Y_blocksizes: List[List[int]]
    dim_S: List[int]
    ranks: List[List[List[int]]]
    x_indices: List[int] = field(default_factory=list)
    rank_sums: list = field(default_factory=list)
    nz_k: list = field(default_factory=list)
    jl_pairs: list = field(default_factory=list)

    def __post_init__(self):
        J = self.J
        self.x_indices = [int(sum(self.dim_S[:j])) for j in range(J + 1)]
        self.rank_sums = [[[0] + list(np.cumsum(self.ranks[j][l])) for l in range(self.L[j])]
                          for j in range(J)]
        self.nz_k = [[next(k for k in range(self.n_samples[j]) if self.ranks[j][l][k] > 0)
                      for l in range(self.L[j])] for j in range(J)]
        self.jl_pairs = [(j, l) for j in range(J) for l in range(self.L[j])]

    @property
    def total_dim(self):
        """size(X, 1): sum of all block sizes (MPMP.jl:716)."""
        return int(sum(sum(b) for b in self.Y_blocksizes))


def get_block_info(constraints: Sequence[Cluster]) -> BlockInfo:
    """MPMP.jl:516-560."""
    J = len(constraints)
    n_y = constraints[0].B.shape[1]
    L = [len(c.A) for c in constraints]
    n_samples = [len(c.A[0]) for c in constraints]
    m = [(-1 + math.isqrt(8 * (len(constraints[j].c) // n_samples[j]) + 1)) // 2 for j in range(J)]
    assert all(len(constraints[j].c) == m[j] * (m[j] + 1) * n_samples[j] // 2 for j in range(J))
    ranks = [[[len(constraints[j].A[l][k]) for k in range(n_samples[j])] for l in range(L[j])]
             for j in range(J)]
    nz = [[next(k for k in range(n_samples[j]) if ranks[j][l][k] > 0) for l in range(L[j])]
          for j in range(J)]
    Yb = [[m[j] * len(constraints[j].A[l][nz[j][l]][0]) for l in range(L[j])] for j in range(J)]
    dim_S = [m[j] * (m[j] + 1) // 2 * n_samples[j] for j in range(J)]
    return BlockInfo(J, n_y, m, L, n_samples, Yb, dim_S, ranks)


def tuple_index(r, s, k, N):
    """0-based index of tuple (r, s<=r, k) (MPMP.jl:1340-1348, 1563, 1601, 1653)."""
    return k + (s + r * (r + 1) // 2) * N


# --------------------------------------------------------------------------------------------
# helpers on block-diagonal matrices: X[j][l] is a dense (m_j delta_jl) square matrix
# --------------------------------------------------------------------------------------------
def vectors_matrix(ar, cl: Cluster, l):
    """hcat of all v_{j,l,k,rnk} (MPMP.jl:1249-1254) and the matching lambdas and sample ids."""
    cols, lam, ks = [], [], []
    for k, vk in enumerate(cl.A[l]):
        for rnk, v in enumerate(vk):
            cols.append(v)
            lam.append(cl.H[l][k][rnk])
            ks.append(k)
    V = ar.zeros(len(cols[0]), len(cols))
    for i, v in enumerate(cols):
        V[:, i] = v
    lv = ar.zeros(len(lam))
    for i, x in enumerate(lam):
        lv[i] = x
    return V, lv, np.array(ks, dtype=np.int64)


def dot_blocks(ar, X, Y):
    """dot(::BlockDiagonal, ::BlockDiagonal) MPMP.jl:205-220: sum_ij X_ij Y_ij."""
    s = ar.num(0)
    for Xj, Yj in zip(X, Y):
        for a, b in zip(Xj, Yj):
            s = s + (a * b).sum()
    return s


def block_map(f, *Ms):
    return [[f(*blks) for blks in zip(*js)] for js in zip(*Ms)]


def max_abs_blocks(ar, P):
    """compute_error(::BlockDiagonal) MPMP.jl:1037-1043."""
    m = ar.num(0)
    for Pj in P:
        for b in Pj:
            if b.size:
                m = max(m, np.abs(b).max())
    return m


def max_abs_vec(ar, v):
    """compute_error(::ArbMatrix) MPMP.jl:1045-1055."""
    return max([ar.num(0)] + list(np.abs(v).reshape(-1)))


# --------------------------------------------------------------------------------------------
# L2 kernels
# --------------------------------------------------------------------------------------------
def compute_residual_R(ar, X, Y, mu, dX=None, dY=None):
    """R = mu I - X Y [- dX dY]  (MPMP.jl:1189-1201, 1203-1215)."""
    def one(Xb, Yb, dXb=None, dYb=None):
        R = mu * ar.eye(Xb.shape[0]) - Xb @ Yb
        if dXb is not None:
            R = R - dXb @ dYb
        return R
    if dX is None:
        return block_map(one, X, Y)
    return block_map(one, X, Y, dX, dY)


def xinv(ar, X):
    """X^-1 per (j,l) block with the Cholesky-based spd_inv! (MPMP.jl:762-801)."""
    return block_map(ar.inv_spd, X)


def compute_S_integrated(ar, constraints, X_inv, Y, bi: BlockInfo):
    """Schur complement S_j and A_Y (MPMP.jl:1218-1414).

    Per (j,l): BX = (I_m (x) V)^T X^-1 (I_m (x) V), BY likewise (MPMP.jl:1272-1318); A_Y[r][s] =
    diagonal of BY block (r,s) (1320-1330); S_j[ver,hor] += lambda1 lambda2/4 (4 pairing products)
    for ver <= hor (1335-1399); S_j symmetrised from its upper triangle (1409).
    """
    S, A_Y = [], []
    for j in range(bi.J):
        m, N, D = bi.m[j], bi.n_samples[j], bi.dim_S[j]
        Sj = ar.zeros(D, D)
        AYj = []
        for l in range(bi.L[j]):
            V, lam, ks = vectors_matrix(ar, constraints[j], l)
            delta, K = V.shape
            BX = [[None] * m for _ in range(m)]
            BY = [[None] * m for _ in range(m)]
            Xi, Yb = X_inv[j][l], Y[j][l]
            for s in range(m):
                TX = Xi[:, s * delta:(s + 1) * delta] @ V    # (m delta) x K, MPMP.jl:1291
                TY = Yb[:, s * delta:(s + 1) * delta] @ V    # MPMP.jl:1294
                for r in range(m):
                    BX[r][s] = V.T @ TX[r * delta:(r + 1) * delta, :]   # MPMP.jl:1300
                    BY[r][s] = V.T @ TY[r * delta:(r + 1) * delta, :]   # MPMP.jl:1308
            AYl = [[np.array([BY[r][s][i, i] for i in range(K)], dtype=ar.dtype) for s in range(m)]
                   for r in range(m)]
            AYj.append(AYl)
            # sample-aggregation matrix: column rho belongs to sample ks[rho]
            Pk = ar.zeros(K, N)
            for rho in range(K):
                Pk[rho, ks[rho]] = ar.num(1)
            LL = np.outer(lam, lam) / 4
            for r1 in range(m):
                for s1 in range(r1 + 1):
                    for r2 in range(m):
                        for s2 in range(r2 + 1):
                            # term[rho1, rho2], MPMP.jl:1373-1396
                            T = (BX[s1][r2] * BY[s2][r1].T + BX[r1][r2] * BY[s2][s1].T
                                 + BX[s1][s2] * BY[r2][r1].T + BX[r1][s2] * BY[r2][s1].T)
                            blk = Pk.T @ (LL * T) @ Pk          # [k1, k2]
                            h0 = tuple_index(r1, s1, 0, N)
                            v0 = tuple_index(r2, s2, 0, N)
                            # S[ver, hor] with hor = (r1,s1,k1), ver = (r2,s2,k2)
                            Sj[v0:v0 + N, h0:h0 + N] = Sj[v0:v0 + N, h0:h0 + N] + blk.T
        # keep the upper triangle (ver <= hor) and mirror it: Symmetric(S[j]) MPMP.jl:1409
        iu = np.triu_indices(D)
        Sup = ar.zeros(D, D)
        Sup[iu] = Sj[iu]
        Sj = Sup + Sup.T
        for i in range(D):
            Sj[i, i] = Sup[i, i]
        S.append(Sj)
        A_Y.append(AYj)
    return S, A_Y


@dataclass
class Decomposition:
    S: list          # LU factors of S_j (in place, MPMP.jl:1436)
    perms: list      # row permutations of S_j
    LinvB: list      # L_j^-1 P_j B_j   (MPMP.jl:1463)
    BTUinv: list     # B_j^T U_j^-1     (MPMP.jl:1459-1460)
    perm: np.ndarray  # permutation of Q
    Q: np.ndarray    # LU factors of Q  (MPMP.jl:1501)
    Q_raw: np.ndarray  # Q before factorisation (for stage parity tests)
    S_raw: list      # S_j before factorisation


def compute_T_decomposition(ar, constraints, X_inv, Y, bi: BlockInfo):
    """MPMP.jl:1417-1514."""
    S, A_Y = compute_S_integrated(ar, constraints, X_inv, Y, bi)
    S_raw = [s.copy() for s in S]
    lus, perms = [], []
    for j in range(bi.J):
        lu, perm = ar.lu(S[j])          # approx_lu!  MPMP.jl:1436
        lus.append(lu)
        perms.append(perm)
    LinvB, BTUinv = [], []
    for j in range(bi.J):
        Bj = constraints[j].B
        # U^T W = B  ->  W^T = B^T U^-1  (MPMP.jl:1457-1460)
        W = ar.solve_tril(lus[j].T, Bj, unit=False)
        BTUinv.append(W.T.copy())
        LinvB.append(ar.solve_tril(lus[j], Bj[perms[j], :], unit=True))   # MPMP.jl:1463
    Q = ar.zeros(bi.n_y, bi.n_y)
    for j in range(bi.J):       # MPMP.jl:1467-1494 (summation order: by cluster)
        Q = Q + BTUinv[j] @ LinvB[j]
    Q_raw = Q.copy()
    qlu, qperm = ar.lu(Q)       # MPMP.jl:1501
    return Decomposition(lus, perms, LinvB, BTUinv, qperm, qlu, Q_raw, S_raw), A_Y


def trace_A(ar, constraints, Z, bi: BlockInfo):
    """Tr(A_* Z) for a symmetric block-diagonal Z (MPMP.jl:1517-1584)."""
    res = ar.zeros(sum(bi.dim_S))
    for j in range(bi.J):
        j_idx = bi.x_indices[j]
        N = bi.n_samples[j]
        for l in range(bi.L[j]):
            V, lam, ks = vectors_matrix(ar, constraints[j], l)
            delta = V.shape[0]
            for r in range(bi.m[j]):
                for s in range(r + 1):
                    Zrs = Z[j][l][r * delta:(r + 1) * delta, s * delta:(s + 1) * delta]
                    VZ = V.T @ Zrs                       # MPMP.jl:1558
                    part = (VZ * V.T).sum(axis=1)        # MPMP.jl:1559-1560
                    off = j_idx + (s + r * (r + 1) // 2) * N
                    for rho in range(V.shape[1]):
                        res[off + ks[rho]] = res[off + ks[rho]] + lam[rho] * part[rho]
    return res


def trace_A_AY(ar, constraints, A_Y, bi: BlockInfo):
    """Tr(A_* Y) from the precomputed pairings A_Y (MPMP.jl:1585-1618)."""
    res = ar.zeros(sum(bi.dim_S))
    for j in range(bi.J):
        j_idx = bi.x_indices[j]
        N = bi.n_samples[j]
        for k in range(N):
            for l in range(bi.L[j]):
                rs = bi.rank_sums[j][l]
                for rnk in range(bi.ranks[j][l][k]):
                    for r in range(bi.m[j]):
                        for s in range(r + 1):
                            t = j_idx + tuple_index(r, s, k, N)
                            res[t] = res[t] + constraints[j].H[l][k][rnk] * A_Y[j][l][r][s][rnk + rs[k]]
    return res


def compute_weighted_A(ar, constraints, a, bi: BlockInfo):
    """sum_i a_i A_i as a block-diagonal matrix (MPMP.jl:1621-1678)."""
    out = []
    for j in range(bi.J):
        j_idx = bi.x_indices[j]
        N, m = bi.n_samples[j], bi.m[j]
        blocks = []
        for l in range(bi.L[j]):
            V, lam, ks = vectors_matrix(ar, constraints[j], l)
            delta = V.shape[0]
            M = ar.zeros(m * delta, m * delta)
            for r in range(m):
                for s in range(r + 1):
                    off = j_idx + (s + r * (r + 1) // 2) * N
                    w = np.array([a[off + ks[rho]] * lam[rho] for rho in range(V.shape[1])],
                                 dtype=ar.dtype)
                    Q = (V * w) @ V.T                    # MPMP.jl:1654-1659
                    if r != s:
                        Q = Q / 2                        # MPMP.jl:1661-1663
                    M[s * delta:(s + 1) * delta, r * delta:(r + 1) * delta] = Q
            if m != 1:                                   # Symmetric(.) keeps the upper triangle
                iu = np.triu_indices(m * delta)
                U = ar.zeros(m * delta, m * delta)
                U[iu] = M[iu]
                M = U + U.T
                for i in range(m * delta):
                    M[i, i] = U[i, i]
            blocks.append(M)
        out.append(blocks)
    return out


def stack_B(constraints):
    return np.concatenate([c.B for c in constraints], axis=0)


def stack_c(constraints):
    return np.concatenate([c.c for c in constraints], axis=0)


def compute_residuals(ar, constraints, x, X, y, Y_or_AY, b, C, bi: BlockInfo, use_AY):
    """P = sum x_i A_i - X - C, d = c - Tr(A_* Y) - B y, p = b - B^T x (MPMP.jl:1107-1144)."""
    P = compute_weighted_A(ar, constraints, x, bi)
    P = [[P[j][l] - X[j][l] - (C[j][l] if C is not None else 0) for l in range(bi.L[j])]
         for j in range(bi.J)]
    tr = trace_A_AY(ar, constraints, Y_or_AY, bi) if use_AY else trace_A(ar, constraints, Y_or_AY, bi)
    d = stack_c(constraints) - stack_B(constraints) @ y - tr        # calculate_res_d 1095-1102
    p = ar.zeros(bi.n_y)
    for j in range(bi.J):                                           # MPMP.jl:1129-1139
        xj = x[bi.x_indices[j]:bi.x_indices[j + 1]]
        p = p - constraints[j].B.T @ xj
    p = p + b
    return P, p, d


def sym(Z):
    return (Z + Z.T) / 2


def compute_search_direction(ar, constraints, P, p, d, R, X_inv, Y, bi, dec: Decomposition):
    """MPMP.jl:1682-1824."""
    # Z = sym(X^-1 (P Y - R))  MPMP.jl:1698-1730
    Z = [[sym(X_inv[j][l] @ (P[j][l] @ Y[j][l] - R[j][l])) for l in range(bi.L[j])]
         for j in range(bi.J)]
    rhs_x = -d - trace_A(ar, constraints, Z, bi)                       # MPMP.jl:1733-1739
    idx = bi.x_indices
    temp_x, temp_y = [], []
    for j in range(bi.J):                                              # MPMP.jl:1751-1759
        t = ar.solve_tril(dec.S[j], rhs_x[idx[j]:idx[j + 1]][dec.perms[j]], unit=True)
        temp_x.append(t)
        temp_y.append(dec.BTUinv[j] @ t)
    dy = p.copy()
    acc = ar.zeros(bi.n_y)
    for j in range(bi.J):
        acc = acc + temp_y[j]
    dy = dy - acc                                                      # MPMP.jl:1761
    dy = ar.solve_triu(dec.Q, ar.solve_tril(dec.Q, dy[dec.perm], unit=True))  # MPMP.jl:1764
    dxs = []
    for j in range(bi.J):                                              # MPMP.jl:1771-1773
        dxs.append(ar.solve_triu(dec.S[j], temp_x[j] + dec.LinvB[j] @ dy))
    dx = np.concatenate(dxs) if dxs else ar.zeros(0)
    WA = compute_weighted_A(ar, constraints, dx, bi)                   # MPMP.jl:1779-1786
    dX = [[WA[j][l] + P[j][l] for l in range(bi.L[j])] for j in range(bi.J)]
    dY = [[sym(X_inv[j][l] @ (R[j][l] - dX[j][l] @ Y[j][l])) for l in range(bi.L[j])]
          for j in range(bi.J)]                                         # MPMP.jl:1789-1821
    return dx, dX, dy, dY


def compute_step_length(ar, M, dM, gamma, bi):
    """min(1, -gamma / lambda_min(L^-1 dM L^-T)) over all blocks (MPMP.jl:1829-1898)."""
    min_eig = None
    for j in range(bi.J):
        for l in range(bi.L[j]):
            chol = ar.cholesky(M[j][l])                                 # cho!  MPMP.jl:1846
            LML = ar.solve_tril(chol, dM[j][l], unit=False)             # MPMP.jl:1853
            LML = ar.solve_tril(chol, LML.T.copy(), unit=False)         # MPMP.jl:1854-1856
            ev = ar.eigvals_real(LML)                                   # MPMP.jl:1860-1870
            e = min(ev)
            min_eig = e if min_eig is None else min(min_eig, e)
    if min_eig > -gamma:
        return ar.num(1)
    return -gamma / min_eig


# --------------------------------------------------------------------------------------------
# objectives / errors / termination (MPMP.jl:1026-1185)
# --------------------------------------------------------------------------------------------
def dot_c(ar, constraints, x):
    return (stack_c(constraints) * x).sum() if len(x) else ar.num(0)


def primal_objective(ar, constraints, x, b0):
    return dot_c(ar, constraints, x) + b0


def dual_objective(ar, y, Y, b, C, b0):
    cy = dot_blocks(ar, C, Y) if C is not None else ar.num(0)
    return cy + (b * y).sum() + b0


def duality_gap(ar, pobj, dobj):
    return abs(pobj - dobj) / max(ar.num(1), abs(pobj + dobj))


def terminate(gap, perr, derr, gap_thr, p_thr, d_thr, need_p, need_d):
    gap_opt = gap < gap_thr
    pf = perr < p_thr
    df = derr < d_thr
    if need_p and pf:
        return True
    if need_d and df:
        return True
    return bool(pf and df and gap_opt)


# --------------------------------------------------------------------------------------------
# the driver loop (MPMP.jl:595-1025)
# --------------------------------------------------------------------------------------------
@dataclass
class IterLog:
    iter: int
    mu: object
    p_obj: object
    d_obj: object
    gap: object
    P_err: object
    p_err: object
    d_err: object
    alpha_p: object
    alpha_d: object
    beta: object


@dataclass
class SolveResult:
    x: object
    X: object
    y: object
    Y: object
    P: object
    p: object
    d: object
    gap: object
    p_obj: object
    d_obj: object
    log: list
    status: str


def initial_point(ar, bi: BlockInfo, omega_p, omega_d):
    """x = 0, X = omega_p I, y = 0, Y = omega_d I (MPMP.jl:660-686)."""
    x = ar.zeros(sum(bi.dim_S))
    X = [[ar.num(omega_p) * ar.eye(bi.Y_blocksizes[j][l]) for l in range(bi.L[j])]
         for j in range(bi.J)]
    y = ar.zeros(bi.n_y)
    Y = [[ar.num(omega_d) * ar.eye(bi.Y_blocksizes[j][l]) for l in range(bi.L[j])]
         for j in range(bi.J)]
    return x, X, y, Y


def iteration(ar, constraints, bi, b, C, b0, state, pd_feas, prm):
    """One pass of the loop body MPMP.jl:755-887; returns (new state, dict of intermediates)."""
    x, X, y, Y = state
    dim = bi.total_dim
    mu = dot_blocks(ar, X, Y) / dim                                          # 755
    mu_p = ar.num(0) if pd_feas else prm["beta_infeasible"] * mu             # 756
    R = compute_residual_R(ar, X, Y, mu_p)                                   # 760
    X_inv = xinv(ar, X)                                                      # 763-801
    dec, A_Y = compute_T_decomposition(ar, constraints, X_inv, Y, bi)       # 806
    P, p, d = compute_residuals(ar, constraints, x, X, y, A_Y, b, C, bi, use_AY=True)  # 812
    pred = compute_search_direction(ar, constraints, P, p, d, R, X_inv, Y, bi, dec)    # 818
    dx, dX, dy, dY = pred
    XdX = block_map(lambda a, b_: a + b_, X, dX)
    YdY = block_map(lambda a, b_: a + b_, Y, dY)
    r = dot_blocks(ar, XdX, YdY) / (mu * dim)                                # 832
    beta = r * r if r < 1 else r                                             # 833
    if pd_feas:
        beta_c = min(max(prm["beta_feasible"], beta), ar.num(1))             # 834-836
    else:
        beta_c = max(prm["beta_infeasible"], beta)
    mu_c = beta_c * mu                                                       # 837
    R2 = compute_residual_R(ar, X, Y, mu_c, dX, dY)                          # 841
    corr = compute_search_direction(ar, constraints, P, p, d, R2, X_inv, Y, bi, dec)   # 846
    dx, dX, dy, dY = corr
    alpha_p = compute_step_length(ar, X, dX, prm["gamma"], bi)               # 863-864
    alpha_d = compute_step_length(ar, Y, dY, prm["gamma"], bi)               # 865-866
    if pd_feas:                                                              # 871-874
        alpha_p = min(alpha_p, alpha_d)
        alpha_d = alpha_p
    x = x + alpha_p * dx                                                     # 877
    y = y + alpha_d * dy                                                     # 878
    X = block_map(lambda a, b_: a + alpha_p * b_, X, dX)                     # 881-887
    Y = block_map(lambda a, b_: a + alpha_d * b_, Y, dY)
    inter = dict(mu=mu, mu_p=mu_p, R=R, X_inv=X_inv, dec=dec, A_Y=A_Y, P=P, p=p, d=d,
                 pred=pred, r=r, beta=beta, beta_c=beta_c, mu_c=mu_c, R2=R2, corr=corr,
                 alpha_p=alpha_p, alpha_d=alpha_d)
    return (x, X, y, Y), inter


DEFAULTS = dict(beta_infeasible="0.3", beta_feasible="0.1", gamma="0.7", omega_p="1e10",
                omega_d="1e10", duality_gap_threshold="1e-15", primal_error_threshold="1e-30",
                dual_error_threshold="1e-30")


def _param(ar, v):
    if isinstance(v, str):
        if isinstance(ar, Mp):
            return mpmath.mpf(v)
        return float(v)
    return ar.num(v)


def solverank1sdp(constraints, b, bi: BlockInfo, ar=None, C=None, b0=0, maxiterations=500,
                  need_primal_feasible=False, need_dual_feasible=False, initial_solutions=None,
                  verbose=False, **kw):
    """MPMP.jl:595-1025 (C = 0 is ``None``; the AbsoluteZero trick of MPMP.jl:589-592)."""
    ar = ar or Fp64()
    prm = {k: _param(ar, kw.get(k, v)) for k, v in DEFAULTS.items()}
    b = ar.asarray(b)
    b0 = ar.num(b0)
    if initial_solutions is not None and len(initial_solutions) == 4:
        x, X, y, Y = initial_solutions
    else:
        x, X, y, Y = initial_point(ar, bi, prm["omega_p"], prm["omega_d"])
    alpha_p = alpha_d = ar.num(0)
    p_obj = primal_objective(ar, constraints, x, b0)                           # 723
    d_obj = dual_objective(ar, y, Y, b, C, b0)                                 # 724
    dual_gap = duality_gap(ar, p_obj - b0, d_obj - b0)                         # 725 (no b0)
    P, p, d = compute_residuals(ar, constraints, x, X, y, Y, b, C, bi, use_AY=False)   # 727
    perr = max(max_abs_vec(ar, p), max_abs_blocks(ar, P))                      # 729
    derr = max_abs_vec(ar, d)                                                  # 730
    pd_feas = perr < prm["primal_error_threshold"] and derr < prm["dual_error_threshold"]
    log = []
    it = 1
    status = "maxiterations"
    while True:
        if terminate(dual_gap, perr, derr, prm["duality_gap_threshold"],
                     prm["primal_error_threshold"], prm["dual_error_threshold"],
                     need_primal_feasible, need_dual_feasible):
            status = "terminated"
            break
        if not it < maxiterations:
            break
        (x, X, y, Y), inter = iteration(ar, constraints, bi, b, C, b0, (x, X, y, Y), pd_feas, prm)
        P, p, d = inter["P"], inter["p"], inter["d"]
        row = IterLog(it, inter["mu"], p_obj, d_obj, dual_gap, max_abs_blocks(ar, P),
                      max_abs_vec(ar, p), max_abs_vec(ar, d), inter["alpha_p"], inter["alpha_d"],
                      inter["beta_c"])
        log.append(row)
        if verbose:
            print(format_row(row))
        p_obj = primal_objective(ar, constraints, x, b0)                      # 940
        d_obj = dual_objective(ar, y, Y, b, C, b0)                            # 941
        dual_gap = duality_gap(ar, p_obj, d_obj)                              # 942
        perr = max(max_abs_vec(ar, p), max_abs_blocks(ar, P))                 # 943
        derr = max_abs_vec(ar, d)                                             # 944
        it += 1
        pd_feas = perr < prm["primal_error_threshold"] and derr < prm["dual_error_threshold"]
    final_gap = duality_gap(ar, primal_objective(ar, constraints, x, 0), dual_objective(ar, y, Y, b, C, 0))
    return SolveResult(x, X, y, Y, P, p, d, final_gap, primal_objective(ar, constraints, x, b0),
                       dual_objective(ar, y, Y, b, C, b0), log, status)


def format_row(r: IterLog):
    f = float
    return ("%5d %11.3e %11.3e %11.3e %10.2e %10.2e %10.2e %10.2e %10.2e %10.2e %10.2e" %
            (r.iter, f(r.mu), f(r.p_obj), f(r.d_obj), f(r.gap), f(r.P_err), f(r.p_err),
             f(r.d_err), f(r.alpha_p), f(r.alpha_d), f(r.beta)))
