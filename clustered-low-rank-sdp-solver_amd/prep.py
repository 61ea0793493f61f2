"""Constraint data from polynomial matrix programs: ``prepareabc`` and ``solvempmp``
(MPMP.jl:225-407, 562-586), host side, at arbitrary precision (mpmath).

A polynomial matrix constraint j is  sum_i y_i M[i](x) - M[0](x) = sum_l G[l](x) <Y_l, (q q^T (x) Pi_l)(x)>
(the reference's sampled low-rank form).  ``prepareabc`` evaluates it at the sample points and
returns the cluster tuple ``(A, B, c, H)`` the solver consumes:

* ``A[l][k][r]`` the vector  Pi_vec_r(x_k) (x) q(x_k) sqrt|G_l(x_k)|  (truncated by degree),
* ``H[l][k][r]`` its eigenvalue  Pi_val_r(x_k) sign(G_l(x_k))  (``A_sign``),
* ``B`` rows ``-M[i][r,s](x_k)`` for i >= 1, ``c`` entries ``M[0][r,s](x_k)``, tuples in the
  order (r, s <= r, k).

Values are numpy object arrays of ``mpmath.mpf`` at ``mpmath.mp.prec`` bits (the reference's
``precision(BigFloat)``); the device upload splits them exactly into fp64 limbs.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import mpmath
import numpy as np
from mpmath import mp, mpf

from .instance import Cluster
from .poly import Poly, evaluate, total_degree


def _sign(v) -> int:
    return (v > 0) - (v < 0)


def _mat_entry(Mmat, r: int, s: int):
    """Entry (r, s) of a polynomial matrix given as a nested list or a 2-D object array."""
    return Mmat[r][s]


def _size(Mmat) -> int:
    return len(Mmat)


def _pi_decompositions(Pi, G, x):
    """Eigen-pairs of Pi[l](x_k) through an SVD (MPMP.jl:255-282).

    The reference takes U[:, r] as the vector and ``sign(dot(U[:, r], Vt[:, r])) * S[r]`` as the
    value (GenericSVD's ``Vt``).  mpmath's ``svd_r`` returns A = U diag(S) V with V = Vt, so the
    same expression is ``dot(U[:, r], V[:, r])``, restated literally.
    """
    L, N = len(G), len(x)
    vecs = [[None] * N for _ in range(L)]
    vals = [[None] * N for _ in range(L)]
    for l in range(L):
        P = Pi[l]
        p = _size(P)
        for k in range(N):
            A = mpmath.matrix(p, p)
            for i in range(p):
                for j in range(p):
                    A[i, j] = evaluate(_mat_entry(P, i, j), x[k])
            U, S, V = mpmath.svd_r(A)
            vecs[l][k] = [[U[i, r] for i in range(p)] for r in range(p)]
            vals[l][k] = [_sign(mpmath.fsum(U[i, r] * V[i, r] for i in range(p))) * S[r]
                          for r in range(p)]
    deg_Pi = [max(total_degree(_mat_entry(Pi[l], i, j)) for i in range(_size(Pi[l]))
                  for j in range(_size(Pi[l]))) for l in range(L)]
    deg_Pi_vec = [[total_degree(_mat_entry(Pi[l], i, i)) for i in range(_size(Pi[l]))]
                  for l in range(L)]
    return vecs, vals, deg_Pi, deg_Pi_vec


def _last_degree_index(q: Sequence, half_delta: int) -> List[int]:
    """``last_deg`` (MPMP.jl:284-303), 1-based counts: last_deg[d] = number of leading basis
    polynomials needed for degree <= d.  Missing degrees inherit the previous entry."""
    degs = [total_degree(p) for p in q]
    for i in range(len(degs) - 1):
        if degs[i] > degs[i + 1]:
            print("Degrees are not monotone. The program will (most probably) not be correct "
                  "if you don't fix this")
    last = []
    for d in range(half_delta + 1):
        idx = [i + 1 for i, e in enumerate(degs) if e == d]
        if idx:
            last.append(idx[-1])
        else:
            if d == 0:
                raise ValueError("the basis q has no constant polynomial")
            last.append(last[d - 1])
    return last


def prepareabc(M, G, q, x, delta: int = -1, Pi=None, prec: Optional[int] = None,
               all_of_Pi: bool = True, threshold=None, qp_precomp=None) -> Cluster:
    """Sample one polynomial matrix constraint (MPMP.jl:225-407).

    ``M`` -- list of m x m polynomial matrices (``M[0]`` the constant part, ``M[i]`` the matrix of
    y_i); ``G`` -- list of weight polynomials (one block per entry); ``q`` -- basis polynomials in
    order of degree; ``x`` -- sample points (numbers or coordinate sequences); ``delta`` -- maximum
    degree (negative: twice the degree of ``q[-1]``); ``Pi`` -- optional list of polynomial
    matrices (symmetry blocks); ``qp_precomp[k][d]`` -- optional precomputed ``q[d](x[k])``.
    Entries of M, G, Pi are :class:`Poly` or numbers.  ``prec`` (bits) defaults to
    ``mpmath.mp.prec``.

    Deviations from the shipped reference, both reference bugs: the ``all_of_Pi = false`` branch
    there reads an undefined ``qd_precomp`` (MPMP.jl:323) -- this reads ``qp_precomp``; and
    SpherePacking.jl passes a ``normalize`` keyword prepareabc does not accept (SP.jl:92).
    """
    prec = mp.prec if prec is None else int(prec)
    with mpmath.workprec(prec):
        threshold = mpf(10) ** -70 if threshold is None else mpf(threshold)
        if not isinstance(x, (list, tuple)):
            x = [x]        # a single BigFloat point iterates as one sample (SP.jl:74)
        m = _size(M[0])
        if delta < 0:
            delta = 2 * total_degree(q[-1])
        L, N = len(G), len(x)
        if Pi is None:
            Pi_vecs = [[[[mpf(1)]] for _ in range(N)] for _ in range(L)]
            Pi_vals = [[[mpf(1)] for _ in range(N)] for _ in range(L)]
            deg_Pi = [0] * L
            deg_Pi_vec = [[0] for _ in range(L)]
        else:
            Pi_vecs, Pi_vals, deg_Pi, deg_Pi_vec = _pi_decompositions(Pi, G, x)
        last_deg = _last_degree_index(q, delta // 2)

        def qval(k, d):  # q[d](x[k]), d 0-based
            if qp_precomp is not None:
                return mpf(qp_precomp[k][d])
            return evaluate(q[d], x[k])

        A: List[List[list]] = [[None] * N for _ in range(L)]
        H: List[List[list]] = [[None] * N for _ in range(L)]
        for l in range(L):
            dG = total_degree(G[l])
            for k in range(N):
                g = evaluate(G[l], x[k])
                sg = mpmath.sqrt(abs(g))
                H[l][k] = [mpf(v) * _sign(g) for v in Pi_vals[l][k]]
                vs = []
                for r, pv in enumerate(Pi_vecs[l][k]):
                    if all_of_Pi:
                        # manual Kronecker product: Pi index outer, basis index inner, each Pi
                        # row truncated by its own degree (MPMP.jl:346-378)
                        vec = [pv[pi] * qval(k, d) * sg
                               for pi in range(len(deg_Pi_vec[l]))
                               for d in range(last_deg[(delta - dG - deg_Pi_vec[l][pi]) // 2])]
                    else:
                        # kron(q-part, Pi vector): basis index outer (MPMP.jl:316-345)
                        nd = last_deg[(delta - dG - deg_Pi[l]) // 2]
                        vec = [qval(k, d) * sg * pv[pi] for d in range(nd) for pi in range(len(pv))]
                    vs.append(np.array(vec, dtype=object))
                A[l][k] = vs
        for l in range(L):
            for k in range(N):
                keep = [i for i in range(len(H[l][k])) if abs(H[l][k][i]) > threshold]
                H[l][k] = [H[l][k][i] for i in keep]
                A[l][k] = [A[l][k][i] for i in keep]
        rows, cvals = [], []
        for r in range(m):
            for s in range(r + 1):
                for k in range(N):
                    rows.append([-evaluate(_mat_entry(M[i], r, s), x[k]) for i in range(1, len(M))])
                    cvals.append(evaluate(_mat_entry(M[0], r, s), x[k]))
        B = np.empty((len(rows), len(M) - 1), dtype=object)
        for t, row in enumerate(rows):
            B[t, :] = row
        c = np.array(cvals, dtype=object)
    return Cluster(A, B, c, H)


def solvempmp(M, G, q, x, delta, b, Pi=None, all_of_Pi: bool = True, **kwargs):
    """``solvempmp`` (MPMP.jl:562-586): sample every constraint, build BlockInfo and solve on the
    device.  ``kwargs`` go to :func:`solver.solverank1sdp` (``precision_words`` selects fp64/dd/qd)."""
    from .blockinfo import get_block_info
    from .solver import solverank1sdp
    if Pi is not None:
        abc = [prepareabc(M[j], G[j], q[j], x[j], delta[j], Pi[j], all_of_Pi=all_of_Pi)
               for j in range(len(M))]
    else:
        abc = [prepareabc(M[j], G[j], q[j], x[j], delta[j]) for j in range(len(M))]
    bi = get_block_info(abc)
    return solverank1sdp(abc, b, bi, **kwargs)
