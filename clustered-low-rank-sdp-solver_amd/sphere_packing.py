"""Two-point bound for packings of spheres of N radii (examples/SpherePacking.jl, SP.jl:1-131).

``Nsphere_packing_2point(n, d, r, N)`` builds the polynomial matrix program of de Laat,
Oliveira and Vallentin (variables M and a_{ij,k}; SP.jl:29-60), samples it with
:func:`prep.prepareabc` and solves it on the GPU.  The objective is ``-M``, so the density
bound is minus the optimal objective.  Reference quirks restated or fixed:

* SP.jl:92 passes ``normalize=`` to prepareabc, which has no such keyword; it is dropped here.
* For N = 2 (J = 7) the clusters are reordered [3,6,5,7,4,1,2] before solving (SP.jl:99-105).
* The reference's ``test_bound_sphere_packing`` prints ``-cur_bound[end]``, i.e. minus the
  solve time (the last element of the returned tuple); :func:`test_bound_sphere_packing`
  returns the bound itself.
"""
from __future__ import annotations

import math
from typing import List, Sequence

import mpmath
from mpmath import mp, mpf

from .blockinfo import get_block_info
from .poly import Poly, create_sample_points_1d, laguerrebasis
from .prep import prepareabc

NACL_DENSITY = 0.793        # SP.jl:125
NACL_BOUND = 0.813          # de Laat et al., SP.jl:126


def spherevolume(n: int, r):
    """Volume of the n-ball of radius r (SP.jl:11-13)."""
    return mpmath.sqrt(mp.pi) ** n / mpmath.gamma(mpf(n) / 2 + 1) * mpf(r) ** n


def laguerre(k: int, alpha, x):
    """L_k^alpha(x) (SP.jl:16)."""
    return laguerrebasis(k, alpha, x)[-1]


def _zero(N):
    return [[mpf(0)] * N for _ in range(N)]


def standard_basis(N: int, i: int, j: int, element=1, symmetric: bool = True):
    """N x N matrix with ``element`` at (i, j) (and (j, i) when symmetric), 1-based (SP.jl:18-27)."""
    E = _zero(N)
    E[i - 1][j - 1] = element
    if symmetric:
        E[j - 1][i - 1] = element
    return E


def sphere_packing_program(n: int, d: int, r: Sequence, N: int = 2):
    """The program of SP.jl:29-86: returns ``(M, G, q, sample_points, delta, b)``."""
    x = Poly.gens(1)[0]
    tri = [(i, j) for i in range(1, N + 1) for j in range(1, i + 1)]
    ks = range(0, 2 * d + 1)
    alpha = mpf(n) / 2 - 1
    # M0: -(vol_i vol_j)^1/2 + sum a_{ij,0} E_ij >= 0, NxN, G = {1}
    M0 = [[[-mpmath.sqrt(spherevolume(n, r[i]) * spherevolume(n, r[j])) for j in range(N)]
           for i in range(N)], _zero(N)]
    M0 += [standard_basis(N, i, j, 1) if k == 0 else _zero(N) for k in ks for (i, j) in tri]
    # M1: sum_k a_{ij,k} E_ij x^k >= 0, NxN, G = {1, x}
    M1 = [_zero(N), _zero(N)] + [standard_basis(N, i, j, x ** k) for k in ks for (i, j) in tri]
    # M2_ij: -sum_k a_{ij,k} k!/pi^k L_k^{n/2-1}(pi x) >= 0 for x >= (r_i + r_j)^2, 1x1
    M2 = []
    for (i, j) in tri:
        Mi = [[[mpf(0)]], [[mpf(0)]]]
        for k in ks:
            for (rr, ss) in tri:
                if (rr, ss) == (i, j):
                    Mi.append([[-mpmath.factorial(k) / mp.pi ** k * laguerre(k, alpha, mp.pi * x)]])
                else:
                    Mi.append([[mpf(0)]])
        M2.append(Mi)
    # M3_i: M - sum_k a_{ii,k} k!/pi^k L_k(0) >= 0, 1x1, G = {1}
    M3 = []
    for i in range(1, N + 1):
        Mi = [[[mpf(0)]], [[mpf(1)]]]
        for k in ks:
            for (rr, ss) in tri:
                if rr == ss == i:
                    Mi.append([[-mpmath.factorial(k) / mp.pi ** k * laguerre(k, alpha, mpf(0))]])
                else:
                    Mi.append([[mpf(0)]])
        M3.append(Mi)
    M = [M0, M1] + M2 + M3
    pts = create_sample_points_1d(2 * d)
    sample_points = [mpf(0), list(pts)] + [[p + (r[i - 1] + r[j - 1]) ** 2 for p in pts] for (i, j) in tri] \
        + [[mpf(0)] for _ in range(N)]
    G = [[Poly.const(1)], [Poly.const(1), x]] + [[Poly.const(1), x - (r[i - 1] + r[j - 1]) ** 2]
                                                 for (i, j) in tri] + [[Poly.const(1)] for _ in range(N)]
    q = laguerrebasis(d, alpha, 2 * mp.pi * x)
    q = [p * (1 / max(p.coeffs())) for p in q]
    delta = [0, 2 * d] + [2 * d] * len(tri) + [0] * N
    b = [mpf(-1)] + [mpf(0)] * (len(ks) * len(tri))
    return M, G, q, sample_points, delta, b


def sphere_packing_constraints(n: int = 3, d: int = 8, r=None, N: int = 2, prec: int = 512,
                               reorder: bool = True):
    """Sampled constraints and BlockInfo of SP.jl:88-105 (with the N = 2 reordering)."""
    with mpmath.workprec(prec):
        if r is None:
            r = [mpf(1), mpmath.sqrt(2) - 1]
        r = [mpf(v) for v in r]
        M, G, q, pts, delta, b = sphere_packing_program(n, d, r, N)
        cons = [prepareabc(M[j], G[j], q, pts[j], delta[j]) for j in range(len(G))]
        if reorder and len(M) == 7:
            cons = [cons[i - 1] for i in (3, 6, 5, 7, 4, 1, 2)]
        bi = get_block_info(cons)
    return cons, b, bi


def Nsphere_packing_2point(n: int, d: int, r=None, N: int = 2, file_path: str = "",
                           write_only: bool = False, omega=100, prec: int = 512, **kwargs):
    """Build and solve the N-radii two-point program (SP.jl:29-110) on the device.

    ``file_path``: also write the sampled instance there (:func:`sdpfiles.write_files`, before
    the reordering, as SP.jl:95-98); ``write_only`` returns True after writing.  ``kwargs`` go to
    :func:`solver.solverank1sdp` (``precision_words=4`` runs quad-double).  Returns the 11-tuple
    of ``solverank1sdp`` (plus RunInfo with ``return_info``).
    """
    from .solver import solverank1sdp
    if file_path:
        from .sdpfiles import write_files
        c0, b0_, bi0 = sphere_packing_constraints(n, d, r, N, prec, reorder=False)
        write_files(file_path, c0, bi0, b0_)
        if write_only:
            return True
    cons, b, bi = sphere_packing_constraints(n, d, r, N, prec)
    return solverank1sdp(cons, b, bi, omega_p=omega, omega_d=omega, **kwargs)


def test_bound_sphere_packing(n: int = 3, d: int = 8, **kwargs):
    """SP.jl:113-129: the bound for radii {1, sqrt 2 - 1} (compare NaCl 0.793, bound 0.813)."""
    res = Nsphere_packing_2point(n, d, None, 2, **kwargs)
    bound = -res[9]
    print(f"{bound}")
    print(f"Compare to the density of NaCL: {NACL_DENSITY} (Current bound: {NACL_BOUND})")
    return bound
