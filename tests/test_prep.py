"""prepareabc, bases, sample points and the sphere-packing program (MPMP.jl:21-407, SP.jl).

The reference ships no fixtures for these, so they are checked against closed
forms (mpmath's special functions, Chebyshev roots, binomial counts) and against the identity
that defines the sampled low-rank form:  sum_r H[l][k][r] v v^T  equals  G_l(x_k) (Pi_l (x) q q^T)(x_k)
on the degree-truncated index set, and B, c are the sampled entries of M in (r, s<=r, k) order.
"""
import math

import mpmath
import numpy as np
import pytest
from mpmath import mpf


@pytest.fixture(scope="module")
def P(pk):
    from clrsdp_amd import poly
    return poly


@pytest.fixture(scope="module")
def prep(pk):
    from clrsdp_amd import prep
    return prep


def test_poly_ring_arithmetic_and_degree(P):
    x, y = P.Poly.gens(2)
    p = (x + 2 * y) ** 2 - 3 * x * y + 1
    assert p.total_degree() == 2
    assert p(mpf(2), mpf(-1)) == (2 - 2) ** 2 - 3 * 2 * (-1) + 1
    assert (p - p).is_zero() and (p - p).total_degree() == -1
    assert (1 - x)(mpf(3), mpf(0)) == -2


def test_laguerre_gegenbauer_against_closed_forms(P):
    with mpmath.workprec(200):
        for alpha in (mpf(0), mpf("0.5"), mpf(3) / 2 - 1):
            xv = mpf("0.37")
            v = P.laguerrebasis(7, alpha, xv)
            for k in range(8):
                assert abs(v[k] - mpmath.laguerre(k, alpha, xv)) < mpf(10) ** -55
            # the same recurrence on a polynomial argument evaluates identically
            x = P.Poly.gens(1)[0]
            vp = P.laguerrebasis(7, alpha, 2 * x)
            assert all(abs(vp[k](xv / 2) - v[k]) < mpf(10) ** -55 for k in range(8))
            assert [q.total_degree() for q in vp] == list(range(8))
        n = 5
        g = P.gegenbauer_basis(6, n, mpf("0.3"))
        lam = mpf(n) / 2 - 1
        for k in range(7):
            ref = mpmath.gegenbauer(k, lam, mpf("0.3")) / mpmath.gegenbauer(k, lam, 1)
            assert abs(g[k] - ref) < mpf(10) ** -55
        J = P.jacobi_basis(1, 1, 1, mpf("0.2"))
        assert J[0] == 1 and J[1] == mpf("0.2")


def test_monomial_basis_and_sample_point_counts(P):
    q = P.make_monomial_basis(3, 4)
    assert len(q) == math.comb(7, 4)
    assert [p.total_degree() for p in q] == sorted(p.total_degree() for p in q)
    assert len(P.create_sample_points(3, 4)) == math.comb(7, 4)
    for d in (3, 4, 7):
        assert len(P.create_sample_points_2d(d)) == math.comb(d + 2, 2)
    assert len(P.create_sample_points_3d(5)) == math.comb(8, 3)
    with mpmath.workprec(120):
        ch = P.create_sample_points_chebyshev(6)
        assert all(abs(mpmath.chebyt(7, t)) < mpf(10) ** -30 for t in ch)
        pts = P.create_sample_points_1d(4)
        c = -mpmath.sqrt(mpmath.pi) / (64 * 5 * mpmath.log(3 - 2 * mpmath.sqrt(2)))
        assert abs(pts[2] - c * 49) < mpf(10) ** -30


def _check_lowrank_identity(cl, M, G, q, x, delta, Pi, degPi):
    m = len(M[0])
    for l, g in enumerate(G):
        for k, xk in enumerate(x):
            gv = g(xk) if hasattr(g, "__call__") else mpf(g)
            vs, hs = cl.A[l][k], cl.H[l][k]
            n = len(vs[0])
            W = mpmath.matrix(n, n)
            for v, h in zip(vs, hs):
                for a in range(n):
                    for b in range(n):
                        W[a, b] += h * v[a] * v[b]
            # expected: G (Pi (x) q q^T) on the truncated index set (Pi index outer)
            idx = []
            npi = 1 if Pi is None else len(Pi[l])
            for pi in range(npi):
                dpi = 0 if Pi is None else degPi[l][pi]
                nd = max(i + 1 for i, p in enumerate(q)
                         if p.total_degree() <= (delta - g.total_degree() - dpi) // 2)
                idx += [(pi, d) for d in range(nd)]
            assert len(idx) == n
            for a, (pa, da) in enumerate(idx):
                for b, (pb, db) in enumerate(idx):
                    piv = 1 if Pi is None else (Pi[l][pa][pb](xk) if hasattr(Pi[l][pa][pb], "__call__")
                                                else mpf(Pi[l][pa][pb]))
                    want = gv * piv * q[da](xk) * q[db](xk)
                    assert abs(W[a, b] - want) <= mpf(10) ** -40 * (1 + abs(want)), (l, k, a, b)
    # B and c: sampled entries of M in (r, s<=r, k) order
    t = 0
    for r in range(m):
        for s in range(r + 1):
            for xk in x:
                assert cl.c[t] == (M[0][r][s](xk) if hasattr(M[0][r][s], "__call__") else mpf(M[0][r][s]))
                for i in range(1, len(M)):
                    e = M[i][r][s]
                    assert cl.B[t, i - 1] == -(e(xk) if hasattr(e, "__call__") else mpf(e))
                t += 1
    assert t == len(cl.c)


def test_prepareabc_rank1_identity(P, prep, pk):
    with mpmath.workprec(160):
        x = P.Poly.gens(1)[0]
        q = P.laguerrebasis(3, mpf("0.5"), x)
        G = [P.Poly.const(1), x, 2 - x]
        M = [[[1 + x, x], [x, 2 * x ** 2]], [[x, 1], [1, x ** 3]], [[P.Poly.const(3), x], [x, 0]]]
        pts = [mpf(i) / 8 + mpf("0.05") for i in range(8)]
        cl = prep.prepareabc(M, G, q, pts, -1)
        _check_lowrank_identity(cl, M, G, q, pts, 6, None, None)
        bi = pk.get_block_info([cl, cl])
        assert bi.m == [2, 2] and bi.L == [3, 3] and bi.n_samples == [8, 8]
        assert bi.Y_blocksizes[0] == [8, 6, 6] and bi.dim_S[0] == 24 and bi.n_y == 2


def test_prepareabc_with_Pi_blocks(P, prep, pk):
    with mpmath.workprec(160):
        x = P.Poly.gens(1)[0]
        q = [P.Poly.const(1), x, x ** 2]
        G = [P.Poly.const(1), x]
        Pi = [[[1 + x ** 2, 0], [0, P.Poly.const(2)]], [[P.Poly.const(3), 0], [0, 1 + x]]]
        M = [[[x ** 2]], [[x]], [[P.Poly.const(1)]]]
        pts = [mpf(i + 1) / 7 for i in range(5)]
        cl = prep.prepareabc(M, G, q, pts, 4, Pi)
        _check_lowrank_identity(cl, M, G, q, pts, 4, Pi, [[2, 0], [0, 1]])
        assert [len(v) for v in cl.A[0][0]] == [5, 5]   # 2 (deg Pi_11 = 2) + 3
        # eigenvalues: Pi_vals * sign(G)
        assert sorted(float(h) for h in cl.H[1][0]) == pytest.approx(sorted([3.0, 1 + 1 / 7]))
        # the threshold removes (near) zero eigenvalues
        Pz = [[[P.Poly.const(1), 0], [0, 0]], [[P.Poly.const(1), 0], [0, 0]]]
        clz = prep.prepareabc(M, G, q, pts, 4, Pz)
        assert all(len(clz.A[l][k]) == 1 for l in range(2) for k in range(5))


def test_sphere_packing_program_shape(pk):
    from clrsdp_amd import sphere_packing as S
    cons, b, bi = S.sphere_packing_constraints(3, 8, prec=256)
    # config 5: J = 7, blocks {2},{18,16},{9,8}x3,{1}x2, n_y = 52, after the
    # reordering [3,6,5,7,4,1,2] of SP.jl:99-105
    assert bi.J == 7 and bi.n_y == 52 and len(b) == 52
    assert bi.Y_blocksizes == [[9, 8], [1], [9, 8], [1], [9, 8], [2], [18, 16]]
    assert bi.dim_S == [17, 1, 17, 1, 17, 3, 51]
    assert sorted(sum(bi.dim_S[j] for j in range(7)) for _ in [0]) == [107]
    # cluster 6 (original 1): c = -(vol_i vol_j)^1/2 for (r,s) = (1,1),(2,1),(2,2)
    with mpmath.workprec(256):
        v1, v2 = S.spherevolume(3, 1), S.spherevolume(3, mpmath.sqrt(2) - 1)
        want = [-v1, -mpmath.sqrt(v1 * v2), -v2]
        assert all(abs(cons[5].c[t] - want[t]) < mpf(10) ** -70 for t in range(3))
        assert abs(S.spherevolume(3, 1) - 4 * mpmath.pi / 3) < mpf(10) ** -70


def test_write_read_files_round_trip_exact(pk, tmp_path):
    from clrsdp_amd import sdpfiles
    from clrsdp_amd import sphere_packing as S
    # multi-precision data (the real sphere-packing instance, 512-bit prepareabc output)
    cons, b, bi = S.sphere_packing_constraints(3, 4, prec=512, reorder=False)
    sdpfiles.write_files(str(tmp_path / "sp"), cons, bi, b)
    c2, b2, bi2 = sdpfiles.read_files(str(tmp_path / "sp"))
    assert bi2.Y_blocksizes == bi.Y_blocksizes and bi2.dim_S == bi.dim_S and bi2.ranks == bi.ranks
    assert list(b2) == list(b)
    for c1, cc in zip(cons, c2):
        assert all(x == y for x, y in zip(c1.c, cc.c))
        assert all(x == y for x, y in zip(np.asarray(c1.B).ravel(), np.asarray(cc.B).ravel()))
        for Al1, Al2 in zip(c1.A, cc.A):
            for Ak1, Ak2 in zip(Al1, Al2):
                assert all((v1 == v2).all() for v1, v2 in zip(Ak1, Ak2))
        assert c1.H == cc.H
    # float data
    cons, b = pk.synth(J=2, delta=3, rank=2, n_y=3, seed=2, m=2, L=2)
    bi = pk.get_block_info(cons)
    sdpfiles.write_files(str(tmp_path / "f"), cons, bi, b)
    c2, b2, bi2 = sdpfiles.read_files(str(tmp_path / "f"), exact=False)
    assert np.array_equal(b2, b) and all(np.array_equal(x.B, y.B) for x, y in zip(cons, c2))
    assert all(np.array_equal(np.stack(x.A[1][2]), np.stack(y.A[1][2])) for x, y in zip(cons, c2))
    # the driver's write_only path (SP.jl:95-98, 107)
    assert S.Nsphere_packing_2point(3, 2, file_path=str(tmp_path / "w"), write_only=True) is True
    assert sdpfiles.read_files(str(tmp_path / "w"))[2].J == 7
