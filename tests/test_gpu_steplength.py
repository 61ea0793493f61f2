"""Step length (compute_step_length, MPMP.jl:1829-1898) through clrsdp_step_length, and the
loop-control thresholds of a reused handle.

Tolerance: lambda_min agrees with numpy.linalg.eigvalsh of the symmetrised L^-1 dM L^-T to
1e-12 of the block's spectral radius (the Sturm multisection stops at 2^-54 of the Gershgorin
span; Householder tridiagonalisation is backward stable to ~n eps ||T||).
"""
import numpy as np
import pytest

from helpers import rand_spd

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _sym(rng, n):
    G = rng.standard_normal((n, n))
    return (G + G.T) / 2


def _ref_eigs(M, dM):
    out = []
    for a, b in zip(M, dM):
        L = np.linalg.cholesky(a)
        T = np.linalg.solve(L, np.linalg.solve(L, b).T)
        out.append(np.linalg.eigvalsh((T + T.T) / 2)[0])
    return np.array(out)


@pytest.mark.parametrize("scale", [1.0, 1e40, 1e-40, 1e200, 1e-200])
@pytest.mark.parametrize("n", [5, 37, 127])
def test_eigmin_scaled_blocks(pk, n, scale):
    """M = I, dM = scale * G: lambda_min of blocks of very large or very small norm, n not a
    multiple of 8 (the register eigen-solver rescales the tridiagonal before its Sturm counts;
    without that the product-form counts overflowed near a span of 1e37)."""
    from clrsdp_amd.solver import compute_step_length
    rng = np.random.default_rng(n)
    dM = [_sym(rng, n) * scale for _ in range(3)]
    M = [np.eye(n) for _ in range(3)]
    alpha, flag, eig = compute_step_length(M, dM, 0.7, return_eigs=True)
    ref = _ref_eigs(M, dM)
    rad = np.array([np.max(np.abs(np.linalg.eigvalsh(b))) for b in dM])
    assert np.all(np.abs(eig - ref) <= TOL * rad), (eig, ref)
    mn = ref.min()
    ref_alpha = 1.0 if mn > -0.7 else -0.7 / mn
    assert abs(alpha - ref_alpha) <= 1e-10 * abs(ref_alpha)
    assert flag is False


@pytest.mark.parametrize("sizes", [[1, 2, 18, 16, 9, 8], [64, 128], [130], [140, 33], [200]])
def test_step_length_against_oracle(pk, oracle, sizes):
    """Random SPD M and symmetric dM over mixed block sizes (the register path for n <= 128,
    the LDS and global eigen-solvers and potrf + trsm above): alpha and every lambda_min against
    the oracle's restatement (Cholesky, two triangular solves, eigenvalues)."""
    from clrsdp_amd.solver import compute_step_length
    rng = np.random.default_rng(sum(sizes))
    M = [rand_spd(n, rng, 0.5) for n in sizes]
    dM = [_sym(rng, n) for n in sizes]
    alpha, _, eig = compute_step_length(M, dM, 0.7, return_eigs=True)
    ref = _ref_eigs(M, dM)
    rad = np.array([np.max(np.abs(np.linalg.eigvalsh(np.linalg.solve(np.linalg.cholesky(a), np.linalg.solve(np.linalg.cholesky(a), b).T)))) for a, b in zip(M, dM)])
    assert np.all(np.abs(eig - ref) <= 1e-11 * rad), (eig, ref)
    ar = oracle.Fp64()
    bi = type("BI", (), {"J": len(sizes), "L": [1] * len(sizes)})()
    a_or = ar.num(oracle.compute_step_length(ar, [[m] for m in M], [[d] for d in dM], 0.7, bi))
    assert abs(alpha - float(a_or)) <= 1e-10 * abs(float(a_or))


def test_step_length_not_pd(pk):
    from clrsdp_amd import _lib
    from clrsdp_amd.solver import compute_step_length
    M = [np.eye(4), -np.eye(6)]
    dM = [np.eye(4), np.eye(6)]
    with pytest.raises(_lib.ClrsdpError) as e:
        compute_step_length(M, dM, 0.7)
    assert e.value.code == _lib.E_STEP


def test_reused_handle_new_thresholds(pk):
    """Two pipelined solves on one handle with different duality_gap_threshold: the second
    stops where a fresh handle stops (the loop-body graphs carry the thresholds by value, so
    clrsdp_set_control must drop them)."""
    cons, b = pk.synth(J=3, delta=5, rank=1, n_y=4, seed=7)
    bi = pk.get_block_info(cons)
    kw = dict(omega_p=10.0, omega_d=10.0, primal_error_threshold=1e-6, dual_error_threshold=1e-6,
              maxiterations=100, verbose=False, return_info=True, pipelined=True)
    dev = pk.DeviceSolver(cons, b, bi)
    try:
        first = pk.solverank1sdp(cons, b, bi, solver=dev, duality_gap_threshold=1e-2, **kw)
        second = pk.solverank1sdp(cons, b, bi, solver=dev, duality_gap_threshold=1e-7, **kw)
    finally:
        dev.close()
    fresh = pk.solverank1sdp(cons, b, bi, duality_gap_threshold=1e-7, **kw)
    assert first[-1].status == second[-1].status == fresh[-1].status == "terminated"
    assert first[-1].iterations < second[-1].iterations
    assert second[-1].iterations == fresh[-1].iterations
    assert [r[2:] for r in second[-1].log] == [r[2:] for r in fresh[-1].log]


def test_step_length_all_1x1_blocks(pk):
    """Every block 1 x 1 (an LP-like instance): the symmetric-epilogue flag and the one-column
    gemv path meet in the plan; the product is trivially symmetric and must not be refused."""
    from clrsdp_amd.solver import compute_step_length
    M = [np.array([[v]]) for v in (2.0, 0.5, 3.0)]
    dM = [np.array([[v]]) for v in (-1.0, 0.25, -6.0)]
    alpha, flag, eig = compute_step_length(M, dM, 0.7, return_eigs=True)
    ref = np.array([-0.5, 0.5, -2.0])
    assert np.allclose(eig, ref, rtol=1e-15, atol=0.0)
    assert abs(alpha - 0.35) <= 1e-15
    assert flag is False


def test_device_solver_all_1x1_blocks(pk):
    """A handle whose local blocks are all 1 x 1 (delta = 1) is created and runs the loop body to
    the same log as the oracle-checked host loop would stop at (no E_ARG at plan build)."""
    cons, b = pk.synth(J=3, delta=1, rank=1, n_y=2, seed=11)
    bi = pk.get_block_info(cons)
    out = pk.solverank1sdp(cons, b, bi, omega_p=10.0, omega_d=10.0, duality_gap_threshold=1e-6,
                           primal_error_threshold=1e-6, dual_error_threshold=1e-6,
                           maxiterations=60, verbose=False, return_info=True)
    assert out[-1].iterations > 0
    assert out[-1].status in ("terminated", "optimal", "maxiterations")


def _mp_tridiag(n, d, e, prec=320):
    import mpmath
    with mpmath.workprec(prec):
        A = np.empty((n, n), dtype=object)
        for i in range(n):
            for j in range(n):
                A[i, j] = mpmath.mpf(0)
        for i in range(n):
            A[i, i] = mpmath.mpf(d[i])
            if i + 1 < n:
                A[i, i + 1] = A[i + 1, i] = mpmath.mpf(e[i])
    return A


def _mp_eigmin(A, prec=320):
    import mpmath
    with mpmath.workprec(prec):
        M = mpmath.matrix(A.tolist())
        ev = mpmath.eigsy(M, eigvals_only=True)
        return min(ev)


# (qd: measured 1.0e-54 on the decoupled n = 64 tridiagonal; the qd stage parity holds 1e-50)
EIG_TOL = {1: 1e-13, 2: 1e-28, 4: 1e-50}


@pytest.mark.parametrize("words,n", [(1, 18), (1, 64), (1, 128), (2, 18), (2, 64), (4, 18),
                                     (4, 64)])
def test_eigmin_decoupled_and_zero_minor_cases(pk, words, n):
    """lambda_min at fp64 / dd / qd (clrsdp_eigmin) on blocks whose Sturm recurrences meet zero
    couplings and exact zero minors (the zero-minor rule of the multi-word count and its fp64
    twin, kernels_dense.h sturm_any_below / the multi-word eig_multisection): c I (every
    coupling zero, every minor zero at sigma = c), a tridiagonal decoupled in the middle with
    constant diagonal (d_i = sigma for the repeated eigenvalue of both halves), a tridiagonal with
    alternating zero couplings (2x2 blocks) and a dense block with one decoupled row.  Against
    320-bit mpmath eigenvalues, to the word's resolution times ||A||."""
    import mpmath
    rng = np.random.default_rng(1000 * words + n)
    blocks = []
    # c I
    blocks.append(np.eye(n) * 0.75)
    # decoupled in the middle, d_i = 1/2, couplings 1/4 except a zero one
    e = [0.25] * (n - 1)
    e[n // 2 - 1] = 0.0
    blocks.append(_mp_tridiag(n, [0.5] * n, e))
    # 2x2 blocks [[a, b], [b, a]] (zero coupling between them), eigenvalues a -/+ b, repeated
    d = [0.5] * n
    e = [(0.125 if i % 2 == 0 else 0.0) for i in range(n - 1)]
    blocks.append(_mp_tridiag(n, d, e))
    # dense random symmetric with row/column 0 decoupled (A[0, 0] is an eigenvalue)
    G = rng.standard_normal((n, n))
    S = (G + G.T) / 4
    S[0, 1:] = 0.0
    S[1:, 0] = 0.0
    S[0, 0] = -3.0
    blocks.append(S)
    got = pk.eigmin(blocks, precision_words=words)
    with mpmath.workprec(320):
        for q, (B, g) in enumerate(zip(blocks, got)):
            Bm = B if B.dtype == object else np.array([[mpmath.mpf(float(x)) for x in row] for row in B], dtype=object)
            ref = _mp_eigmin(Bm)
            nrm = max(abs(x) for x in Bm.reshape(-1))
            err = abs(mpmath.mpf(g) - ref) / nrm
            assert err <= EIG_TOL[words], (q, float(g), float(ref), float(err))


@pytest.mark.parametrize("words,n", [(2, 18), (2, 40), (2, 64), (4, 18), (4, 40)])
def test_eigmin_refined_fp64_eigenpair(pk, words, n):
    """The multi-word lambda_min of blocks up to 64 (eigmin_mx: fp64 tridiagonalisation and
    eigenpair, refined at the word's width, accepted by Temple's bound, else the multi-word
    tridiagonalisation) on blocks whose leading words alone would give the wrong answer:
    Q diag(lam) Q^T at 320 bits with lambda_2 - lambda_1 = 2^-g (g = 3, 30, 60; 2^-60 is below
    the fp64 resolution, so that block takes the multi-word path) and a random symmetric block
    with entries carrying lower words.  Against 320-bit mpmath eigenvalues, to the word's
    resolution times ||A|| (the limb split of the 320-bit entries moves lambda_min by about
    2^-BITS ||A||, far inside the tolerance)."""
    import mpmath
    rng = np.random.default_rng(7000 + 100 * words + n)
    blocks = []
    with mpmath.workprec(320):
        for g in (3, 30, 60):
            Qf, _ = np.linalg.qr(rng.standard_normal((n, n)))
            lam = [mpmath.mpf(-0.5), mpmath.mpf(-0.5) + mpmath.ldexp(1, -g)]
            lam += [mpmath.mpf(-0.4) + mpmath.mpf(0.8) * i / n for i in range(2, n)]
            Qm = [[mpmath.mpf(float(Qf[i, k])) for k in range(n)] for i in range(n)]
            B = np.empty((n, n), dtype=object)
            for i in range(n):
                for j in range(i + 1):
                    s = mpmath.fsum(Qm[i][k] * Qm[j][k] * lam[k] for k in range(n))
                    B[i, j] = B[j, i] = s
            blocks.append(B)
        G = rng.standard_normal((n, n))
        L = rng.standard_normal((n, n)) * 2.0 ** -60
        B = np.empty((n, n), dtype=object)
        for i in range(n):
            for j in range(i + 1):
                B[i, j] = B[j, i] = mpmath.mpf(float(G[i, j] + G[j, i])) / 4 + mpmath.mpf(float(L[i, j]))
        blocks.append(B)
    got = pk.eigmin(blocks, precision_words=words)
    with mpmath.workprec(320):
        for q, (B, g) in enumerate(zip(blocks, got)):
            ref = _mp_eigmin(B)
            nrm = max(abs(x) for x in B.reshape(-1))
            err = abs(mpmath.mpf(g) - ref) / nrm
            assert err <= EIG_TOL[words], (q, float(g), float(ref), float(err))


# --- structured batches (the inputs of tools/micro/eig_split_bench.hip) ---
#
# An eigmin_split variant of round 5 (the single-wave tail, build r5r) returned lambda_min off by
# up to 11.2 ||A|| on near-diagonal and decoupled-16-block inputs and at n = 33/64/127 and batch
# 256, and the small random batches above did not catch it.  These run the structures of that
# microbenchmark through clrsdp_eigmin at the batch sizes of the loop bodies.

def _structured(kind, n, rng, scale=1.0):
    """kind 0 random symmetric, 1 near-diagonal SPD, 2 tridiagonal (d_i = i mod 7, e_i = 1),
    3 random symmetric decoupled into 16 x 16 diagonal blocks (eig_split_bench.hip:68-80)."""
    A = rng.random((n, n)) - 0.5
    A = np.tril(A) + np.tril(A, -1).T
    if kind == 1:
        A = 1e-3 * A
        A[np.diag_indices(n)] = 1.0 + 0.1 * (rng.random(n) - 0.5)
    elif kind == 2:
        A = np.zeros((n, n))
        A[np.diag_indices(n)] = np.arange(n) % 7
        idx = np.arange(n - 1)
        A[idx + 1, idx] = A[idx, idx + 1] = 1.0
    elif kind == 3:
        blk = np.arange(n) // 16
        A[blk[:, None] != blk[None, :]] = 0.0
    return A * scale


@pytest.mark.parametrize("batch", [64, 256])
@pytest.mark.parametrize("n", [33, 64, 127, 128])
def test_eigmin_structured_batches_fp64(pk, n, batch):
    """fp64 lambda_min (eigmin_split, the loop body's kernel for n <= 128) of batches cycling
    through the four structures, against numpy eigvalsh, to 1e-12 of the block's spectral
    radius."""
    rng = np.random.default_rng(31 * n + batch)
    blocks = [_structured(q % 4, n, rng) for q in range(batch)]
    got = pk.eigmin(blocks, precision_words=1)
    for q, B in enumerate(blocks):
        ev = np.linalg.eigvalsh(B)
        rad = max(abs(ev[0]), abs(ev[-1]))
        assert abs(got[q] - ev[0]) <= 1e-12 * rad, (q, q % 4, got[q], ev[0], abs(got[q] - ev[0]) / rad)


@pytest.mark.parametrize("scale", [1e-200, 1e200])
def test_eigmin_structured_scaled_fp64(pk, scale):
    """The same structures at n = 128 scaled to the ends of the fp64 range (the Sturm counts'
    rescaling)."""
    rng = np.random.default_rng(5)
    blocks = [_structured(q % 4, 128, rng, scale) for q in range(64)]
    got = pk.eigmin(blocks, precision_words=1)
    for q, B in enumerate(blocks):
        ev = np.linalg.eigvalsh(B / scale) * scale
        rad = max(abs(ev[0]), abs(ev[-1]))
        assert abs(got[q] - ev[0]) <= 1e-12 * rad, (q, q % 4, got[q], ev[0])


_MP_REF = {}


def _mp_ref_structured(kind, n):
    """(block, 320-bit lambda_min, max-norm) of one structured block, cached across words."""
    import mpmath
    key = (kind, n)
    if key not in _MP_REF:
        B = _structured(kind, n, np.random.default_rng(900 + 10 * n + kind))
        with mpmath.workprec(320):
            Bm = np.array([[mpmath.mpf(float(x)) for x in row] for row in B], dtype=object)
            _MP_REF[key] = (B, _mp_eigmin(Bm), float(np.max(np.abs(B))))
    return _MP_REF[key]


@pytest.mark.parametrize("words", [2, 4])
@pytest.mark.parametrize("n", [33, 64])
def test_eigmin_structured_batches_multiword(pk, words, n):
    """Multi-word lambda_min (eigmin_mx with its eigmin_lds2 fallback) on a batch of 64 built
    from the four structures (16 copies each), against 320-bit mpmath at the word's tolerance;
    copies of one block must give the same value."""
    import mpmath
    refs = [_mp_ref_structured(k, n) for k in range(4)]
    blocks = [refs[q % 4][0] for q in range(64)]
    got = pk.eigmin(blocks, precision_words=words)
    with mpmath.workprec(320):
        for q in range(64):
            B, ref, nrm = refs[q % 4]
            err = abs(mpmath.mpf(got[q]) - ref) / nrm
            assert err <= EIG_TOL[words], (q, q % 4, float(got[q]), float(ref), float(err))
            assert got[q] == got[q % 4], (q, got[q], got[q % 4])
