"""GPU tests of the pivoted-LU factorisations (the reference's approx_lu! for S_j and Q,
MPMP.jl:1433-1505, and approx_inv! for X^-1, MPMP.jl:774-786) and of the Cholesky -> LU
fallback (clrsdp_set_factorization, include/clrsdp.h).

The oracle (oracle/mpmp_oracle.py) factorises S_j and Q by partially pivoted LU exactly as the
reference, so with CLRSDP_FACT_LU_SQ the device path is the same algorithm; tolerances are the
stage-parity ones of test_gpu_parity.py (fp64 1e-11, dd 1e-25, qd 1e-50, scale-aware).
"""
import numpy as np
import pytest

from helpers import CONFIGS_SMALL, rel_err, residual_scales, stage_device, stage_reference

pytestmark = pytest.mark.gpu

CONFIGS_LU = CONFIGS_SMALL + [
    dict(J=2, delta=64, rank=2, n_y=64),      # C2 cluster shape (dim_S = 127)
    dict(J=2, delta=128, rank=1, n_y=128),    # C3 cluster shape (dim_S = 255)
]


def _mp_cons(pk, ar, cons):
    return [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in Al] for Al in cl.A],
                       ar.asarray(cl.B), ar.asarray(cl.c),
                       [[[ar.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]


def _lu_stage_compare(pk, oracle, cons, b, flags, words=1, ar=None, tol=1e-11, iters_before=2):
    from clrsdp_amd import _lib as L
    ar = ar or oracle.Fp64()
    bi = oracle.get_block_info(cons)
    prm = {k: oracle._param(ar, v) for k, v in oracle.DEFAULTS.items()}
    state = oracle.initial_point(ar, bi, 10.0, 10.0)
    for _ in range(iters_before):
        state, _ = oracle.iteration(ar, cons, bi, b, None, ar.num(0), state, False, prm)
    nxt, it = oracle.iteration(ar, cons, bi, b, None, ar.num(0), state, False, prm)
    dev = pk.DeviceSolver(cons, b, pk.get_block_info(cons), precision_words=words)
    try:
        dev.set_factorization(flags)
        assert dev.factorization == flags
        dev.set_state(*state)
        got = stage_device(dev, words > 1)
    finally:
        dev.close()
    ref = stage_reference(it, nxt, bi)
    sc = residual_scales(cons, b, state[1])
    e = {k: rel_err(got[k], ref[k], sc.get(k, 0.0)) for k in ref}
    bad = {k: v for k, v in e.items() if not v <= tol}
    assert not bad, f"LU stage parity failures: {bad}"
    return e


@pytest.mark.parametrize("cfg", CONFIGS_LU, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_lu_stage_parity_fp64(pk, oracle, cfg):
    """S_j and Q by pivoted LU (CLRSDP_FACT_LU_SQ) against the oracle's LU, every stage."""
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=3, **cfg)
    _lu_stage_compare(pk, oracle, cons, b, L.FACT_LU_SQ)


@pytest.mark.parametrize("cfg", [CONFIGS_SMALL[0], CONFIGS_SMALL[3], dict(J=2, delta=64, rank=2, n_y=64)],
                         ids=["c1", "m3L2", "c2shape"])
def test_lu_inverse_stage_parity_fp64(pk, oracle, cfg):
    """X^-1 by approx_inv! (CLRSDP_FACT_LU_X) together with LU for S_j and Q."""
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=3, **cfg)
    _lu_stage_compare(pk, oracle, cons, b, L.FACT_LU_SQ | L.FACT_LU_X)


@pytest.mark.parametrize("words,tol", [(2, 1e-25), (4, 1e-50)])
def test_lu_stage_parity_multiword(pk, oracle, words, tol):
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=3, J=2, delta=5, rank=2, n_y=4)
    ar = oracle.Mp(256)
    _lu_stage_compare(pk, oracle, _mp_cons(pk, ar, cons), ar.asarray(b), L.FACT_LU_SQ | L.FACT_LU_X,
                      words=words, ar=ar, tol=tol)


def _run(dev, stage, P, L):
    """run_stage, tolerating the Y status (the step length's cho!(Y), reported from XINV on:
    Y is indefinite in these states on purpose)."""
    try:
        dev.run_stage(stage, P, False)
    except L.ClrsdpError as e:
        if e.code != L.E_STEP:
            raise


def _indefinite_Y_state(oracle, cons, b, bi):
    """A mid-run state whose Y blocks are shifted to be indefinite: S_j = (V^T X^-1 V) o (V^T Y V)
    is then indefinite (but well conditioned), so its Cholesky fails while pivoted LU does not."""
    ar = oracle.Fp64()
    prm = {k: oracle._param(ar, v) for k, v in oracle.DEFAULTS.items()}
    state = oracle.initial_point(ar, bi, 10.0, 10.0)
    for _ in range(2):
        state, _ = oracle.iteration(ar, cons, bi, b, None, 0.0, state, False, prm)
    x, X, y, Y = state
    Y2 = []
    for Yj in Y:
        row = []
        for Yb in Yj:
            ev = np.linalg.eigvalsh(Yb)
            row.append(Yb - (ev[0] + 0.37 * (ev[-1] - ev[0])) * np.eye(Yb.shape[0]))
        Y2.append(row)
    return x, X, y, Y2


@pytest.mark.parametrize("blk", ["1", "0"], ids=["blocked", "one-cu"])
def test_cholesky_fails_dd_c2_shape(pk, oracle, blk, monkeypatch):
    """Double-double S_j of 127 (the config-4 cluster shape) on the indefinite-Y state: both
    Cholesky factorisations of S_j -- the blocked potrf across workgroups (potrf_blk_*, default
    above n = 64) and the one-CU chol_lookahead (CLRSDP_POTRF_BLK=0) -- report the failure
    (CLRSDP_E_NOT_PD_S), as the fp64 path does."""
    from clrsdp_amd import _lib as L
    monkeypatch.setenv("CLRSDP_POTRF_BLK", blk)
    cons, b = pk.synth(seed=5, J=2, delta=64, rank=2, n_y=64)
    bi = oracle.get_block_info(cons)
    x, X, y, Y = _indefinite_Y_state(oracle, cons, b, bi)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    dev = pk.DeviceSolver(cons, b, pk.get_block_info(cons), precision_words=2)
    try:
        dev.set_factorization(0)
        dev.set_state(x, X, y, Y)
        for s in (L.STAGE_MU_R, L.STAGE_XINV, L.STAGE_SCHUR):
            _run(dev, s, P, L)
        with pytest.raises(L.ClrsdpError) as ei:
            dev.run_stage(L.STAGE_FACTOR, P, False)
        assert ei.value.code == L.E_NOT_PD_S
    finally:
        dev.close()


@pytest.mark.parametrize("cfg", [dict(J=2, delta=6, rank=1, n_y=4), dict(J=2, delta=64, rank=2, n_y=64)],
                         ids=["small", "c2shape"])
def test_cholesky_fails_lu_matches_oracle(pk, oracle, cfg):
    """Cholesky of an indefinite S_j fails (CLRSDP_E_NOT_PD_S); pivoted LU on the same S_j gives
    Q and the predictor direction of the oracle's approx_lu! path (MPMP.jl:1433-1505, 1682-1776)."""
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=5, **cfg)
    bi = oracle.get_block_info(cons)
    x, X, y, Y = _indefinite_Y_state(oracle, cons, b, bi)
    ar = oracle.Fp64()
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    # Cholesky path: FACTOR reports the reference's "S was not decomposed" outcome
    dev = pk.DeviceSolver(cons, b, pk.get_block_info(cons))
    try:
        dev.set_factorization(0)
        dev.set_state(x, X, y, Y)
        for s in (L.STAGE_MU_R, L.STAGE_XINV, L.STAGE_SCHUR):
            _run(dev, s, P, L)
        with pytest.raises(L.ClrsdpError) as ei:
            dev.run_stage(L.STAGE_FACTOR, P, False)
        assert ei.value.code == L.E_NOT_PD_S
    finally:
        dev.close()
    # oracle: the same stages with approx_lu!
    mu = oracle.dot_blocks(ar, X, Y) / bi.total_dim
    R = oracle.compute_residual_R(ar, X, Y, 0.3 * mu)
    Xi = oracle.xinv(ar, X)
    dec, AY = oracle.compute_T_decomposition(ar, cons, Xi, Y, bi)
    Pm, p, d = oracle.compute_residuals(ar, cons, x, X, y, AY, b, None, bi, use_AY=True)
    dx, dX, dy, dY = oracle.compute_search_direction(ar, cons, Pm, p, d, R, Xi, Y, bi, dec)
    dev = pk.DeviceSolver(cons, b, pk.get_block_info(cons))
    try:
        dev.set_factorization(L.FACT_LU_SQ)
        dev.set_state(x, X, y, Y)
        for s in (L.STAGE_MU_R, L.STAGE_XINV, L.STAGE_SCHUR, L.STAGE_FACTOR, L.STAGE_RESIDUALS,
                  L.STAGE_PREDICTOR):
            _run(dev, s, P, L)
        from clrsdp_amd import instance as inst
        e = {"Q": rel_err(dev.buffer(L.BUF_Q), dec.Q_raw.reshape(-1, order="F")),
             "dx": rel_err(dev.buffer(L.BUF_DX), dx), "dy": rel_err(dev.buffer(L.BUF_DY), dy),
             "dX": rel_err(dev.buffer(L.BUF_DXMAT), inst.blocks_to_flat(dX)),
             "dY": rel_err(dev.buffer(L.BUF_DYMAT), inst.blocks_to_flat(dY))}
    finally:
        dev.close()
    # S_j is indefinite but not ill-conditioned: the LU results agree to round-off
    print(e)
    assert all(v < 1e-9 for v in e.values()), e


def test_iterate_falls_back_to_lu(pk, oracle):
    """clrsdp_iterate with the default CLRSDP_FACT_FALLBACK on a state whose S_j Cholesky fails:
    the body is re-run with LU (flags gain CLRSDP_FACT_LU_SQ) and fails only where the reference
    fails too -- here the step length, cho!(Y) of an indefinite Y (MPMP.jl:1846-1882)."""
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=5, J=2, delta=6, rank=1, n_y=4)
    bi = oracle.get_block_info(cons)
    st = _indefinite_Y_state(oracle, cons, b, bi)
    dev = pk.DeviceSolver(cons, b, pk.get_block_info(cons))
    try:
        assert dev.factorization == L.FACT_FALLBACK
        dev.set_state(*st)
        with pytest.raises(L.ClrsdpError) as ei:
            dev.iterate(pk.make_params("0.3", "0.1", "0.7", 0), False)
        assert ei.value.code == L.E_STEP
        assert dev.factorization == L.FACT_FALLBACK | L.FACT_LU_SQ
        x, X, y, Y = dev.get_state()        # nothing was applied
        assert np.array_equal(x, st[0]) and np.array_equal(y, st[2])
    finally:
        dev.close()


def test_lu_run_matches_golden(pk):
    """A whole solve with LU for S_j and Q from the start (the reference's factorisation)
    reproduces the 256-bit golden log at dd to the golden tolerance, as the Cholesky path does."""
    import json
    import os

    import mpmath
    from clrsdp_amd import _lib as L
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rank2_mp256_seed5.json")))
    cons, b = pk.synth(**g["instance"])
    bi = pk.get_block_info(cons)
    res = pk.solverank1sdp(cons, b, bi, maxiterations=g["iterations"] + 1, precision_words=2,
                           verbose=False, return_info=True, record_exact=True,
                           factorization=L.FACT_LU_SQ, **g["params"])
    mpmath.mp.prec = 256
    for it, (sc, ref) in enumerate(zip(res[-1].exact, g["log"])):
        for key, slot in (("mu", "mu"), ("alpha_p", "alpha_p"), ("alpha_d", "alpha_d"), ("beta", "beta_c")):
            r = mpmath.mpf(ref[key])
            assert abs(mpmath.mpf(sc[slot]) - r) <= 1e-24 * max(1, abs(r)), (it + 1, key)


def test_pipelined_loop_falls_back_like_the_synchronous_one(pk):
    """The real sphere-packing instance at quad-double with the reference's default thresholds:
    the Cholesky of S_j fails mid-run (iteration ~43) and the LU fallback takes over.  In the
    pipelined loop the failure is seen one body late, with the next body already in flight
    (replayed from the graph that fallback() then drops): that body is waited for before the
    graphs go, both are re-run with LU, and the run ends exactly as the synchronous one --
    same iterations, same LU switch, same log and objectives."""
    from clrsdp_amd import _lib as L
    from clrsdp_amd import sphere_packing as S
    runs = []
    for pipe in (False, True):
        res = S.Nsphere_packing_2point(3, 8, precision_words=4, maxiterations=200, verbose=False,
                                       return_info=True, pipelined=pipe)
        runs.append(res)
    a, c = runs
    ia, ic = a[-1], c[-1]
    assert ia.status == ic.status == "terminated"
    assert ia.factorization & L.FACT_LU_SQ and ic.factorization & L.FACT_LU_SQ
    assert ia.lu_switch == ic.lu_switch > 30
    assert ia.iterations == ic.iterations
    for ra, rc in zip(ia.log, ic.log):
        assert ra[2:] == rc[2:]
    assert a[8] == c[8] and a[9] == c[9]
