"""GPU parity tests: the HIP path (through the C ABI) against the oracle on the same seeded inputs.

Tolerances (stated per precision):
  fp64 stage outputs: 1e-11 relative to the largest entry (or to the input scale for residuals
  that are themselves at round-off level);  double-double: 1e-25 relative against the 256-bit
  oracle on well-conditioned states.  The reference factors S_j and Q with pivoted LU; the GPU
  uses Cholesky + L^-1 (S and Q are SPD), so results agree to conditioning-scaled round-off.
"""
import json
import os

import numpy as np
import pytest

from helpers import (CONFIGS_SMALL, compare_summary, poly_min_instance, rand_spd, rel_err, residual_scales,
                     stage_device, stage_reference)

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL64 = 1e-11


def _blocks(inst, blocks):
    return inst.blocks_to_flat(blocks)


def _oracle_states(oracle, cons, bi, b, iters_before, ar=None, omega=10.0):
    ar = ar or oracle.Fp64()
    prm = {k: oracle._param(ar, v) for k, v in oracle.DEFAULTS.items()}
    state = oracle.initial_point(ar, bi, omega, omega)
    for _ in range(iters_before):
        state, _ = oracle.iteration(ar, cons, bi, b, None, ar.num(0), state, False, prm)
    nxt, it = oracle.iteration(ar, cons, bi, b, None, ar.num(0), state, False, prm)
    return state, nxt, it


def _stage_compare(pk, oracle, cons, b, iters_before=2, words=1, ar=None, tol=TOL64):
    bi = oracle.get_block_info(cons)
    state, nxt, it = _oracle_states(oracle, cons, bi, b, iters_before, ar)
    dev = pk.DeviceSolver(cons, b, pk.get_block_info(cons), precision_words=words)
    try:
        dev.set_state(*state)
        got = stage_device(dev, words > 1)
    finally:
        dev.close()
    ref = stage_reference(it, nxt, bi)
    sc = residual_scales(cons, b, state[1])
    e = {k: rel_err(got[k], ref[k], sc.get(k, 0.0)) for k in ref}
    bad = {k: v for k, v in e.items() if not v <= tol}
    assert not bad, f"stage parity failures: {bad}"
    return e


def _stage_compare_fixture(pk, name, words, tol, bits=256):
    """Stage parity against a precomputed multi-precision oracle fixture
    (tests/golden/make_stage_fixtures.py): sampled entries and linear sketches of every stage
    buffer, scale-aware relative error <= tol."""
    import gzip
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_stage_fixtures",
                                                  os.path.join(GOLDEN, "make_stage_fixtures.py"))
    M = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(M)
    sf = os.path.join(GOLDEN, f"stage_{name}.npz")
    cons, b = M.instance(name, sf)
    bi = pk.get_block_info(cons)
    state = M.load_state(sf, bi)
    with gzip.open(os.path.join(GOLDEN, f"stage_{name}_mp{bits}.json.gz"), "rt") as f:
        fx = json.load(f)
    dev = pk.DeviceSolver(cons, b, bi, precision_words=words)
    try:
        dev.set_state(*state)
        got = stage_device(dev, True)
    finally:
        dev.close()
    sc = residual_scales(cons, b, state[1])
    e = {k: compare_summary(got[k], rec, sc.get(k, 0.0)) for k, rec in fx["buffers"].items()}
    print(name, words, bits, " ".join(f"{k}={v:.1e}" for k, v in e.items()))
    bad = {k: v for k, v in e.items() if not v <= tol}
    assert not bad, f"stage parity failures vs mp{bits}: {bad}"
    return e


CONFIGS_GPU = CONFIGS_SMALL + [
    dict(J=4, delta=20, rank=1, n_y=8),
    dict(J=2, delta=64, rank=2, n_y=64),      # C2 cluster shape (dim_S = 127)
    dict(J=2, delta=128, rank=1, n_y=128),    # C3 cluster shape (dim_S = 255 > on-chip limit)
    dict(J=2, delta=150, rank=1, n_y=140),    # blocks > 128: global-memory factorisation path
]


@pytest.mark.parametrize("cfg", CONFIGS_GPU, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_stage_parity_fp64(pk, oracle, cfg):
    cons, b = pk.synth(seed=3, **cfg)
    _stage_compare(pk, oracle, cons, b)


@pytest.mark.parametrize("cfg", [dict(J=4, delta=20, rank=1, n_y=8), dict(J=2, delta=64, rank=2, n_y=64),
                                 dict(J=3, delta=100, rank=1, n_y=40), dict(J=2, delta=128, rank=1, n_y=128)],
                         ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
@pytest.mark.parametrize("chain", ["0", "1"])
def test_stage_parity_fp64_strip_chains(pk, oracle, cfg, chain, monkeypatch):
    """The strip-chain launches (chain_f64: Z = X^-1 (P Y - R), dY = X^-1 (R - dX Y), the step
    length's L^-1 dM L^-T, U = Z V with the right-hand side's column sums) forced on (1) and off
    (0) for block sizes below one strip (20), not a multiple of the strip (100), rank 2 (no fused
    trace) and the C3 block: every stage against the oracle at the fp64 tolerance."""
    monkeypatch.setenv("CLRSDP_CHAIN", chain)
    cons, b = pk.synth(seed=5, **cfg)
    _stage_compare(pk, oracle, cons, b)


@pytest.mark.parametrize("cfg", [dict(J=2, delta=64, rank=2, n_y=64), dict(J=3, delta=100, rank=1, n_y=40),
                                 dict(J=2, delta=128, rank=1, n_y=128)],
                         ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
@pytest.mark.parametrize("switch", ["CLRSDP_CL_SOLVE", "CLRSDP_CHOL256"])
def test_stage_parity_fp64_opt_in_paths(pk, oracle, cfg, switch, monkeypatch):
    """The opt-in fp64 variants kept in the library (both measured slower or equal at C3, round 5),
    so their kernels and plan wiring cannot break unnoticed: CLRSDP_CL_SOLVE=1 (the cluster block
    solve as cl_solve_t / slab_qsolve / cl_solve_dx, MPMP.jl:1751-1773, instead of four GEMVs) and
    CLRSDP_CHOL256=1 (chol_inv_tiles<256>: S_j of dim_S up to 256 factorised and inverted by one
    768-thread workgroup instead of the 2x2-blocked sequence, with its x4 slab and scratch
    sizing), at dim_S 127, 199 and 255: every stage against the oracle."""
    monkeypatch.setenv(switch, "1")
    cons, b = pk.synth(seed=5, **cfg)
    _stage_compare(pk, oracle, cons, b)


@pytest.mark.parametrize("cfg", CONFIGS_GPU[-3:], ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_stage_parity_fp64_64x64_tiles(pk, oracle, cfg, monkeypatch):
    """The batches of these small instances take the 32x32-tile GEMM (gemm_f64_uni TS = 32);
    the same stages with every uniform batch forced onto the 64x64 tiles the full-size C2/C3
    batches use."""
    monkeypatch.setenv("CLRSDP_GEMM_TS32_BELOW", "0")
    cons, b = pk.synth(seed=3, **cfg)
    _stage_compare(pk, oracle, cons, b)


@pytest.mark.parametrize("cfg", [dict(J=3, delta=4, rank=2, n_y=5), dict(J=2, delta=64, rank=2, n_y=64),
                                 dict(J=3, delta=100, rank=2, n_y=40)],
                         ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
@pytest.mark.parametrize("grp2", ["0", "1", "1-fused"])
def test_stage_parity_fp64_rank2_group_sums(pk, oracle, cfg, grp2, monkeypatch):
    """Rank-2 clusters (C2: every sample a pair of vectors): schur_pairs_f64 summing each 2 x 2
    group of the pairing tile straight into S ("1", the default; K = 14, 254 and 398 -- a partial
    last tile and dim_S 199), the same in schur_fused_f64's epilogue ("1-fused"), against the G
    arena + schur_gsum path ("0"): every stage against the oracle (the 4-term formula,
    MPMP.jl:1373-1398)."""
    monkeypatch.setenv("CLRSDP_SCHUR_GRP2", grp2[0])
    monkeypatch.setenv("CLRSDP_SCHUR_FUSED", "1" if grp2 == "1-fused" else "0")
    cons, b = pk.synth(seed=4, **cfg)
    _stage_compare(pk, oracle, cons, b)


@pytest.mark.parametrize("fused", ["0", "1", "1-ty", "1-multi", "1-pad"])
@pytest.mark.parametrize("cfg", CONFIGS_GPU[-4:-1], ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_stage_parity_fp64_schur_paths(pk, oracle, cfg, fused, monkeypatch):
    """Every Schur path at every stage: schur_fused_f64 with V^T Y formed on chip, one column tile
    per workgroup ("1": what these small batches take by default since round 6), the same with
    all of a row block's tiles per workgroup ("1-multi", the C3 form), the fused kernel reading
    V^T Y from the side-stream GEMM ("1-ty"), and the V^T X^-1 GEMM + schur_pairs_f64 pair ("0").
    At delta <= 64 (the delta-20 and C2-shape cases) "1" is the D64 instance of the one-tile form
    (16 k-chunks) and "1-pad" the same form on the zero-padded 32 chunks."""
    monkeypatch.setenv("CLRSDP_SCHUR_FUSED", fused[0])
    monkeypatch.setenv("CLRSDP_SCHUR_FUSED_D64", "0" if fused == "1-pad" else "1")
    monkeypatch.setenv("CLRSDP_SCHUR_FUSED_Y", "0" if fused == "1-ty" else "1")
    monkeypatch.setenv("CLRSDP_SCHUR_FUSED_ONE", "0" if fused == "1-multi" else "1")
    cons, b = pk.synth(seed=3, **cfg)
    _stage_compare(pk, oracle, cons, b)


def test_schur_fused_matches_unfused(pk, monkeypatch):
    """schur_fused_f64 against the unfused kernels on the C3 cluster shape (K = 255: four row
    blocks, the last one ragged, and the wrapped tile assignment), on rank-2 blocks (G into the
    BX arena, then schur_gsum) and on K = 40 (one row block): S and A_Y agree to fp64 round-off,
    and every S_j the kernel writes directly (rank-1 samples) is exactly symmetric."""
    from clrsdp_amd import _lib as L
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    for cfg in (dict(J=3, delta=128, rank=1, n_y=20), dict(J=2, delta=64, rank=2, n_y=16),
                dict(J=2, delta=40, rank=1, n_y=9)):
        cons, b = pk.synth(seed=11, **cfg)
        bi = pk.get_block_info(cons)
        st = pk.initial_point(bi, 10.0, 10.0)
        out = {}
        for fused in ("1", "0"):
            monkeypatch.setenv("CLRSDP_SCHUR_FUSED", fused)
            dev = pk.DeviceSolver(cons, b, bi)
            try:
                dev.set_state(*st)
                for stage in (L.STAGE_MU_R, L.STAGE_XINV, L.STAGE_SCHUR):
                    dev.run_stage(stage, P, False)
                out[fused] = (np.array(dev.buffer(L.BUF_S, False), dtype=float),
                              np.array(dev.buffer(L.BUF_AY, False), dtype=float))
            finally:
                dev.close()
        for u, v in zip(out["1"], out["0"]):
            assert rel_err(u, v) < 1e-13, (cfg, rel_err(u, v))
        S, off = out["1"][0], 0
        for D in bi.dim_S:
            blk = S[off:off + D * D].reshape(D, D)
            if cfg["rank"] == 1:
                assert np.array_equal(blk, blk.T), cfg
            off += D * D


def test_stage_parity_sphere_packing_shape(pk, oracle):
    """Mixed block sizes 1..18, m = 2 and m = 1 clusters, 2 blocks per cluster (config 5 shape)."""
    cons, b = pk.synth_mixed(**pk.SPHERE_PACKING_SHAPE, seed=1)
    _stage_compare(pk, oracle, cons, b, iters_before=3)


def test_stage_parity_zero_rank_samples(pk, oracle):
    """Samples with rank 0 (nz_k > 0, MPMP.jl:489-491) and unequal ranks."""
    ranks = [[0, 1, 2, 1, 0, 3, 1], [1, 1, 1, 0, 2, 1, 1]]
    cons, b = pk.synth(seed=4, J=2, delta=3, rank=1, n_y=3, m=2, L=2, ranks=ranks, N=7)
    _stage_compare(pk, oracle, cons, b)


def test_stage_parity_dd_vs_256bit(pk, oracle):
    """double-double kernels against the 256-bit oracle."""
    cons, b = pk.synth(seed=3, J=2, delta=4, rank=1, n_y=4)
    ar = oracle.Mp(256)
    consm = [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in Al] for Al in cl.A],
                        ar.asarray(cl.B), ar.asarray(cl.c),
                        [[[ar.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]
    _stage_compare(pk, oracle, consm, ar.asarray(b), words=2, ar=ar, tol=1e-25)


def test_stage_parity_qd_vs_256bit(pk, oracle):
    """quad-double kernels against the 256-bit oracle (qd carries ~212 bits; the state is
    well-conditioned, so 1e-50 leaves three to six orders of magnitude for conditioning)."""
    cons, b = pk.synth(seed=3, J=2, delta=4, rank=1, n_y=4)
    ar = oracle.Mp(256)
    consm = [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in Al] for Al in cl.A],
                        ar.asarray(cl.B), ar.asarray(cl.c),
                        [[[ar.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]
    _stage_compare(pk, oracle, consm, ar.asarray(b), words=4, ar=ar, tol=1e-50)


def test_stage_parity_sphere_packing_shape_qd(pk, oracle):
    """Config 5 (sphere-packing shape: blocks 1..18, dim_S up to 51, n_y = 52) at quad-double
    against the 256-bit oracle."""
    cons, b = pk.synth_mixed(**pk.SPHERE_PACKING_SHAPE, seed=1)
    ar = oracle.Mp(256)
    consm = [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in Al] for Al in cl.A],
                        ar.asarray(cl.B), ar.asarray(cl.c),
                        [[[ar.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]
    _stage_compare(pk, oracle, consm, ar.asarray(b), iters_before=3, words=4, ar=ar, tol=1e-45)


@pytest.mark.parametrize("variant", ["default", "full-pairs", "one-cu-potrf", "valu-products"])
@pytest.mark.parametrize("bits", [128, 256])
def test_stage_parity_dd_c4_shape(pk, bits, variant, monkeypatch):
    """Config 4 at its own cluster shape (J = 2, delta = 64, rank 2, n_y = 64, dim_S = 127,
    blocks of 64) at double-double against the 128- and 256-bit oracle: drives
    potrf_batched<dd> / trsm_batched<dd> (dim_S > 64), chol_inv_reg<dd> and eigmin_lds<dd> at
    n = 64 (MPMP.jl:1433-1465, 762-801, 1829-1898).  dd carries ~106 bits; 1e-25 relative
    (scale-aware) leaves ~6 orders for the conditioning of S_j at this state.  Both forms of the
    Schur pairings: only the upper tiles of V^T X^-1 V, V^T Y V with schur_assemble reading
    (min, max) (the m = 1 default, round 6) and the full products (CLRSDP_MW_PAIR_UPPER=0); both
    factorisations of S_j: the blocked potrf across workgroups (potrf_blk_*, the default above
    n = 64, round 6) and the one-CU chol_lookahead (CLRSDP_POTRF_BLK=0); both forms of the four
    Schur products: on the int8 matrix cores (Ozaki scheme, oz_split / oz_gemm, the double-double
    default for m = 1, round 6) and on the VALU (gemm_valu_ks, CLRSDP_OZAKI=0)."""
    monkeypatch.setenv("CLRSDP_MW_PAIR_UPPER", "0" if variant == "full-pairs" else "1")
    monkeypatch.setenv("CLRSDP_POTRF_BLK", "0" if variant == "one-cu-potrf" else "1")
    monkeypatch.setenv("CLRSDP_OZAKI", "0" if variant == "valu-products" else "1")
    _stage_compare_fixture(pk, "c4dd", 2, 1e-25, bits)


def test_stage_parity_qd_twin(pk):
    """Quad-double twin (J = 2, delta = 32, rank 2, n_y = 32, dim_S = 63): chol_inv_reg<qd> at
    n = 32, potrf_batched<qd> / trsm_batched<qd> at dim_S > 32, eigmin_lds<qd> at n = 32,
    against the 256-bit oracle at 1e-50 relative (qd carries ~212 bits)."""
    _stage_compare_fixture(pk, "qd32", 4, 1e-50, 256)


def _golden(name):
    return json.load(open(os.path.join(GOLDEN, name + ".json")))


@pytest.mark.parametrize("name,words,tol", [("c1_fp64_seed3", 1, 1e-9), ("m2L2_fp64_seed4", 1, 1e-9),
                                            ("c1_mp256_seed3", 1, 1e-9), ("c1_mp256_seed3", 2, 1e-24),
                                            ("rank2_mp256_seed5", 2, 1e-24), ("c1_mp256_seed3", 4, 1e-45),
                                            ("rank2_mp256_seed5", 4, 1e-45), ("sp_mp256_seed1", 1, 1e-8),
                                            ("sp_mp256_seed1", 2, 1e-22), ("sp_mp256_seed1", 4, 1e-40)])
def test_full_run_matches_golden(pk, name, words, tol):
    """solverank1sdp on the GPU reproduces the golden iteration log (mu, alpha_p, alpha_d, beta)."""
    import mpmath
    mpmath.mp.prec = 256
    g = _golden(name)
    inst = dict(g["instance"])
    if inst.pop("kind", None) == "sphere_packing_shape":   # config 5 shape (synth_mixed)
        cons, b = pk.synth_mixed(**pk.SPHERE_PACKING_SHAPE, **inst)
    else:
        cons, b = pk.synth(**inst)
    bi = pk.get_block_info(cons)
    res = pk.solverank1sdp(cons, b, bi, maxiterations=g["iterations"] + 1, precision_words=words,
                           verbose=False, return_info=True, record_exact=True, **g["params"])
    info = res[-1]
    assert len(info.exact) >= len(g["log"]) - 1
    for it, (sc, ref) in enumerate(zip(info.exact, g["log"])):
        for key, slot in (("mu", "mu"), ("alpha_p", "alpha_p"), ("alpha_d", "alpha_d"),
                          ("beta", "beta_c")):
            r = mpmath.mpf(ref[key])
            v = mpmath.mpf(sc[slot])
            assert abs(v - r) <= tol * max(1, abs(r)), (it + 1, key, float(v), float(r))
        # the objectives after this iteration's update are the next log row's (MPMP.jl:940-941)
        if it + 1 < len(g["log"]):
            for key in ("p_obj", "d_obj"):
                r = mpmath.mpf(g["log"][it + 1][key])
                v = mpmath.mpf(sc[key])
                assert abs(v - r) <= tol * max(1, abs(r)), (it + 1, key, float(v), float(r))
    # the returned gap and objectives of the final state (MPMP.jl:1021-1023), at the state's
    # precision when words > 1 (mpmath numbers, not leading limbs)
    if "final" in g and len(info.exact) == len(g["log"]):
        if words > 1:
            assert all(isinstance(v, mpmath.mpf) for v in res[7:10])
        for v, key in zip(res[7:10], ("gap", "p_obj", "d_obj")):
            r = mpmath.mpf(g["final"][key])
            assert abs(mpmath.mpf(v) - r) <= tol * max(1, abs(r)), (key, float(v), float(r))


def test_known_answer_polynomial_minimum_gpu(pk):
    cons, b, pmin = poly_min_instance(pk)
    bi = pk.get_block_info(cons)
    # fp64 Cholesky of S breaks down one or two iterations earlier than the reference's pivoted
    # LU near optimality (S becomes numerically semidefinite), so stop at a 1e-8 gap here.
    res = pk.solverank1sdp(cons, b, bi, omega_p=10.0, omega_d=10.0, maxiterations=100,
                           duality_gap_threshold=1e-8, primal_error_threshold=1e-8,
                           dual_error_threshold=1e-8, verbose=True, return_info=True)
    assert res[-1].status == "terminated"
    assert abs(res[9] - pmin) < 1e-7 and abs(res[8] - pmin) < 1e-7


def test_iterate_equals_stagewise(pk):
    """clrsdp_iterate == the ten stages run one by one (bitwise)."""
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=9, J=3, delta=6, rank=1, n_y=5, m=2)
    bi = pk.get_block_info(cons)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    st0 = pk.initial_point(bi, 10.0, 10.0)
    outs = []
    for mode in ("iterate", "stages"):
        dev = pk.DeviceSolver(cons, b, bi)
        dev.set_state(*st0)
        for _ in range(3):
            if mode == "iterate":
                dev.iterate(P, False)
            else:
                for s in range(L.NUM_STAGES):
                    dev.run_stage(s, P, False)
        outs.append(dev.get_state())
        dev.close()
    a, c = outs
    assert np.array_equal(a[0], c[0]) and np.array_equal(a[2], c[2])
    for j in range(bi.J):
        assert np.array_equal(a[1][j][0], c[1][j][0])


def test_live_schur_timing_keeps_iterates_bitwise(pk):
    """Timing mode 2 (device-clock stamps inside the replayed graph, clrsdp_set_timing) reports a
    positive Schur time and changes nothing else: iterates equal the untimed run bitwise."""
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=4, J=8, delta=32, rank=1, n_y=16)
    bi = pk.get_block_info(cons)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    st0 = pk.initial_point(bi, 10.0, 10.0)
    outs, schur = [], []
    for timing in (0, 2):
        dev = pk.DeviceSolver(cons, b, bi)
        dev.set_timing(timing)
        dev.set_state(*st0)
        for _ in range(3):
            st = dev.iterate(P, False)
            schur.append(st.phase_ms[L.STAGE_SCHUR])
        outs.append(dev.get_state())
        dev.close()
    assert all(t > 0 for t in schur[3:]) and all(t < 1e3 for t in schur[3:])
    a, c = outs
    assert np.array_equal(a[0], c[0]) and np.array_equal(a[2], c[2])
    for j in range(bi.J):
        assert np.array_equal(a[1][j][0], c[1][j][0])
        assert np.array_equal(a[3][j], c[3][j])


@pytest.mark.parametrize("fallback", [False, True])
def test_not_positive_definite_reports_error(pk, fallback):
    """X not PD: spd_inv! fails (CLRSDP_E_NOT_PD_X, MPMP.jl:774-797).  With the default LU
    fallback X^-1 comes from approx_inv! instead and the step length's cho!(X) fails, as in the
    reference (CLRSDP_E_STEP, MPMP.jl:1846-1882)."""
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=9, J=2, delta=4, rank=1, n_y=3)
    bi = pk.get_block_info(cons)
    x, X, y, Y = pk.initial_point(bi, 10.0, 10.0)
    X[1][0][2, 2] = -5.0
    dev = pk.DeviceSolver(cons, b, bi)
    if not fallback:
        dev.set_factorization(0)
    dev.set_state(x, X, y, Y)
    with pytest.raises(L.ClrsdpError) as ei:
        dev.iterate(pk.make_params("0.3", "0.1", "0.7", 0), False)
    assert ei.value.code == (L.E_STEP if fallback else L.E_NOT_PD_X)
    assert dev.factorization == (L.FACT_FALLBACK | L.FACT_LU_X if fallback else 0)
    dev.close()


def _newton_identities(pk, oracle, dev, cons, b, bi, words, what):
    """The Newton-system identities of the direction in the device buffers: B^T dx = p,
    Tr(A_* dY) + B dy = d, dX = P + sum dx_i A_i (MPMP.jl:1741-1786)."""
    from clrsdp_amd import _lib as L
    from clrsdp_amd import instance as inst
    ar = oracle.Fp64()
    dx, dy = dev.buffer(L.BUF_DX), dev.buffer(L.BUF_DY)
    dY = inst.flat_to_blocks(dev.buffer(L.BUF_DYMAT), bi)
    dX = inst.flat_to_blocks(dev.buffer(L.BUF_DXMAT), bi)
    Pm = inst.flat_to_blocks(dev.buffer(L.BUF_P), bi)
    p, d = dev.buffer(L.BUF_PVEC), dev.buffer(L.BUF_DVEC)
    Bst = oracle.stack_B(cons)
    assert rel_err(Bst.T @ dx, p, np.abs(b).max()) < 1e-9, what
    if words > 1:
        import mpmath
        # (decimal strings: np.longdouble(mpf) would round through a double)
        dxl = np.array([np.longdouble(mpmath.nstr(v, 30)) for v in dev.buffer(L.BUF_DX, exact=True)])
        pl = np.array([np.longdouble(mpmath.nstr(v, 30)) for v in dev.buffer(L.BUF_PVEC, exact=True)])
        r = Bst.astype(np.longdouble).T @ dxl - pl
        assert float(np.max(np.abs(r))) / float(np.abs(b).max()) < 1e-16, what
    lhs = oracle.trace_A(ar, cons, dY, bi) + Bst @ dy
    assert rel_err(lhs, d, np.abs(oracle.stack_c(cons)).max()) < 1e-8, what
    WA = oracle.compute_weighted_A(ar, cons, dx, bi)
    for j in range(0, bi.J, 5):
        assert rel_err(dX[j][0], WA[j][0] + Pm[j][0]) < 1e-12, what
    return dX, dY


def _full_size_iteration_checks(pk, oracle, cons, b, words=1, gamma=0.7, bitwise_sym=False):
    """One GPU iteration of a full-size instance, stage by stage, through size-independent
    properties (MPMP.jl:755-887):
      * S symmetric after SCHUR (bitwise on the fused rank-1 path, round-off otherwise);
      * the predictor's and the corrector's Newton identities (_newton_identities);
      * STEP: alpha_p, alpha_d in (0, 1]; lambda_min of L^-1 dM L^-T of every block recomputed on
        the host (scipy eigh of the pencil (dM, M), the same spectrum) and the device's minimum
        over blocks equal to it to 1e-10 relative; alpha = min(1, -gamma/lambda_min)
        (MPMP.jl:1893-1897) to 1e-10;
      * UPDATE: X + alpha_p dX and Y + alpha_d dY, and both Cholesky-factorisable."""
    import scipy.linalg as sla
    from clrsdp_amd import _lib as L
    bi = pk.get_block_info(cons)
    dev = pk.DeviceSolver(cons, b, bi, precision_words=words)
    try:
        P = pk.make_params("0.3", "0.1", str(gamma), 0)
        dev.set_state(*pk.initial_point(bi, 100.0, 100.0))
        for _ in range(2):
            dev.iterate(P, False)
        _, Xs, _, Ys = dev.get_state()
        for s in (L.STAGE_MU_R, L.STAGE_XINV, L.STAGE_SCHUR):
            dev.run_stage(s, P, False)
        S = dev.buffer(L.BUF_S)
        # On the fused rank-1 path the device assembles S_j's lower triangle only and
        # clrsdp_get_buffer mirrors it for the host, so a symmetry check of the returned S says
        # nothing about the device: instead the lower triangle of S_0 and S_{J-1} against the
        # host's (Lambda V^T X^-1 V Lambda) o (V^T Y V) (compute_S_integrated at m = 1,
        # MPMP.jl:1272-1318, 1373-1398) with X^-1 from numpy
        ar = oracle.Fp64()
        off = 0
        for j in range(bi.J):
            D = bi.dim_S[j]
            if j in (0, bi.J - 1) and bi.m[j] == 1 and bi.L[j] == 1:
                Sj = np.asarray(S[off:off + D * D], dtype=float).reshape(D, D, order="F")
                V, lam, ks = oracle.vectors_matrix(ar, cons[j], 0)
                V, lam = np.asarray(V, dtype=float), np.asarray(lam, dtype=float)
                BX = V.T @ np.linalg.inv(np.asarray(Xs[j][0], dtype=float)) @ V
                BY = V.T @ np.asarray(Ys[j][0], dtype=float) @ V
                G = np.outer(lam, lam) * BX * BY
                Pk = np.zeros((len(lam), D))
                Pk[np.arange(len(lam)), np.asarray(ks)] = 1.0
                Sref = Pk.T @ G @ Pk
                il = np.tril_indices(D)
                err = np.max(np.abs(Sj[il] - Sref[il])) / np.max(np.abs(Sref))
                assert err < 1e-10, (j, err)
                if bitwise_sym:  # (the host mirror of the lower triangle)
                    assert np.array_equal(Sj, Sj.T)
            off += D * D
        for s in (L.STAGE_FACTOR, L.STAGE_RESIDUALS, L.STAGE_PREDICTOR):
            dev.run_stage(s, P, False)
        _newton_identities(pk, oracle, dev, cons, b, bi, words, "predictor")
        for s in (L.STAGE_CORRECTOR_R, L.STAGE_CORRECTOR):
            dev.run_stage(s, P, False)
        dX, dY = _newton_identities(pk, oracle, dev, cons, b, bi, words, "corrector")
        _, X, _, Y = dev.get_state()
        dev.run_stage(L.STAGE_STEP, P, False)
        sc = dev.buffer(L.BUF_SCALARS)
        a_p, a_d = float(sc[L.SC["alpha_p"]]), float(sc[L.SC["alpha_d"]])
        assert 0.0 < a_p <= 1.0 and 0.0 < a_d <= 1.0, (a_p, a_d)
        for M, dM, key, a in ((X, dX, "mineig_X", a_p), (Y, dY, "mineig_Y", a_d)):
            lam = [sla.eigh(dM[j][l], M[j][l], eigvals_only=True)[0]
                   for j in range(bi.J) for l in range(len(M[j]))]
            ref = min(lam)
            scale = max(abs(v) for v in lam)
            got = float(sc[L.SC[key]])
            assert abs(got - ref) <= 1e-10 * scale, (key, got, ref)
            a_ref = 1.0 if ref > -gamma else -gamma / ref
            assert abs(a - a_ref) <= 1e-10 * a_ref, (key, a, a_ref)
        dev.run_stage(L.STAGE_UPDATE, P, False)
        _, X1, _, Y1 = dev.get_state()
        for M, dM, M1, a in ((X, dX, X1, a_p), (Y, dY, Y1, a_d)):
            for j in range(bi.J):
                for l in range(len(M[j])):
                    assert rel_err(M1[j][l], M[j][l] + a * dM[j][l]) < 1e-13
                    np.linalg.cholesky(np.asarray(M1[j][l], dtype=float))
        return a_p, a_d
    finally:
        dev.close()


def test_c3_full_size_newton_identities(pk, oracle):
    """At the bench size (64 clusters x 128x128 blocks, rank 1, n_y = 128) one GPU iteration
    through every stage: S symmetric (bitwise), the predictor's and the corrector's Newton
    identities, the step lengths against the host's lambda_min of every block's L^-1 dM L^-T,
    and the updated X, Y positive definite (_full_size_iteration_checks)."""
    cons, b = pk.synth(seed=0, J=64, delta=128, rank=1, n_y=128)
    a_p, a_d = _full_size_iteration_checks(pk, oracle, cons, b, bitwise_sym=True)
    print("C3 alpha_p", a_p, "alpha_d", a_d)


def _sp_real_deviation(pk, words):
    """Per-iteration relative deviation of the GPU run on the real sphere-packing instance
    (prepareabc at 512 bits, SP.jl:29-105) from the 256-bit oracle log."""
    import mpmath
    from clrsdp_amd import sphere_packing as S
    g = _golden("sp_real_d8_mp256")
    inst = g["instance"]
    cons, b, bi = S.sphere_packing_constraints(inst["n"], inst["d"], prec=512)
    res = pk.solverank1sdp(cons, b, bi, maxiterations=g["iterations"] + 1, precision_words=words,
                           verbose=False, return_info=True, record_exact=True, **g["params"])
    info = res[-1]
    dev = []
    with mpmath.workprec(256):
        for sc, ref in zip(info.exact, g["log"]):
            dev.append(max(abs(mpmath.mpf(sc[s]) - mpmath.mpf(ref[k])) / max(1, abs(mpmath.mpf(ref[k])))
                           for k, s in (("mu", "mu"), ("alpha_p", "alpha_p"),
                                        ("alpha_d", "alpha_d"), ("beta", "beta_c"))))
    return dev, len(g["log"])


def test_sphere_packing_real_instance_qd_matches_256bit_log(pk):
    """Config 5 with the real constraint data at quad-double against the 256-bit oracle log.
    The instance is ill-conditioned (cond S_j ~ 1e23 at the start, Q worse, growing as mu -> 0):
    the 212-bit mpmath oracle itself deviates from the 256-bit log by 1.9e-31 / 4.3e-30 / 5.9e-30
    at iterations 1-3 (measured), so qd (~212 bits) is held to the same class: 1e-29 through
    iteration 12, 1e-17 through 25, 1e-13 through 30.  The reference runs it at 512 bits
    (SP.jl:30-31)."""
    dev, n = _sp_real_deviation(pk, 4)
    print("deviation per iteration:", " ".join("%.1e" % float(d) for d in dev))
    assert len(dev) >= 30
    assert max(dev[:12]) < 1e-29, dev[:12]
    assert max(dev[:25]) < 1e-17, dev[:25]
    assert max(dev[:30]) < 1e-13, dev[:30]


def test_sphere_packing_bound_qd(pk):
    """Application anchor at the reference's own settings: SP.jl:110 calls solverank1sdp with its
    default thresholds (gap 1e-15, errors 1e-30, MPMP.jl:606-611).  At quad-double the Cholesky
    of S_j breaks down near iteration 43 (gap ~2e-6); the LU fallback (approx_lu!, the reference's
    factorisation) takes over and the run terminates at the optimum.  The bound lies between the
    NaCl density 0.793 and de Laat et al.'s 0.813-class value (SP.jl:124-127); the 256-bit oracle's
    iterate at gap 1.6e-5 (iteration 40, tests/golden) brackets it, and the 256-bit oracle run to
    termination (91 iterations, gap 2.4e-22, sp_real_d8_mp256_full) pins it to 1e-13."""
    from clrsdp_amd import _lib as L
    from clrsdp_amd import sphere_packing as S
    res = S.Nsphere_packing_2point(3, 8, precision_words=4, maxiterations=200, verbose=False,
                                   return_info=True)
    info = res[-1]
    print("status", info.status, "iterations", info.iterations, "LU from", info.lu_switch,
          "gap", res[7], "bound", -res[9])
    assert info.status == "terminated"
    assert res[7] < 1e-15
    assert info.factorization & L.FACT_LU_SQ and info.lu_switch > 30
    bound = -res[9]
    assert S.NACL_DENSITY < bound < 0.82
    g = _golden("sp_real_d8_mp256")["log"][-1]
    lo, hi = sorted((-float(g["p_obj"]), -float(g["d_obj"])))
    assert lo - 1e-9 <= float(bound) <= hi + 1e-9, (float(bound), lo, hi)
    full = _golden("sp_real_d8_mp256_full")
    assert full["status"] == "terminated"
    ref = -float(full["final"]["p_obj"])
    assert abs(float(bound) - ref) < 1e-13 * ref, (float(bound), ref)


def test_fp64_reaches_where_the_oracle_stops(pk, oracle):
    """At fp64 with the reference's default thresholds the pivoted-LU oracle (as approx_lu!)
    itself stops with a singular factorisation near gap 1e-10 (the reference's "S was not
    decomposed" outcome, MPMP.jl:1439).  The device run gets at least as far: every iteration
    the oracle completed also completes here, at a gap no worse than the oracle's."""
    cons, b, pmin = poly_min_instance(pk)
    bi = oracle.get_block_info(cons)
    import warnings
    # the last maxiterations at which the oracle still returns (it raises one iteration later)
    k, last = 0, None
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for n in range(5, 100):
            try:
                r = oracle.solverank1sdp(cons, b, bi, maxiterations=n, omega_p=10.0, omega_d=10.0)
            except Exception:
                break
            k, last = n - 1, r
    assert 10 < k < 98
    res = pk.solverank1sdp(cons, b, pk.get_block_info(cons), omega_p=10.0, omega_d=10.0,
                           maxiterations=k + 1, verbose=False, return_info=True)
    assert res[-1].iterations == k
    assert res[7] <= 10 * float(last.gap) + 1e-12, (res[7], float(last.gap))
    assert abs(res[9] - pmin) < 1e-7


@pytest.mark.parametrize("words,maxit", [(1, 100), (1, 5), (2, 100)])
def test_pipelined_loop_equals_synchronous(pk, words, maxit):
    """The pipelined host loop (device-side pd_feas / terminate, host one body behind) gives
    the same log, iterates, residuals and objectives as the synchronous loop, bit for bit,
    whether it stops by termination (the speculative body is skipped) or by maxiterations."""
    cons, b = pk.synth(J=3, delta=5, rank=1, n_y=4, seed=7, m=2, L=2)
    bi = pk.get_block_info(cons)
    # thresholds well above the fp64 Cholesky breakdown near optimality
    kw = dict(omega_p=10.0, omega_d=10.0, duality_gap_threshold=1e-6, primal_error_threshold=1e-6,
              dual_error_threshold=1e-6, maxiterations=maxit, precision_words=words,
              verbose=False, return_info=True)
    a = pk.solverank1sdp(cons, b, bi, pipelined=False, **kw)
    p = pk.solverank1sdp(cons, b, bi, pipelined=True, **kw)
    assert a[-1].status == p[-1].status and a[-1].iterations == p[-1].iterations
    if maxit == 100:
        assert a[-1].status == "terminated"
    assert [r[2:] for r in a[-1].log] == [r[2:] for r in p[-1].log]
    assert np.array_equal(a[0], p[0]) and np.array_equal(a[2], p[2])
    for i in (1, 3, 4):   # X, Y, P blocks
        assert all(np.array_equal(u, v) for bu, bv in zip(a[i], p[i]) for u, v in zip(bu, bv))
    assert np.array_equal(a[5], p[5]) and np.array_equal(a[6], p[6])
    assert a[7:10] == p[7:10]


def test_save_restore_state_replays_bitwise(pk):
    """clrsdp_save_state / clrsdp_restore_state: after a restore the same loop bodies give the
    same log rows and iterates bit for bit (graph replay and eager enqueue alike)."""
    cons, b = pk.synth(seed=4, J=3, delta=8, rank=1, n_y=5, m=1)
    bi = pk.get_block_info(cons)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    dev = pk.DeviceSolver(cons, b, bi)
    dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
    dev.initial_residuals(P)
    for _ in range(3):
        dev.iterate(P, False)
    dev.save_state()
    runs = []
    for _ in range(2):
        rows = [tuple(getattr(st, f) for f in ("mu", "alpha_p", "alpha_d", "p_obj", "d_obj", "P_err"))
                for st in (dev.iterate(P, False) for _ in range(3))]
        x, X, y, Y = dev.get_state()
        runs.append((rows, x, y))
        dev.restore_state()
    dev.close()
    assert runs[0][0] == runs[1][0]
    assert np.array_equal(runs[0][1], runs[1][1]) and np.array_equal(runs[0][2], runs[1][2])


@pytest.mark.parametrize("words", [1, 2])
def test_c2_c4_full_size_newton_identities(pk, oracle, words):
    """Config 2 (fp64) and config 4 (the C2 instance at double-double) at their full size (16
    clusters x 64x64 blocks, rank 2, n_y = 64): the checks of the C3 test through every stage.
    At double-double B^T dx = p is checked in extended precision (longdouble, all limbs of dx)
    to 1e-16, below what an fp64 solve reaches; the trace, weighted-A and step-length checks use
    fp64 (the leading limbs).  (Rank 2: the rank-group sums of the general pairing leave S
    symmetric to round-off, not bitwise as the fused rank-1 path of C3.)"""
    cons, b = pk.synth(seed=0, J=16, delta=64, rank=2, n_y=64)
    a_p, a_d = _full_size_iteration_checks(pk, oracle, cons, b, words)
    print("C2/C4 words", words, "alpha_p", a_p, "alpha_d", a_d)


@pytest.mark.parametrize("delta", [18, 40])
def test_chol_lookahead_qd_one_newton_step(pk, delta):
    """X^-1 at quad-double (STAGE_XINV: chol_lookahead's LDL^T factor and L^-1 with the default
    CLRSDP_LA_OPTS = 2, i.e. ONE Newton step for the pivot reciprocal, ~2^-208 relative instead of
    chol_packed's ~2^-212; then L^-T L^-1) against the 320-bit inverse of the same exactly
    representable X: the factor is no longer bitwise chol_packed's, so this pins it to a stated
    tolerance, 1e-56 of max|X^-1| (qd eps ~1.5e-64, pivot ~2.4e-63, times n cond(X)).  delta 18
    takes the 4-wave instance (n <= 32), 40 the 16-wave one (n <= 64)."""
    import mpmath
    from clrsdp_amd import _lib as L
    cons, b = pk.synth(seed=12, J=2, delta=delta, rank=1, n_y=3)
    bi = pk.get_block_info(cons)
    rng = np.random.default_rng(delta)
    x, X, y, Y = pk.initial_point(bi, 10.0, 10.0)
    X = [[rand_spd(n, rng, 0.5) for n in bj] for bj in bi.Y_blocksizes]
    dev = pk.DeviceSolver(cons, b, bi, precision_words=4)
    try:
        dev.set_state(x, X, y, Y)
        P = pk.make_params("0.3", "0.1", "0.7", 0)
        for s in (L.STAGE_MU_R, L.STAGE_XINV):
            dev.run_stage(s, P, False)
        Xi = dev.buffer(L.BUF_XINV, exact=True)
    finally:
        dev.close()
    off = 0
    with mpmath.workprec(320):
        for j in range(bi.J):
            n = bi.Y_blocksizes[j][0]
            ref = mpmath.inverse(mpmath.matrix([[mpmath.mpf(float(v)) for v in row] for row in X[j][0]]))
            got = Xi[off:off + n * n]
            nrm = max(abs(ref[i, k]) for i in range(n) for k in range(n))
            err = max(abs(mpmath.mpf(got[i + n * k]) - ref[i, k]) for i in range(n) for k in range(n))
            assert err / nrm < 1e-56, (j, float(err / nrm))
            off += n * n


def test_failed_capture_falls_back_eagerly(pk, monkeypatch):
    """A loop body whose graph capture fails half-way (injected after FACTOR forked the side
    streams and set its pending flags: CLRSDP_INJECT_CAPTURE_FAIL, the sharded path's fallback
    taken at one rank) is re-enqueued eagerly with the per-body state reset; three loop bodies then
    give bitwise the iterates of a handle whose captures succeed."""
    cons, b = pk.synth(seed=3, J=4, delta=20, rank=1, n_y=8)
    bi = pk.get_block_info(cons)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    outs = []
    for inj in ("0", "1"):
        monkeypatch.setenv("CLRSDP_INJECT_CAPTURE_FAIL", inj)
        dev = pk.DeviceSolver(cons, b, bi)
        try:
            dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
            for _ in range(3):
                dev.iterate(P, False)
            x, X, y, Y = dev.get_state()
            outs.append(np.concatenate([np.ravel(x), np.ravel(y)] +
                                       [np.ravel(m) for bj in X + Y for m in bj]))
        finally:
            dev.close()
    assert np.array_equal(outs[0], outs[1])


def test_overlapped_step_length_equals_joint(pk, monkeypatch):
    """CLRSDP_XY_OVERLAP=1 (small batches): the X step length (its congruence and eigen launch)
    on the side stream from the corrector's dX on, beside dY and the Y step length; the same
    kernels per block, so five loop bodies give bitwise the iterates of the joint launches."""
    cons, b = pk.synth(seed=6, J=3, delta=128, rank=1, n_y=16)
    bi = pk.get_block_info(cons)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    outs = []
    for ov in ("0", "1"):
        monkeypatch.setenv("CLRSDP_XY_OVERLAP", ov)
        dev = pk.DeviceSolver(cons, b, bi)
        try:
            dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
            for _ in range(5):
                st = dev.iterate(P, False)
            x, X, y, Y = dev.get_state()
            outs.append((np.concatenate([np.ravel(x), np.ravel(y)] +
                                        [np.ravel(m) for bj in X + Y for m in bj]),
                         st.alpha_p, st.alpha_d))
        finally:
            dev.close()
    assert np.array_equal(outs[0][0], outs[1][0])
    assert outs[0][1:] == outs[1][1:]
