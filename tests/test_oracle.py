"""CPU tests of the oracle (oracle/mpmp_oracle.py) against exact identities, known answers and the
committed golden vectors -- the reference ships none of its own, so this is what
anchors the restatement ("parity unpinned" w.r.t. the Julia reference itself)."""
import json
import os

import numpy as np
import pytest

from helpers import CONFIGS_SMALL, dense_A, poly_min_instance, rand_spd, rel_err

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _random_state(bi, rng):
    X = [[rand_spd(n, rng) for n in bj] for bj in bi.Y_blocksizes]
    Y = [[rand_spd(n, rng) for n in bj] for bj in bi.Y_blocksizes]
    return X, Y


@pytest.mark.parametrize("cfg", CONFIGS_SMALL)
def test_schur_equals_dense_trace_formula(pk, oracle, cfg):
    """S_ij = Tr(A_i X^-1 A_j Y) summed over blocks (what MPMP.jl:1335-1406 assembles)."""
    cons, b = pk.synth(seed=5, **cfg)
    bi = oracle.get_block_info(cons)
    rng = np.random.default_rng(0)
    X, Y = _random_state(bi, rng)
    ar = oracle.Fp64()
    Xi = oracle.xinv(ar, X)
    S, AY = oracle.compute_S_integrated(ar, cons, Xi, Y, bi)
    for j in range(bi.J):
        D = bi.dim_S[j]
        As = [dense_A(cons[j], bi, j, t) for t in range(D)]
        Sd = np.zeros((D, D))
        for a in range(D):
            for c in range(D):
                Sd[a, c] = sum(np.trace(As[a][l] @ Xi[j][l] @ As[c][l] @ Y[j][l])
                               for l in range(bi.L[j]))
        assert rel_err(S[j], Sd) < 1e-12
        assert np.allclose(S[j], S[j].T, rtol=0, atol=1e-14 * np.abs(S[j]).max())


@pytest.mark.parametrize("cfg", CONFIGS_SMALL)
def test_trace_and_weighted_A_are_adjoint(pk, oracle, cfg):
    """<sum_i a_i A_i, Z> = a . Tr(A_* Z)  (MPMP.jl:1517-1584 vs 1621-1678), and both match the
    dense constraint matrices; the A_Y shortcut (1585-1618) equals trace_A(Y)."""
    cons, b = pk.synth(seed=6, **cfg)
    bi = oracle.get_block_info(cons)
    rng = np.random.default_rng(1)
    ar = oracle.Fp64()
    Z = [[(lambda M: (M + M.T) / 2)(rng.standard_normal((n, n))) for n in bj]
         for bj in bi.Y_blocksizes]
    a = rng.standard_normal(sum(bi.dim_S))
    tr = oracle.trace_A(ar, cons, Z, bi)
    W = oracle.compute_weighted_A(ar, cons, a, bi)
    lhs = sum(np.sum(W[j][l] * Z[j][l]) for j in range(bi.J) for l in range(bi.L[j]))
    assert abs(lhs - a @ tr) < 1e-11 * (1 + abs(lhs))
    for j in range(bi.J):
        for t in range(bi.dim_S[j]):
            Ad = dense_A(cons[j], bi, j, t)
            ref = sum(np.sum(Ad[l] * Z[j][l]) for l in range(bi.L[j]))
            assert abs(tr[bi.x_indices[j] + t] - ref) < 1e-12 * (1 + abs(ref))
    X, Y = _random_state(bi, rng)
    _, AY = oracle.compute_S_integrated(ar, cons, oracle.xinv(ar, X), Y, bi)
    assert rel_err(oracle.trace_A_AY(ar, cons, AY, bi), oracle.trace_A(ar, cons, Y, bi)) < 1e-13


@pytest.mark.parametrize("cfg", CONFIGS_SMALL)
def test_search_direction_solves_newton_system(pk, oracle, cfg):
    """The 3-stage block solve (MPMP.jl:1743-1776) gives B^T dx = p and
    Tr(A_* dY) + B dy = d; dX = P + sum dx_i A_i (1779-1786)."""
    cons, b = pk.synth(seed=7, **cfg)
    bi = oracle.get_block_info(cons)
    ar = oracle.Fp64()
    prm = {k: oracle._param(ar, v) for k, v in oracle.DEFAULTS.items()}
    st = oracle.initial_point(ar, bi, 10.0, 10.0)
    st, _ = oracle.iteration(ar, cons, bi, b, None, 0.0, st, False, prm)
    _, it = oracle.iteration(ar, cons, bi, b, None, 0.0, st, False, prm)
    for key in ("pred", "corr"):
        dx, dX, dy, dY = it[key]
        Bst = oracle.stack_B(cons)
        assert rel_err(Bst.T @ dx, it["p"], np.abs(b).max()) < 1e-10
        lhs = oracle.trace_A(ar, cons, dY, bi) + Bst @ dy
        assert rel_err(lhs, it["d"], np.abs(oracle.stack_c(cons)).max()) < 1e-9
        WA = oracle.compute_weighted_A(ar, cons, dx, bi)
        for j in range(bi.J):
            for l in range(bi.L[j]):
                assert rel_err(dX[j][l], WA[j][l] + it["P"][j][l]) < 1e-13


def test_known_answer_polynomial_minimum(pk, oracle):
    """max y s.t. p(x) - y is SOS: the IPM (fp64) converges to min_x p(x)."""
    cons, b, pmin = poly_min_instance(pk)
    bi = oracle.get_block_info(cons)
    res = oracle.solverank1sdp(cons, b, bi, omega_p=10.0, omega_d=10.0, maxiterations=100,
                               duality_gap_threshold=1e-10, primal_error_threshold=1e-10,
                               dual_error_threshold=1e-10)
    assert res.status == "terminated"
    assert abs(float(res.d_obj) - pmin) < 1e-8
    assert abs(float(res.p_obj) - pmin) < 1e-8


def test_known_answer_polynomial_minimum_mp(pk, oracle):
    """Same at 128 bits: the multiprecision backend reaches a far smaller gap."""
    import mpmath
    cons, b, pmin = poly_min_instance(pk)
    ar = oracle.Mp(128)
    consm = [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in cl.A[0]]], ar.asarray(cl.B),
                        ar.asarray(cl.c), [[[ar.num(x) for x in hk] for hk in cl.H[0]]])
             for cl in cons]
    bi = oracle.get_block_info(consm)
    res = oracle.solverank1sdp(consm, b, bi, ar=ar, omega_p=10.0, omega_d=10.0, maxiterations=60,
                               duality_gap_threshold="1e-20", primal_error_threshold="1e-20",
                               dual_error_threshold="1e-20")
    assert res.status == "terminated"
    assert abs(float(res.d_obj) - pmin) < 1e-12


def test_mp_backend_agrees_with_fp64(pk, oracle):
    """One loop body at 200 bits vs fp64 on a well-conditioned state."""
    cons, b = pk.synth(seed=8, J=2, delta=3, rank=1, n_y=3, m=2, L=1)
    bi = oracle.get_block_info(cons)
    a64 = oracle.Fp64()
    amp = oracle.Mp(200)
    prm64 = {k: oracle._param(a64, v) for k, v in oracle.DEFAULTS.items()}
    prmmp = {k: oracle._param(amp, v) for k, v in oracle.DEFAULTS.items()}
    consm = [pk.Cluster([[[amp.asarray(v) for v in vk] for vk in Al] for Al in cl.A],
                        amp.asarray(cl.B), amp.asarray(cl.c),
                        [[[amp.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]
    s64 = oracle.initial_point(a64, bi, 10.0, 10.0)
    smp = oracle.initial_point(amp, bi, 10.0, 10.0)
    s64, i64 = oracle.iteration(a64, cons, bi, b, None, 0.0, s64, False, prm64)
    smp, imp = oracle.iteration(amp, consm, bi, amp.asarray(b), None, amp.num(0), smp, False, prmmp)
    assert rel_err(np.array(smp[0], dtype=float), s64[0]) < 1e-12
    assert abs(float(imp["alpha_p"]) - i64["alpha_p"]) < 1e-12
    assert abs(float(imp["mu"]) - i64["mu"]) < 1e-12 * abs(i64["mu"])


def test_block_info_and_balancer(pk, oracle):
    cons, b = pk.synth(seed=1, J=3, delta=4, rank=1, n_y=2, m=2, L=2,
                       ranks=[[1, 0, 2, 1, 1, 1, 1], [2, 2, 0, 1, 1, 1, 1]])
    bo = oracle.get_block_info(cons)
    bp = pk.get_block_info(cons)
    for f in ("J", "n_y", "m", "L", "n_samples", "Y_blocksizes", "dim_S", "ranks", "x_indices",
              "rank_sums", "nz_k", "jl_pairs"):
        assert getattr(bo, f) == getattr(bp, f), f
    assert bp.dim_S == [3 * 7] * 3
    assert bp.rank_sums[0][0] == [0, 1, 1, 3, 4, 5, 6, 7]
    assert bp.nz_k[0][1] == 0 and bp.Y_blocksizes[0] == [8, 8]
    # balancer: partition, improves the initial contiguous split (MPMP.jl:425-465)
    w = [100, 1, 1, 1, 50, 50, 2, 2]
    sets, sw = pk.distribute_weights_swapping(w, 3)
    assert sorted(i for s in sets for i in s) == list(range(len(w)))
    assert max(sw) <= max(sum(w[0:3]), sum(w[3:6]), sum(w[6:8]))
    assert sets == oracle.distribute_weights_swapping(w, 3)[0]


@pytest.mark.parametrize("name", ["c1_fp64_seed3", "m2L2_fp64_seed4", "c1_mp256_seed3"])
def test_golden_vectors(pk, oracle, name):
    """The oracle reproduces the committed golden vectors (tests/golden/make_golden.py)."""
    path = os.path.join(GOLDEN, name + ".json")
    g = json.load(open(path))
    cons, b = pk.synth(**g["instance"])
    bi = oracle.get_block_info(cons)
    ar = oracle.Fp64()
    res = oracle.solverank1sdp(cons, b, bi, ar=ar, maxiterations=g["iterations"] + 1,
                               **g["params"])
    tol = g["tolerance_fp64"]
    for row, ref in zip(res.log, g["log"]):
        for key in ("mu", "alpha_p", "alpha_d", "beta"):
            assert abs(float(getattr(row, key)) - float(ref[key])) <= tol * max(1.0, abs(float(ref[key]))), key
    assert rel_err(res.x, np.array([float(v) for v in g["x"]])) < tol


def test_sphere_packing_golden_runs_are_consistent():
    """The two 256-bit oracle runs on the real sphere-packing instance (40 iterations, and to
    termination at the reference's default thresholds) share their first 40 log rows exactly, and
    the terminated run satisfies the stopping rule (MPMP.jl:734-742): gap < 1e-15 and the final
    objectives inside the 40-iteration bracket."""
    import mpmath
    a = json.load(open(os.path.join(GOLDEN, "sp_real_d8_mp256.json")))
    f = json.load(open(os.path.join(GOLDEN, "sp_real_d8_mp256_full.json")))
    assert a["instance"] == f["instance"]
    for ra, rf in zip(a["log"], f["log"]):
        assert all(ra[k] == rf[k] for k in ("mu", "alpha_p", "alpha_d", "beta"))
    assert f["status"] == "terminated" and len(f["log"]) > len(a["log"])
    with mpmath.workprec(256):
        fin = {k: mpmath.mpf(v) for k, v in f["final"].items()}
        assert fin["gap"] < mpmath.mpf("1e-15")
        lo, hi = sorted((mpmath.mpf(a["log"][-1]["p_obj"]), mpmath.mpf(a["log"][-1]["d_obj"])))
        assert lo <= fin["p_obj"] <= hi and lo <= fin["d_obj"] <= hi


@pytest.mark.parametrize("name,bits", [("c4dd", 128), ("c4dd", 256), ("qd32", 256)])
def test_stage_fixtures_agree_with_fp64_oracle(pk, oracle, name, bits):
    """The precomputed multi-precision stage fixtures (tests/golden/make_stage_fixtures.py) are
    consistent with the fp64 oracle run on the same stored state: every sampled entry and
    sketch within fp64 round-off times the conditioning of this mid-run state."""
    import gzip
    import importlib.util
    import json
    import os

    from helpers import compare_summary, residual_scales, stage_reference
    gdir = os.path.join(os.path.dirname(__file__), "golden")
    spec = importlib.util.spec_from_file_location("make_stage_fixtures",
                                                  os.path.join(gdir, "make_stage_fixtures.py"))
    M = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(M)
    sf = os.path.join(gdir, f"stage_{name}.npz")
    if not os.path.exists(os.path.join(gdir, f"stage_{name}_mp{bits}.json.gz")):
        pytest.skip("fixture not generated")
    cons, b = M.instance(name, sf)
    bi = oracle.get_block_info(cons)
    state = M.load_state(sf, bi)
    ar = oracle.Fp64()
    prm = {k: oracle._param(ar, v) for k, v in oracle.DEFAULTS.items()}
    nxt, it = oracle.iteration(ar, cons, bi, b, None, 0.0, state, False, prm)
    ref = stage_reference(it, nxt, bi)
    with gzip.open(os.path.join(gdir, f"stage_{name}_mp{bits}.json.gz"), "rt") as f:
        fx = json.load(f)
    assert set(fx["buffers"]) == set(ref)
    sc = residual_scales(cons, b, state[1])
    e = {k: compare_summary(ref[k], rec, sc.get(k, 0.0)) for k, rec in fx["buffers"].items()}
    assert max(e.values()) < 1e-9, e


@pytest.mark.parametrize("name", ["kw_C_b0_mp256", "kw_needp_mp256", "kw_needd_mp256",
                                  "kw_start_mp256"])
def test_keyword_goldens_fp64_oracle(pk, oracle, name):
    """The fp64 oracle with the golden's keywords (C, b0, need_*_feasible, initial_solutions;
    MPMP.jl:599-613) reproduces the 256-bit keyword goldens' logs to fp64 round-off and stops
    at the same iteration with the same status."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    M = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(M)
    g = json.load(open(os.path.join(GOLDEN, name + ".json")))
    cons, b = pk.synth(**g["instance"])
    bi = oracle.get_block_info(cons)
    ar = oracle.Fp64()
    kw = M.keyword_args(pk, ar, bi, g["keywords"])
    res = oracle.solverank1sdp(cons, b, bi, ar=ar, maxiterations=g["iterations"] + 1,
                               **g["params"], **kw)
    assert res.status == g["status"] and len(res.log) == len(g["log"])
    for row, ref in zip(res.log, g["log"]):
        for key in ("mu", "alpha_p", "alpha_d", "beta", "p_obj", "d_obj", "gap"):
            assert abs(float(getattr(row, key)) - float(ref[key])) <= 1e-9 * max(1.0, abs(float(ref[key]))), key
