"""GPU full runs with the solverank1sdp keywords every other golden leaves at their defaults
(MPMP.jl:599-613), and loop control below fp64 resolution.

* ``C`` != 0 (MPMP.jl:599, 691-695: in P at 1108 and in <C,Y> of the dual objective 1031),
  ``b0`` != 0 (the initial gap excludes it, 725; later gaps include it, 942),
  ``need_primal_feasible`` / ``need_dual_feasible`` (terminate, 1147-1173) and
  ``initial_solutions`` (613, 687-689): the device against 256-bit oracle logs
  (tests/golden/make_golden.py keywords) at fp64 (1e-9) and double-double (1e-24), with the
  synchronous loop and the pipelined one (device-side terminate()).
* ``duality_gap_threshold = 1e-20`` at double-double: the synchronous and pipelined loops must
  stop at the iteration the 256-bit oracle stops at (tests/golden/rank2_mp256_seed5_gap20.json,
  45 iterations), which needs the gap and the thresholds at full width (a leading-limb gap is
  exactly 0 once the objectives agree to 2^-53, ~15 iterations earlier).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _golden(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


def _keywords(pk, bi, kw):
    """Device-side keywords of a golden (the same construction as make_golden.keyword_args)."""
    out = {}
    if "C_seed" in kw:
        out["C"] = pk.synth_C(bi, kw["C_seed"], kw.get("C_scale", 0.125))
    if "b0" in kw:
        out["b0"] = kw["b0"]
    for k in ("need_primal_feasible", "need_dual_feasible"):
        if kw.get(k):
            out[k] = True
    if "start_seed" in kw:
        out["initial_solutions"] = pk.synth_start(bi, kw["start_seed"])
    return out


def _check_log(info, g, tol, exact_rows):
    import mpmath
    mpmath.mp.prec = 256
    assert len(info.log) == len(g["log"]), (len(info.log), len(g["log"]))
    for row, ref in zip(info.log, g["log"]):
        # (it, time, mu, p_obj, d_obj, gap, P_err, p_err, d_err, alpha_p, alpha_d, beta)
        for idx, key in ((2, "mu"), (3, "p_obj"), (4, "d_obj"), (5, "gap"), (9, "alpha_p"),
                         (10, "alpha_d"), (11, "beta")):
            r = mpmath.mpf(ref[key])
            v = mpmath.mpf(row[idx])
            # log rows are leading limbs except the gap at dd/qd (full width); compare the
            # leading-limb columns at fp64 resolution
            t = tol if (exact_rows and key == "gap") or tol >= 1e-12 else 4e-16
            assert abs(v - r) <= t * max(1, abs(r)), (row[0], key, float(v), float(r))


KW_CASES = ["kw_C_b0_mp256", "kw_needp_mp256", "kw_needd_mp256", "kw_start_mp256"]


@pytest.mark.parametrize("words,tol", [(1, 1e-9), (2, 1e-24)])
@pytest.mark.parametrize("name", KW_CASES)
def test_keywords_match_golden(pk, name, words, tol):
    import mpmath
    mpmath.mp.prec = 256
    g = _golden(name)
    cons, b = pk.synth(**g["instance"])
    bi = pk.get_block_info(cons)
    kw = _keywords(pk, bi, g["keywords"])
    res = pk.solverank1sdp(cons, b, bi, maxiterations=g["iterations"] + 1, precision_words=words,
                           verbose=False, return_info=True, record_exact=True, **g["params"], **kw)
    info = res[-1]
    assert info.status == g["status"]
    _check_log(info, g, tol, words > 1)
    # full-width per-iteration scalars against the oracle (mu, steps, beta, objectives)
    for it, (sc, ref) in enumerate(zip(info.exact, g["log"])):
        for key, slot in (("mu", "mu"), ("alpha_p", "alpha_p"), ("alpha_d", "alpha_d"),
                          ("beta", "beta_c")):
            r, v = mpmath.mpf(ref[key]), mpmath.mpf(sc[slot])
            assert abs(v - r) <= tol * max(1, abs(r)), (it + 1, key, float(v), float(r))
        if it + 1 < len(g["log"]):
            for key in ("p_obj", "d_obj"):
                r, v = mpmath.mpf(g["log"][it + 1][key]), mpmath.mpf(sc[key])
                assert abs(v - r) <= tol * max(1, abs(r)), (it + 1, key, float(v), float(r))
    for v, key in zip(res[7:10], ("gap", "p_obj", "d_obj")):
        r = mpmath.mpf(g["final"][key])
        assert abs(mpmath.mpf(v) - r) <= tol * max(1, abs(r)), (key, float(v), float(r))
    yr = np.array([float(mpmath.mpf(v)) for v in g["y"]])
    assert np.max(np.abs(np.asarray(res[2], dtype=float) - yr)) <= max(tol, 1e-15) * 10 * max(1, np.max(np.abs(yr)))


@pytest.mark.parametrize("name", ["kw_C_b0_mp256", "kw_needp_mp256", "kw_needd_mp256"])
def test_keywords_pipelined_equals_synchronous(pk, name):
    """The pipelined loop (terminate() and pd_feas decided on the device) gives the same log,
    status and final state as the synchronous loop with every keyword, at dd."""
    g = _golden(name)
    cons, b = pk.synth(**g["instance"])
    bi = pk.get_block_info(cons)
    kw = _keywords(pk, bi, g["keywords"])
    outs = []
    for pipe in (False, True):
        res = pk.solverank1sdp(cons, b, bi, maxiterations=g["iterations"] + 1, precision_words=2,
                               verbose=False, return_info=True, pipelined=pipe,
                               **g["params"], **kw)
        outs.append(res)
    a, c = outs
    assert a[-1].status == c[-1].status == g["status"]
    assert len(a[-1].log) == len(c[-1].log) == len(g["log"])
    for ra, rc in zip(a[-1].log, c[-1].log):
        assert ra[2:] == rc[2:]
    assert np.array_equal(np.asarray(a[0], dtype=float), np.asarray(c[0], dtype=float))
    assert np.array_equal(np.asarray(a[2], dtype=float), np.asarray(c[2], dtype=float))


@pytest.mark.parametrize("pipelined", [False, True])
def test_dd_gap_threshold_below_fp64(pk, pipelined):
    """duality_gap_threshold = 1e-20 at double-double stops at the 256-bit oracle's iteration."""
    import mpmath
    mpmath.mp.prec = 256
    g = _golden("rank2_mp256_seed5_gap20")
    assert g["status"] == "terminated"
    cons, b = pk.synth(**g["instance"])
    bi = pk.get_block_info(cons)
    res = pk.solverank1sdp(cons, b, bi, maxiterations=g["iterations"], precision_words=2,
                           verbose=False, return_info=True, pipelined=pipelined, **g["params"])
    info = res[-1]
    assert info.status == "terminated"
    assert info.iterations == len(g["log"]), (info.iterations, len(g["log"]))
    gap = res[7]
    assert isinstance(gap, mpmath.mpf) and gap < mpmath.mpf("1e-20")
    for v, key in zip(res[7:10], ("gap", "p_obj", "d_obj")):
        r = mpmath.mpf(g["final"][key])
        # the objectives agree far below fp64 resolution; the gap (their ~6e-21 difference) to 1 %
        t = 1e-2 * abs(r) if key == "gap" else 1e-24
        assert abs(mpmath.mpf(v) - r) <= t, (key, float(v), float(r))
