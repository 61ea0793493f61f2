"""CPU tests of the C++ OpenMP restatement (oracle/cpu_restatement.cpp): it must agree with the
Python oracle (oracle/mpmp_oracle.py) and the golden logs it generated, at every word type.
It is the bench's CPU baseline, so it has to compute the same iterations as the reference
algorithm, not merely something as expensive."""
import json
import os

import mpmath
import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def cr():
    from oracle import cpurest
    cpurest.build()
    return cpurest


def _instance(pk, inst):
    inst = dict(inst)
    if inst.pop("kind", None) == "sphere_packing_shape":
        return pk.synth_mixed(**pk.SPHERE_PACKING_SHAPE, **inst)
    return pk.synth(**inst)


@pytest.mark.parametrize("name,words,tol", [("c1_fp64_seed3", 1, 1e-9), ("m2L2_fp64_seed4", 1, 1e-9),
                                            ("c1_mp256_seed3", 2, 1e-24), ("rank2_mp256_seed5", 2, 1e-24),
                                            ("c1_mp256_seed3", 4, 1e-45), ("rank2_mp256_seed5", 4, 1e-45),
                                            ("sp_mp256_seed1", 1, 1e-8), ("sp_mp256_seed1", 2, 1e-22),
                                            ("sp_mp256_seed1", 4, 1e-40)])
def test_golden_logs(pk, cr, name, words, tol):
    """mu, alpha_p, alpha_d, beta of every iteration of the golden solverank1sdp logs."""
    g = json.load(open(os.path.join(GOLDEN, name + ".json")))
    cons, b = _instance(pk, g["instance"])
    bi = pk.get_block_info(cons)
    prm = g["params"]
    st = pk.initial_point(bi, prm["omega_p"], prm["omega_d"])
    n = len(g["log"])
    rc, log, _, _ = cr.run(pk, cons, b, bi, words, st, n, threads=4,
                           thresholds=(prm["primal_error_threshold"], prm["dual_error_threshold"]))
    assert rc == n, rc
    mpmath.mp.prec = 256
    for it, ref in enumerate(g["log"]):
        for q, key in ((0, "mu"), (1, "alpha_p"), (2, "alpha_d"), (3, "beta")):
            r = mpmath.mpf(ref[key])
            assert abs(mpmath.mpf(log[it, q]) - r) <= tol * max(1, abs(r)), (it + 1, key, float(log[it, q]), float(r))


@pytest.mark.parametrize("words,tol", [(2, 1e-24), (4, 1e-45)])
def test_state_after_golden_run_full_precision(pk, cr, words, tol):
    """The full-width state after the golden run equals the 256-bit oracle's final x and y."""
    g = json.load(open(os.path.join(GOLDEN, "c1_mp256_seed3.json")))
    cons, b = _instance(pk, g["instance"])
    bi = pk.get_block_info(cons)
    prm = g["params"]
    st = pk.initial_point(bi, prm["omega_p"], prm["omega_d"])
    n = len(g["log"])
    rc, _, _, (x, X, y, Y) = cr.run(pk, cons, b, bi, words, st, n, threads=2,
                                    thresholds=(prm["primal_error_threshold"], prm["dual_error_threshold"]))
    assert rc == n
    mpmath.mp.prec = 256
    for got, ref in ((x, g["x"]), (y, g["y"])):
        sc = max(abs(mpmath.mpf(v)) for v in ref)
        err = max(abs(mpmath.mpf(a) - mpmath.mpf(r)) for a, r in zip(got, ref)) / max(1, sc)
        assert err < tol, float(err)


def test_fp64_matches_python_oracle_mid_size(pk, cr, oracle):
    """Three iterations of a 4-cluster, 20x20-block instance: every logged quantity and the state
    against the numpy oracle (same algorithm, different summation order)."""
    cons, b = pk.synth(seed=7, J=4, delta=20, rank=2, n_y=8)
    bi = oracle.get_block_info(cons)
    ar = oracle.Fp64()
    prm = {k: oracle._param(ar, v) for k, v in oracle.DEFAULTS.items()}
    st = oracle.initial_point(ar, bi, 10.0, 10.0)
    rows = []
    s = st
    for _ in range(3):
        s, it = oracle.iteration(ar, cons, bi, b, None, 0.0, s, False, prm)
        rows.append((it["mu"], it["alpha_p"], it["alpha_d"], it["beta_c"]))
    rc, log, _, (x, X, y, Y) = cr.run(pk, cons, b, pk.get_block_info(cons), 1,
                                      oracle.initial_point(ar, bi, 10.0, 10.0), 3, threads=4)
    assert rc == 3
    assert np.allclose(log[:, :4], np.array(rows, dtype=float), rtol=1e-10, atol=0)
    assert np.max(np.abs(x - s[0])) <= 1e-9 * max(1, np.max(np.abs(s[0])))
    assert np.max(np.abs(y - s[2])) <= 1e-9 * max(1, np.max(np.abs(s[2])))


def test_thread_count_does_not_change_results(pk, cr):
    """The OpenMP partitions only distribute independent blocks and clusters: bitwise the same
    iterates with 1 and 4 threads."""
    cons, b = pk.synth(seed=2, J=5, delta=6, rank=1, n_y=4, m=2, L=2)
    bi = pk.get_block_info(cons)
    st = pk.initial_point(bi, 10.0, 10.0)
    out = [cr.run(pk, cons, b, bi, 2, st, 4, threads=t) for t in (1, 4)]
    assert np.array_equal(out[0][1], out[1][1])
    assert all(a == c for a, c in zip(out[0][3][0], out[1][3][0]))
