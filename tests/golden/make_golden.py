"""Generate the golden vectors under tests/golden/ with the oracle (oracle/mpmp_oracle.py).

The reference (Julia + Arblib) cannot run in this container, so these vectors
are produced by the restatement itself: an fp64 run and a 256-bit run of solverank1sdp on small
seeded synthetic instances.  They pin the oracle and the HIP path against regressions and give
the multi-word (double-double) path something exact to converge to.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import mpmath  # noqa: E402

import _clrsdp_pkg  # noqa: E402
from oracle import mpmp_oracle as O  # noqa: E402

pk = _clrsdp_pkg.load()
PARAMS = dict(omega_p=10.0, omega_d=10.0, primal_error_threshold=1e-10, dual_error_threshold=1e-10,
              duality_gap_threshold=1e-10)


def to_mp(ar, cons):
    return [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in Al] for Al in cl.A],
                       ar.asarray(cl.B), ar.asarray(cl.c),
                       [[[ar.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]


def make_instance(inst):
    """synth(**inst), or synth_mixed for inst["kind"] == "sphere_packing_shape" (config 5)."""
    inst = dict(inst)
    if inst.get("kind") == "sphere_packing":
        # the real SpherePacking.jl instance (SP.jl:29-105), sampled at 512 bits by prepareabc
        from clrsdp_amd import sphere_packing as S
        cons, b, _ = S.sphere_packing_constraints(inst["n"], inst["d"], prec=inst.get("prep_bits", 512))
        return cons, b
    if inst.pop("kind", None) == "sphere_packing_shape":
        return pk.synth_mixed(**pk.SPHERE_PACKING_SHAPE, **inst)
    return pk.synth(**inst)


def keyword_args(pk_, ar, bi, kw):
    """The solverank1sdp keywords of a golden run (round 4): C from synth_C(C_seed, C_scale), b0,
    need_primal/dual_feasible, initial_solutions from synth_start(start_seed); the same
    construction is used by the GPU tests (tests/test_gpu_keywords.py)."""
    out = {}
    if not kw:
        return out
    if "C_seed" in kw:
        Cb = pk_.synth_C(bi, kw["C_seed"], kw.get("C_scale", 0.125))
        out["C"] = [[ar.asarray(m) for m in row] for row in Cb]
    if "b0" in kw:
        out["b0"] = kw["b0"]
    for k in ("need_primal_feasible", "need_dual_feasible"):
        if kw.get(k):
            out[k] = True
    if "start_seed" in kw:
        x, X, y, Y = pk_.synth_start(bi, kw["start_seed"])
        out["initial_solutions"] = (ar.asarray(x), [[ar.asarray(m) for m in r] for r in X],
                                    ar.asarray(y), [[ar.asarray(m) for m in r] for r in Y])
    return out


def run(name, inst, iters, prec=None, tol=1e-9, params=None, keywords=None):
    cons, b = make_instance(inst)
    bi = O.get_block_info(cons)
    if prec:
        ar = O.Mp(prec)
        consr = to_mp(ar, cons)
        br = ar.asarray(b)
    else:
        ar = O.Fp64()
        consr, br = cons, b
    params = params or PARAMS
    kwa = keyword_args(pk, ar, bi, keywords)
    if "b0" in kwa:
        kwa["b0"] = ar.num(kwa["b0"]) if prec else kwa["b0"]
    res = O.solverank1sdp(consr, br, bi, ar=ar, maxiterations=iters + 1, **params, **kwa)
    fmt = (lambda v: mpmath.nstr(v, 70)) if prec else (lambda v: repr(float(v)))
    out = {
        "generator": "tests/golden/make_golden.py (oracle/mpmp_oracle.py, %s)" % ar.name,
        "instance": inst, "params": params, "iterations": iters, "tolerance_fp64": tol,
        "keywords": keywords or {},
        "log": [{k: fmt(getattr(r, k)) for k in ("mu", "p_obj", "d_obj", "gap", "P_err", "p_err",
                                                  "d_err", "alpha_p", "alpha_d", "beta")}
                for r in res.log],
        "status": res.status,
        "final": {"gap": fmt(res.gap), "p_obj": fmt(res.p_obj), "d_obj": fmt(res.d_obj)},
        "x": [fmt(v) for v in res.x],
        "y": [fmt(v) for v in res.y],
    }
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(out, f, indent=1)
    print(name, len(res.log), "iterations")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "sp_real":  # real sphere-packing instance (~15 min)
        run("sp_real_d8_mp256", dict(kind="sphere_packing", n=3, d=8), 40, prec=256,
            params=dict(omega_p=100.0, omega_d=100.0, duality_gap_threshold=1e-30))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "sp_real_full":  # to the reference's defaults (~40 min)
        # SP.jl:110 passes no thresholds: solverank1sdp's defaults gap 1e-15, errors 1e-30
        run("sp_real_d8_mp256_full", dict(kind="sphere_packing", n=3, d=8), 120, prec=256,
            params=dict(omega_p=100.0, omega_d=100.0, duality_gap_threshold=1e-15,
                        primal_error_threshold=1e-30, dual_error_threshold=1e-30))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "gap20":
        # round 4: loop control below fp64 resolution (duality gap 1e-20, double-double on the
        # device; a leading-limb gap is 0 once the objectives agree to 2^-53, ~15 iterations
        # earlier): the 256-bit run to termination fixes the iteration the dd loops must stop at.
        # (1e-24 is out of double-double's reach on this instance: its dual error grows from
        # ~1e-27 at gap 1e-21 and the gap stalls near 1e-22, tools/dd_gap_probe.py)
        run("rank2_mp256_seed5_gap20", dict(J=2, delta=3, rank=2, n_y=3, seed=5), 120, prec=256,
            params=dict(omega_p=10.0, omega_d=10.0, duality_gap_threshold=1e-20,
                        primal_error_threshold=1e-20, dual_error_threshold=1e-20))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "keywords":
        # round 4: the solverank1sdp keywords every earlier golden left at their defaults
        # (C = 0, b0 = 0, no early feasibility stop, the default start; MPMP.jl:599-613)
        m2 = dict(J=2, delta=3, rank=1, n_y=3, m=2, L=2, seed=4)
        c1 = dict(J=2, delta=4, rank=1, n_y=4, seed=3)
        run("kw_C_b0_mp256", m2, 12, prec=256, keywords=dict(C_seed=21, C_scale=0.125, b0=0.75))
        run("kw_needp_mp256", c1, 40, prec=256, keywords=dict(need_primal_feasible=True),
            params=dict(PARAMS, primal_error_threshold=1e-6))
        run("kw_needd_mp256", m2, 40, prec=256, keywords=dict(need_dual_feasible=True),
            params=dict(PARAMS, dual_error_threshold=1e-6))
        run("kw_start_mp256", c1, 12, prec=256, keywords=dict(start_seed=5, C_seed=22))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "sp":  # only the config-5-shape vector (~40 s)
        run("sp_mp256_seed1", dict(kind="sphere_packing_shape", seed=1), 12, prec=256)
        sys.exit(0)
    run("c1_fp64_seed3", dict(J=2, delta=4, rank=1, n_y=4, seed=3), 10)
    run("m2L2_fp64_seed4", dict(J=2, delta=3, rank=1, n_y=3, m=2, L=2, seed=4), 10)
    run("c1_mp256_seed3", dict(J=2, delta=4, rank=1, n_y=4, seed=3), 10, prec=256)
    run("rank2_mp256_seed5", dict(J=2, delta=3, rank=2, n_y=3, seed=5), 8, prec=256)
    run("sp_mp256_seed1", dict(kind="sphere_packing_shape", seed=1), 12, prec=256)
