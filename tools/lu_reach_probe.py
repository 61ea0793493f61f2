"""How far do runs get with the LU fallback at the reference's default thresholds?
(a) the fp64 polynomial-minimum known answer next to the fp64 oracle (approx_lu! throughout);
(b) the real sphere-packing instance at quad-double (SP.jl defaults: gap 1e-15, errors 1e-30)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _clrsdp_pkg  # noqa: E402
from helpers import poly_min_instance  # noqa: E402

pk = _clrsdp_pkg.load()
which = sys.argv[1] if len(sys.argv) > 1 else "all"
if which in ("all", "poly"):
    from oracle import mpmp_oracle as O
    cons, b, pmin = poly_min_instance(pk)
    bi = pk.get_block_info(cons)
    for fact in (0, 1, 2, 3):
        print("=== poly fp64 GPU factorization flags", fact, flush=True)
        try:
            res = pk.solverank1sdp(cons, b, bi, omega_p=10.0, omega_d=10.0, maxiterations=100,
                                   verbose=True, return_info=True, factorization=fact)
            info = res[-1]
            print("poly fp64 GPU fact=%d: status %s after %d it, gap %.3e, p_obj-pmin %.3e d_obj-pmin %.3e"
                  % (fact, info.status, info.iterations, res[7], res[8] - pmin, res[9] - pmin), flush=True)
        except Exception as e:
            print("poly fp64 GPU fact=%d raised: %s" % (fact, e), flush=True)
    print("=== poly fp64 oracle", flush=True)
    try:
        r = O.solverank1sdp(cons, b, O.get_block_info(cons), maxiterations=100, omega_p=10.0,
                            omega_d=10.0, verbose=True)
        print("poly fp64 oracle: status %s after %d it, gap %.3e, p-pmin %.3e" %
              (r.status, len(r.log), r.gap, r.p_obj - pmin), flush=True)
    except Exception as e:
        print("poly fp64 oracle raised:", e, flush=True)
if which in ("all", "sp"):
    from clrsdp_amd import sphere_packing as S
    t0 = time.time()
    try:
        res = S.Nsphere_packing_2point(3, 8, precision_words=4, maxiterations=int(os.environ.get("MAXIT", "120")),
                                       verbose=True, return_info=True)
        print("sphere packing qd: status %s after %d it, bound %s, gap %s (%.1f s)" %
              (res[-1].status, res[-1].iterations, -res[9], res[7], time.time() - t0), flush=True)
    except Exception as e:
        print("sphere packing qd raised:", e, flush=True)
