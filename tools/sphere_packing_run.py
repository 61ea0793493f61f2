"""Solve the sphere-packing two-point program (SP.jl) on the GPU and print the bound.

    python tools/sphere_packing_run.py [--words 4] [--gap 1e-30] [--maxit 300] [--d 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--words", type=int, default=4)
ap.add_argument("--gap", default="1e-30")
ap.add_argument("--maxit", type=int, default=300)
ap.add_argument("--n", type=int, default=3)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--prec", type=int, default=512)
ap.add_argument("--json", default="")
a = ap.parse_args()
pk = _clrsdp_pkg.load()
from clrsdp_amd import sphere_packing as S  # noqa: E402

t0 = time.time()
cons, b, bi = S.sphere_packing_constraints(a.n, a.d, prec=a.prec)
t1 = time.time()
res = pk.solverank1sdp(cons, b, bi, omega_p=100, omega_d=100, precision_words=a.words,
                       duality_gap_threshold=a.gap, maxiterations=a.maxit, return_info=True,
                       record_exact=True)
info = res[-1]
import mpmath  # noqa: E402
last = info.exact[-1] if info.exact else {}
print(f"prepareabc {t1 - t0:.2f} s; solve {res[10]:.3f} s, {info.iterations} iterations, "
      f"status {info.status}")
print(f"bound (-dual objective) = {-res[9]!r}  (-primal objective {-res[8]!r})")
if a.json:
    with open(a.json, "w") as f:
        json.dump({"words": a.words, "iterations": info.iterations, "status": info.status,
                   "time_s": res[10], "p_obj": res[8], "d_obj": res[9], "gap": res[7],
                   "exact_last": {k: mpmath.nstr(v, 60) for k, v in last.items()},
                   "log": [list(map(float, r)) for r in info.log]}, f, indent=1)
