"""Print the double-double log of the gap-1e-20 golden instance next to the 256-bit oracle's."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg  # noqa: E402

pk = _clrsdp_pkg.load()
g = json.load(open(os.path.join(ROOT, "tests/golden/rank2_mp256_seed5_gap20.json")))
cons, b = pk.synth(**g["instance"])
bi = pk.get_block_info(cons)
res = pk.solverank1sdp(cons, b, bi, maxiterations=int(sys.argv[1]) if len(sys.argv) > 1 else 70,
                       precision_words=2, verbose=False, return_info=True, **g["params"])
info = res[-1]
print("status", info.status, "iterations", info.iterations)
for row, ref in zip(info.log, g["log"] + [None] * 200):
    r = ("%.3e %.3e %.3e %.3e" % tuple(float(ref[k]) for k in ("gap", "P_err", "p_err", "d_err"))
         if ref else "")
    print("%3d gap %.3e P %.3e p %.3e d %.3e | oracle %s" % (row[0], float(row[5]), row[6], row[7],
                                                             row[8], r))
