"""Iterate the bench instance (C3 by default) with pd_feas = False until the device reports a
failure; prints the iteration count and the last mu (how far fp64 gets before breakdown)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg  # noqa: E402

pk = _clrsdp_pkg.load()
J = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cons, b = pk.synth(seed=0, J=J, delta=128, rank=1, n_y=128)
bi = pk.get_block_info(cons)
dev = pk.DeviceSolver(cons, b, bi)
prm = pk.make_params("0.3", "0.1", "0.7", 0)
dev.set_state(*pk.initial_point(bi, 100.0, 100.0))
dev.initial_residuals(prm)
last = None
for it in range(1, 2001):
    try:
        st = dev.iterate(prm, False)
    except Exception as e:
        print(f"failed at iteration {it}: {e}; last mu {last[0]:.3e} P_err {last[1]:.2e} d_err {last[2]:.2e} "
              f"pobj {last[3]:.12e} dobj {last[4]:.12e}")
        break
    last = (st.mu, st.P_err, st.d_err, st.p_obj, st.d_obj)
else:
    print("no failure in 2000 iterations", last)
