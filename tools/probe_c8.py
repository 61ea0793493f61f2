"""Loop bodies of the 8-cluster C3 shard from the bench's initial point: mu / alpha per body and
the first failure, with the current build (env switches apply)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg  # noqa: E402

pk = _clrsdp_pkg.load()
J = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
cons, b = pk.synth(seed=0, J=J, delta=128, rank=1, n_y=128)
bi = pk.get_block_info(cons)
dev = pk.DeviceSolver(cons, b, bi)
P = pk.make_params("0.3", "0.1", "0.7", 0)
dev.set_state(*pk.initial_point(bi, 100.0, 100.0))
feas = False
for it in range(n):
    try:
        st = dev.iterate(P, feas)
    except Exception as e:  # noqa: BLE001
        print("body", it + 1, "failed:", e)
        break
    feas = max(st.p_err, st.P_err) < 1e-30 and st.d_err < 1e-30
    if it % 4 == 0 or it > n - 10:
        print("body %3d mu %.3e alpha_p %.4f alpha_d %.4f perr %.2e derr %.2e" % (
            it + 1, st.mu, st.alpha_p, st.alpha_d, max(st.p_err, st.P_err), st.d_err))
