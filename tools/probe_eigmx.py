"""Loop bodies of a bench instance with eigmin_mx on (CLRSDP_EIG_MX=1, CLRSDP_EIGMX_STATS=1 print
the fallback count at close): how often the refined fp64 eigenpair is not accepted."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg  # noqa: E402

pk = _clrsdp_pkg.load()
cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
words = int(sys.argv[3]) if len(sys.argv) > 3 else 2
if cfg == "c2":
    cons, b = pk.synth(seed=0, J=16, delta=64, rank=2, n_y=64)
else:
    cons, b = pk.synth_mixed(**pk.SPHERE_PACKING_SHAPE, seed=0)
bi = pk.get_block_info(cons)
dev = pk.DeviceSolver(cons, b, bi, precision_words=words)
P = pk.make_params("0.3", "0.1", "0.7", 0)
dev.set_state(*pk.initial_point(bi, 100.0, 100.0))
dev.initial_residuals(P)
feas = False
nblk = 2 * sum(len(x) for x in bi.Y_blocksizes)
for it in range(n):
    st = dev.iterate(P, feas)
    feas = max(st.p_err, st.P_err) < 1e-30 and st.d_err < 1e-30
print("bodies", n, "blocks per eigen launch", nblk)
dev.close()
