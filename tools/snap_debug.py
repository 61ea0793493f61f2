import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg
pk = _clrsdp_pkg.load()
cons, b = pk.synth(seed=4, J=3, delta=8, rank=1, n_y=5, m=1)
bi = pk.get_block_info(cons)
P = pk.make_params("0.3", "0.1", "0.7", 0)
dev = pk.DeviceSolver(cons, b, bi)
dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
dev.initial_residuals(P)
for _ in range(3):
    dev.iterate(P, False)
dev.save_state()
x0, X0, y0, Y0 = dev.get_state()
sc0 = dev.buffer(16)
for _ in range(3):
    dev.iterate(P, False)
dev.restore_state()
dev.synchronize()
x1, X1, y1, Y1 = dev.get_state()
sc1 = dev.buffer(16)
print("x", np.max(np.abs(x1 - x0)), "y", np.max(np.abs(y1 - y0)),
      "X", max(np.max(np.abs(a - c)) for ba, bc in zip(X0, X1) for a, c in zip(ba, bc)),
      "Y", max(np.max(np.abs(a - c)) for ba, bc in zip(Y0, Y1) for a, c in zip(ba, bc)),
      "sc", np.max(np.abs(sc1 - sc0)))
print("nx", len(x0), x0[:4], x1[:4])
# one body after the snapshot, twice
st_a = dev.iterate(P, False); Pa = dev.buffer(7); da = dev.buffer(9); pa = dev.buffer(8); dxa = dev.buffer(10)
dev.restore_state()
st_b = dev.iterate(P, False); Pb = dev.buffer(7); db = dev.buffer(9); pb = dev.buffer(8); dxb = dev.buffer(10)
print("P_err", st_a.P_err, st_b.P_err, "p_err", st_a.p_err, st_b.p_err, "pobj", st_a.p_obj, st_b.p_obj)
print("dP", np.max(np.abs(Pa - Pb)), "dd", np.max(np.abs(da - db)), "dp", np.max(np.abs(pa - pb)), "ddx", np.max(np.abs(dxa - dxb)))
dev.set_timing(True)
dev.restore_state()
st_c = dev.iterate(P, False)
print("timed (no graph):", st_c.P_err, st_c.p_obj)
