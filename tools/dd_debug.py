import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, mpmath
import _clrsdp_pkg
pk = _clrsdp_pkg.load()
from clrsdp_amd import _lib as L, instance as inst
from oracle import mpmp_oracle as O
from helpers import rel_err
mpmath.mp.prec = 256
cons, b = pk.synth(seed=3, J=2, delta=4, rank=1, n_y=4)
ar = O.Mp(256)
consm = [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in Al] for Al in cl.A], ar.asarray(cl.B), ar.asarray(cl.c), [[[ar.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]
bi = O.get_block_info(consm)
prm = {k: O._param(ar, v) for k, v in O.DEFAULTS.items()}
st = O.initial_point(ar, bi, 10.0, 10.0)
st, _ = O.iteration(ar, consm, bi, ar.asarray(b), None, ar.num(0), st, False, prm)
dev = pk.DeviceSolver(consm, ar.asarray(b), pk.get_block_info(cons), precision_words=2)
dev.set_state(*st)
x, X, y, Y = dev.get_state(exact=True)
print("roundtrip x", rel_err(x, st[0]), "X", rel_err(inst.blocks_to_flat(X), inst.blocks_to_flat(st[1])))
P = pk.make_params("0.3", "0.1", "0.7", 0)
dev.run_stage(L.STAGE_MU_R, P, False)
sc = dev.buffer(L.BUF_SCALARS, exact=True)
print("dotXY", sc[15], O.dot_blocks(ar, st[1], st[3]))
print("mu", sc[0], O.dot_blocks(ar, st[1], st[3]) / bi.total_dim)
raw = np.zeros(2 * 24); import ctypes as C
cnt = C.c_int64()
dev.L.clrsdp_get_buffer(dev.h, L.BUF_SCALARS, raw.ctypes.data_as(L.P_f64), C.byref(cnt))
print("raw planes", raw.reshape(2, -1)[:, :2])
