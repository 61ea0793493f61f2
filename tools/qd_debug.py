"""Debug helper: qd (4-word) stage outputs against the 256-bit oracle on a C1 instance."""
import sys
import numpy as np
import mpmath
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import _clrsdp_pkg
pk = _clrsdp_pkg.load()
from oracle import mpmp_oracle as O
from clrsdp_amd import _lib as L
from helpers import rel_err

words = int(sys.argv[1]) if len(sys.argv) > 1 else 4
J = int(sys.argv[2]) if len(sys.argv) > 2 else 2
mpmath.mp.prec = 256
cons, b = pk.synth(seed=3, J=J, delta=4, rank=1, n_y=4)
ar = O.Mp(256)
consm = [pk.Cluster([[[ar.asarray(v) for v in vk] for vk in Al] for Al in cl.A], ar.asarray(cl.B),
                    ar.asarray(cl.c), [[[ar.num(x) for x in hk] for hk in Hl] for Hl in cl.H]) for cl in cons]
bm = ar.asarray(b)
bi = O.get_block_info(consm)
prm = {k: O._param(ar, v) for k, v in O.DEFAULTS.items()}
state = O.initial_point(ar, bi, 10.0, 10.0)
for _ in range(2):
    state, _ = O.iteration(ar, consm, bi, bm, None, ar.num(0), state, False, prm)
dev = pk.DeviceSolver(consm, bm, pk.get_block_info(consm), precision_words=words)
dev.set_state(*state)
x = state[0]
print("x roundtrip", rel_err(dev.buffer(L.BUF_XVEC, True), x))
P = pk.make_params("0.3", "0.1", "0.7", 0)
for s in (L.STAGE_MU_R, L.STAGE_XINV, L.STAGE_SCHUR, L.STAGE_FACTOR, L.STAGE_RESIDUALS):
    dev.run_stage(s, P, False)
Bst = O.stack_B(consm)
pexp = bm - Bst.T.dot(x)
print("p", rel_err(dev.buffer(L.BUF_PVEC, True), pexp))
print("B dtype", Bst.dtype, type(Bst[0, 0]))
pd = dev.buffer(L.BUF_PVEC, True)
for i in range(len(pexp)):
    print(i, mpmath.nstr(pd[i], 40), mpmath.nstr(pexp[i], 40))
print("b", [mpmath.nstr(v, 30) for v in bm])
print("x", [mpmath.nstr(v, 30) for v in x])
xd = np.array([mpmath.mpf(float(v)) for v in x], dtype=object)
pexp2 = bm - Bst.T.dot(xd)
print("p vs x-rounded-to-double", rel_err(pd, pexp2))
print("x after stages", rel_err(dev.buffer(L.BUF_XVEC, True), x))
pf = np.array(b, dtype=float) - np.array(Bst, dtype=float).T @ np.array([float(v) for v in x])
print("p vs float64 evaluation", rel_err(pd, np.array([mpmath.mpf(v) for v in pf], dtype=object)))
