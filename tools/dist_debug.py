import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import _clrsdp_pkg
pk = _clrsdp_pkg.load()
from clrsdp_amd import dist as cdist, _lib as L
rank = int(os.environ.get("RANK", 0)); world = int(os.environ.get("WORLD_SIZE", 1))
cons, b = pk.synth(seed=12, J=5, delta=16, rank=1, n_y=9, m=1)
bi = pk.get_block_info(cons)
ex = None
if world > 1:
    ex = cdist.TorchExchange(0, backend="gloo")
owned = pk.partition_clusters(bi, world)[rank] if world > 1 else None
dev = pk.DeviceSolver(cons, b, bi, device=0, rank=rank, world=world, owned=owned)
if ex: ex.attach(dev)
P = pk.make_params("0.3", "0.1", "0.7", 0)
dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
for s in range(4):
    try:
        dev.run_stage(s, P, False)
    except Exception as e:
        print(rank, "stage", s, e)
sc = dev.buffer(L.BUF_SCALARS)
Q = dev.buffer(L.BUF_Q)
print(rank, owned, "dotXY", sc[15], "mu", sc[0], "Q[:4]", Q[:4], flush=True)
