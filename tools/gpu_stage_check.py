"""Ad-hoc stage-by-stage comparison of the HIP path with the oracle (prints relative errors)."""
import sys, os, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg
pk = _clrsdp_pkg.load()
L = pk._lib
from oracle import mpmp_oracle as O
from importlib import import_module
inst = import_module("clrsdp_amd.instance")


def rel(a, b, scale=0.0):
    a = np.asarray(a, dtype=float).ravel(); b = np.asarray(b, dtype=float).ravel()
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b)), scale))


def run(cfg, iters_before=2):
    cons, b = pk.synth(seed=3, **cfg)
    bi = O.get_block_info(cons)
    ar = O.Fp64()
    prm = {k: O._param(ar, v) for k, v in O.DEFAULTS.items()}
    state = O.initial_point(ar, bi, 100.0, 100.0)
    pd = False
    for _ in range(iters_before):
        state, inter = O.iteration(ar, cons, bi, b, None, 0.0, state, pd, prm)
    x, X, y, Y = state
    state2, it = O.iteration(ar, cons, bi, b, None, 0.0, state, pd, prm)
    dev = pk.DeviceSolver(cons, b, pk.get_block_info(cons))
    dev.set_state(x, X, y, Y)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    fl = lambda blocks: inst.blocks_to_flat(blocks)
    out = {}
    dev.run_stage(L.STAGE_MU_R, P, pd)
    out["mu"] = rel(dev.scalar("mu"), it["mu"])
    out["R"] = rel(dev.buffer(L.BUF_R), fl(it["R"]))
    dev.run_stage(L.STAGE_XINV, P, pd)
    out["Xinv"] = rel(dev.buffer(L.BUF_XINV), fl(it["X_inv"]))
    dev.run_stage(L.STAGE_SCHUR, P, pd)
    out["S"] = rel(dev.buffer(L.BUF_S), np.concatenate([s.reshape(-1, order="F") for s in it["dec"].S_raw]))
    ay = []
    for j in range(bi.J):
        for l in range(bi.L[j]):
            for r in range(bi.m[j]):
                for s in range(r + 1):
                    ay.append(it["A_Y"][j][l][r][s])
    out["A_Y"] = rel(dev.buffer(L.BUF_AY), np.concatenate(ay))
    dev.run_stage(L.STAGE_FACTOR, P, pd)
    out["Q"] = rel(dev.buffer(L.BUF_Q), it["dec"].Q_raw.reshape(-1, order="F"))
    dev.run_stage(L.STAGE_RESIDUALS, P, pd)
    out["P"] = rel(dev.buffer(L.BUF_P), fl(it["P"]), np.max(np.abs(fl(X))))
    out["p"] = rel(dev.buffer(L.BUF_PVEC), it["p"], np.max(np.abs(b)))
    out["d"] = rel(dev.buffer(L.BUF_DVEC), it["d"])
    dev.run_stage(L.STAGE_PREDICTOR, P, pd)
    dx, dXp, dy, dYp = it["pred"]
    out["pred_dx"] = rel(dev.buffer(L.BUF_DX), dx)
    out["pred_dy"] = rel(dev.buffer(L.BUF_DY), dy)
    out["pred_dX"] = rel(dev.buffer(L.BUF_DXMAT), fl(dXp))
    out["pred_dY"] = rel(dev.buffer(L.BUF_DYMAT), fl(dYp))
    dev.run_stage(L.STAGE_CORRECTOR_R, P, pd)
    out["beta_c"] = rel(dev.scalar("beta_c"), it["beta_c"])
    out["R2"] = rel(dev.buffer(L.BUF_R), fl(it["R2"]))
    dev.run_stage(L.STAGE_CORRECTOR, P, pd)
    dx, dXc, dy, dYc = it["corr"]
    out["corr_dx"] = rel(dev.buffer(L.BUF_DX), dx)
    out["corr_dy"] = rel(dev.buffer(L.BUF_DY), dy)
    out["corr_dX"] = rel(dev.buffer(L.BUF_DXMAT), fl(dXc))
    out["corr_dY"] = rel(dev.buffer(L.BUF_DYMAT), fl(dYc))
    dev.run_stage(L.STAGE_STEP, P, pd)
    out["alpha_p"] = rel(dev.scalar("alpha_p"), it["alpha_p"])
    out["alpha_d"] = rel(dev.scalar("alpha_d"), it["alpha_d"])
    dev.run_stage(L.STAGE_UPDATE, P, pd)
    xg, Xg, yg, Yg = dev.get_state()
    out["x+"] = rel(xg, state2[0]); out["X+"] = rel(fl(Xg), fl(state2[1]))
    out["y+"] = rel(yg, state2[2]); out["Y+"] = rel(fl(Yg), fl(state2[3]))
    out["pobj"] = rel(dev.scalar("p_obj"), O.primal_objective(ar, cons, state2[0], 0.0))
    dev.close()
    return out


if __name__ == "__main__":
    cfgs = [dict(J=2, delta=4, rank=1, n_y=4), dict(J=2, delta=3, rank=1, n_y=3, m=2, L=2),
            dict(J=3, delta=4, rank=2, n_y=5), dict(J=4, delta=20, rank=1, n_y=8),
            dict(J=2, delta=64, rank=2, n_y=64), dict(J=2, delta=128, rank=1, n_y=128),
            dict(J=2, delta=150, rank=1, n_y=140), dict(J=3, delta=5, rank=1, n_y=4, m=3, L=2)]
    for cfg in cfgs:
        t = time.time()
        try:
            o = run(cfg)
            worst = max(o.values())
            print(cfg, "worst=%.2e" % worst, "(%.1fs)" % (time.time() - t))
            print("   ", " ".join("%s=%.1e" % kv for kv in o.items()))
        except Exception as e:
            import traceback; traceback.print_exc()
            print(cfg, "FAILED", e)
