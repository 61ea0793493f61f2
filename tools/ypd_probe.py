"""Find the loop body after which Y loses definiteness on a bench instance
and save what is needed to decide whether the device or fp64 itself is at fault.

Runs bench.py's setup (synthetic instance, reference initial point, device loop control, the
synchronous loop) WITHOUT bench.py's restarts.  Keeps the state before every body; when a body
fails, re-runs the body before it (the one that produced the failing iterate) stage by stage from
its saved state -- bitwise the loop body -- and saves to --out (npz): that state (x, X, y, Y), its
dX, dY, alpha_p, alpha_d, mu, the next state the device produced, and the per-iteration log.
GPU box:  python3 tools/ypd_probe.py --clusters 8 --iters 300 --out gpurun_out/ypd/state.npz
CPU:      python3 tools/ypd_check.py gpurun_out/ypd/state.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def flat(blocks):
    return np.concatenate([np.ravel(m, order="F") for bj in blocks for m in bj])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=8)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/ypd/state.npz")
    args = ap.parse_args()
    import bench
    import _clrsdp_pkg
    pk = _clrsdp_pkg.load()
    from clrsdp_amd import _lib as L
    from clrsdp_amd.solver import make_control
    cfg = dict(bench.CONFIGS[args.config])
    if args.clusters:
        cfg["J"] = args.clusters
    cons, b = pk.synth(seed=args.seed, **cfg)
    bi = pk.get_block_info(cons)
    dev = pk.DeviceSolver(cons, b, bi, precision_words=1, device=0, rank=0, world=1, owned=None,
                          timing=False)
    prm = pk.make_params("0.3", "0.1", "0.7", 0)
    dev.set_control(make_control("1e-15", "1e-30", "1e-30"))
    x0, X0, y0, Y0 = pk.initial_point(bi, 100.0, 100.0)
    dev.set_state(x0, X0, y0, Y0)
    dev.initial_residuals(prm)
    feas = False
    log = []
    hist = []  # (state, feas) before each body, the last three
    fail = None
    for it in range(1, args.iters + 1):
        hist = (hist + [(dev.get_state(), feas)])[-3:]
        try:
            st = dev.iterate(prm, feas)
        except Exception as e:  # noqa: BLE001
            print(f"iter {it}: {e}", flush=True)
            fail = (it, str(e))
            break
        feas = max(st.p_err, st.P_err) < 1e-30 and st.d_err < 1e-30
        log.append([it, st.mu, st.alpha_p, st.alpha_d, st.P_err, st.p_err, st.d_err, st.gap_w[0]])
        print(f"iter {it:3d} mu {st.mu:.3e} ap {st.alpha_p:.4f} ad {st.alpha_d:.4f} "
              f"P {st.P_err:.2e} p {st.p_err:.2e} d {st.d_err:.2e} gap {st.gap_w[0]:.3e}", flush=True)
    out = {"log": np.array(log), "J": bi.J, "seed": args.seed, "n_y": bi.n_y,
           "delta": cfg["delta"], "rank": cfg["rank"], "failed_at": fail[0] if fail else -1,
           "error": fail[1] if fail else ""}
    if fail and len(hist) >= 2:
        (x, X, y, Y), feas_b = hist[-2]       # the state before the body that produced the bad iterate
        (xn, Xn, yn, Yn), _ = hist[-1]        # the iterate it produced (on which the next body failed)
        dev.set_graph(False)
        dev.set_state(x, X, y, Y)
        for s in range(L.NUM_STAGES):
            dev.run_stage(s, prm, feas_b)
            if s == L.STAGE_CORRECTOR:
                dXm, dYm = dev.buffer(L.BUF_DXMAT), dev.buffer(L.BUF_DYMAT)
                dx, dy = dev.buffer(L.BUF_DX), dev.buffer(L.BUF_DY)
            if s == L.STAGE_STEP:
                sc = dev.buffer(L.BUF_SCALARS)
        x2, X2, y2, Y2 = dev.get_state()
        out.update(x=x, X=flat(X), y=y, Y=flat(Y), xn=xn, Xn=flat(Xn), yn=yn, Yn=flat(Yn),
                   dX=dXm, dY=dYm, dx=dx, dy=dy, feas=feas_b,
                   alpha_p=float(sc[L.SC["alpha_p"]]), alpha_d=float(sc[L.SC["alpha_d"]]),
                   mineig_X=float(sc[L.SC["mineig_X"]]), mineig_Y=float(sc[L.SC["mineig_Y"]]),
                   mu=float(sc[L.SC["mu"]]),
                   replay_equal=bool(np.array_equal(flat(Y2), flat(Yn)) and np.array_equal(flat(X2), flat(Xn))))
        print("replayed body equal to the loop's:", out["replay_equal"], " alpha_d", out["alpha_d"],
              " mineig_Y", out["mineig_Y"], flush=True)
    dev.close()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    np.savez_compressed(args.out, **out)
    print("saved", args.out, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
