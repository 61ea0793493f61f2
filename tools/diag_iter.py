"""Per-iteration log of one bench instance (bench.py's setup), for hunting numerical breakdowns:
prints mu, the steps, the errors and the gap of every loop body until --iters or the first
library error.  GPU box:  python3 tools/diag_iter.py --clusters 8 --iters 70 [--env K=V ...]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=0)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=70)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--restart", type=int, default=0, help="restore the initial point every N bodies (bench.py)")
    ap.add_argument("--timing2-after", type=int, default=0, help="timing mode 2 from body N on (bench.py: 6)")
    args = ap.parse_args()
    import bench
    import _clrsdp_pkg
    pk = _clrsdp_pkg.load()
    from clrsdp_amd.solver import make_control
    cfg = dict(bench.CONFIGS[args.config])
    if args.clusters:
        cfg["J"] = args.clusters
    cons, b = pk.synth(seed=args.seed, **cfg)
    bi = pk.get_block_info(cons)
    dev = pk.DeviceSolver(cons, b, bi, precision_words=1, device=0, rank=0, world=1, owned=None,
                          timing=False)
    if args.no_graph:
        dev.set_graph(False)
    prm = pk.make_params("0.3", "0.1", "0.7", 0)
    dev.set_control(make_control("1e-15", "1e-30", "1e-30"))
    x0, X0, y0, Y0 = pk.initial_point(bi, 100.0, 100.0)
    dev.set_state(x0, X0, y0, Y0)
    dev.initial_residuals(prm)
    dev.save_state()
    feas = False
    for it in range(1, args.iters + 1):
        if args.timing2_after and it == args.timing2_after:
            dev.set_timing(2)
        try:
            st = dev.iterate(prm, feas)
        except Exception as e:  # the library's error of this body
            print(f"iter {it}: {e}", flush=True)
            return 1
        feas = max(st.p_err, st.P_err) < 1e-30 and st.d_err < 1e-30
        if args.restart and it % args.restart == 0:
            dev.restore_state()
            feas = False
            print("restore", flush=True)
        print(f"iter {it:3d} mu {st.mu:.3e} ap {st.alpha_p:.4f} ad {st.alpha_d:.4f} "
              f"P {st.P_err:.2e} p {st.p_err:.2e} d {st.d_err:.2e} gap {st.gap_w[0]:.3e}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
