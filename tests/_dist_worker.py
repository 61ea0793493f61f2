"""Worker for tests/test_gpu_dist.py: one rank of a sharded run on a (shared) GPU, exchanging
through torch.distributed gloo (host-staged) or, with argv[4] = "rccl", the library's own RCCL
communicator, printing its iteration log as JSON."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import _clrsdp_pkg  # noqa: E402


def main():
    out = sys.argv[1]
    iters = int(sys.argv[2])
    pk = _clrsdp_pkg.load()
    from clrsdp_amd import dist as cdist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    backend = sys.argv[4] if len(sys.argv) > 4 else "gloo"
    ex = cdist.RcclExchange(0) if backend == "rccl" else cdist.TorchExchange(0, backend="gloo")
    J = int(os.environ.get("CLRSDP_TEST_J", "5"))
    cons, b = pk.synth(seed=12, J=J, delta=16, rank=1, n_y=9, m=1)
    bi = pk.get_block_info(cons)
    owned = pk.partition_clusters(bi, world)[rank]
    dev = pk.DeviceSolver(cons, b, bi, device=0, rank=rank, world=world, owned=owned)
    ex.attach(dev)
    if len(sys.argv) > 3 and sys.argv[3] == "solve":
        # the whole solverank1sdp loop, sharded (pipelined host loop by default at world > 1)
        res = pk.solverank1sdp(cons, b, bi, solver=dev, omega_p=10.0, omega_d=10.0,
                               duality_gap_threshold=1e-6, primal_error_threshold=1e-6,
                               dual_error_threshold=1e-6, verbose=False, return_info=True)
        info = res[-1]
        json.dump({"rank": rank, "log": [list(r[2:]) for r in info.log], "status": info.status,
                   "y": list(map(float, res[2])), "p_obj": res[8], "d_obj": res[9]},
                  open(f"{out}.{rank}.json", "w"))
        dev.close()
        ex.close()
        return
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    if len(sys.argv) > 3 and sys.argv[3] == "failone":
        # Y of one cluster of rank 0 negative definite: its S_j Cholesky fails on rank 0 only;
        # the failure bits travel with STEP's exchange, so both ranks must fall back to LU
        # together and then report the reference's step-length error (cho!(Y) fails)
        from clrsdp_amd import _lib as L
        x, X, y, Y = pk.initial_point(bi, 10.0, 10.0)
        bad = pk.partition_clusters(bi, world)[0][0]
        Y[bad] = [-0.5 * yb for yb in Y[bad]]
        dev.set_state(x, X, y, Y)
        code = 0
        try:
            dev.iterate(P, False)
        except L.ClrsdpError as e:
            code = e.code
        x2, X2, y2, Y2 = dev.get_state()
        unchanged = bool((x2 == x).all() and (y2 == y).all())
        json.dump({"rank": rank, "owned": owned, "bad": bad, "code": code,
                   "fact": dev.factorization, "unchanged": unchanged},
                  open(f"{out}.{rank}.json", "w"))
        dev.close()
        ex.close()
        return
    dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
    log = []
    for _ in range(iters):
        st = dev.iterate(P, False)
        log.append([st.mu, st.alpha_p, st.alpha_d, st.beta_c, st.p_obj, st.d_obj, st.P_err,
                    st.p_err, st.d_err])
    x, X, y, Y = dev.get_state()
    json.dump({"rank": rank, "owned": owned, "log": log, "y": list(map(float, y)),
               "x": list(map(float, x))}, open(f"{out}.{rank}.json", "w"))
    dev.close()
    ex.close()


if __name__ == "__main__":
    main()
