"""CPU side of tools/ypd_probe.py: given the saved state of the body after which the device's Y
lost definiteness, run the fp64 oracle's iteration (oracle/mpmp_oracle.py, MPMP.jl:755-887) from
the same state and compare the two bodies: alpha_p, alpha_d, lambda_min of L^-1 dY L^-T, and the
definiteness of the new Y (numpy Cholesky per block, and lambda_min of the exact sum
Y + alpha_d dY of the device's own fp64 operands at 200 bits for the blocks that fail).
   python3 tools/ypd_check.py gpurun_out/r6e/ypd.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def blocks(flat, bi):
    out, off = [], 0
    for bj in bi.Y_blocksizes:
        row = []
        for n in bj:
            row.append(np.asarray(flat[off:off + n * n]).reshape(n, n, order="F"))
            off += n * n
        out.append(row)
    return out


def pd(M):
    try:
        np.linalg.cholesky(M)
        return True
    except np.linalg.LinAlgError:
        return False


def main(path):
    import _clrsdp_pkg
    from oracle import mpmp_oracle as O
    pk = _clrsdp_pkg.load()
    z = np.load(path)
    J, seed = int(z["J"]), int(z["seed"])
    cons, b = pk.synth(seed=seed, J=J, delta=int(z["delta"]), rank=int(z["rank"]), n_y=int(z["n_y"]))
    bi = pk.get_block_info(cons)
    print(f"instance J={J} seed={seed}; device failed at body {int(z['failed_at'])}: {z['error']}")
    X, Y, Xn, Yn = (blocks(z[k], bi) for k in ("X", "Y", "Xn", "Yn"))
    dX, dY = blocks(z["dX"], bi), blocks(z["dY"], bi)
    a_p, a_d = float(z["alpha_p"]), float(z["alpha_d"])
    print(f"device body before it: mu {float(z['mu']):.4e} alpha_p {a_p:.6e} alpha_d {a_d:.6e} "
          f"lambda_min(L^-1 dX L^-T) {float(z['mineig_X']):.6e} lambda_min(L^-1 dY L^-T) {float(z['mineig_Y']):.6e}")
    cond_Y = max(np.linalg.cond(Y[j][0]) for j in range(J))
    print(f"cond(Y) max over blocks at that state: {cond_Y:.3e};  ||dY|| / ||Y|| max: "
          f"{max(np.abs(dY[j][0]).max() / np.abs(Y[j][0]).max() for j in range(J)):.3e}")
    bad = [j for j in range(J) if not pd(Yn[j][0])]
    print("device's new Y: blocks failing numpy Cholesky:", bad)
    # the same body through the fp64 oracle
    ar = O.Fp64()
    prm = {k: O._param(ar, v) for k, v in O.DEFAULTS.items()}
    bo = O.get_block_info(cons)
    st = (np.asarray(z["x"]), [[m.copy() for m in bj] for bj in X], np.asarray(z["y"]),
          [[m.copy() for m in bj] for bj in Y])
    try:
        (xo, Xo, yo, Yo), it = O.iteration(ar, cons, bo, b, None, 0.0, st, bool(z["feas"]), prm)
        print(f"oracle body:           mu {float(it['mu']):.4e} alpha_p {float(it['alpha_p']):.6e} "
              f"alpha_d {float(it['alpha_d']):.6e}")
        badO = [j for j in range(J) if not pd(np.asarray(Yo[j][0], dtype=float))]
        print("oracle's new Y: blocks failing numpy Cholesky:", badO)
    except Exception as e:  # noqa: BLE001  (the oracle's own error, e.g. a singular S_j)
        print("oracle body raised:", type(e).__name__, e)
    # exact Y + alpha_d dY from the device's own operands, for the failing blocks
    import mpmath
    with mpmath.workprec(200):
        for j in bad[:2]:
            n = Y[j][0].shape[0]
            A = mpmath.matrix(n, n)
            for r in range(n):
                for c in range(n):
                    A[r, c] = mpmath.mpf(float(Y[j][0][r, c])) + mpmath.mpf(a_d) * mpmath.mpf(float(dY[j][0][r, c]))
            ev = mpmath.eigsy(A, eigvals_only=True)
            lo = min(ev)
            evd = np.linalg.eigvalsh(Yn[j][0])
            print(f"block {j}: exact lambda_min(Y + alpha_d dY) = {float(lo):.6e} "
                  f"(largest {float(max(ev)):.3e});  fp64 device Y_new lambda_min {evd[0]:.6e}; "
                  f"lambda_min(Y) {np.linalg.eigvalsh(Y[j][0])[0]:.6e}")


if __name__ == "__main__":
    main(sys.argv[1])
