"""The fp64 loss of definiteness of Y on the 8-cluster C3 shard, pinned on
the device's own saved state (tests/golden/ypd_c3_8cl_block2.npz: block 2 of the dual iterate
before the body after which the next body reported "Y not PD", its dY and the device's alpha_d;
written by tools/ypd_probe.py on the GPU, J = 8, seed 0, body 54 of the synchronous loop without
bench.py's restarts; tools/ypd_check.py runs the comparison with the fp64 oracle).

What it shows ("fp64 stagnation"): at that state Y itself is singular to fp64
resolution (lambda_min / lambda_max ~ 1e-18), and Y + alpha_d dY formed EXACTLY from the device's
fp64 operands is indefinite -- so the failure is fp64's, not a device rounding or step-length
error.  The fp64 oracle (numpy restatement of MPMP.jl:755-887) raises "not positive definite" on
the same state before it completes the body."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "ypd_c3_8cl_block2.npz")


def test_y_singular_to_fp64_resolution():
    z = np.load(GOLDEN)
    ev = np.linalg.eigvalsh(z["Y"])
    assert abs(ev[0]) / ev[-1] < 1e-16, (ev[0], ev[-1])


def test_exact_update_is_indefinite():
    """v^T (Y + alpha_d dY) v < 0, evaluated exactly (every fp64 product and sum at 400 bits),
    for the eigenvector v (rounded to fp64) of the smallest eigenvalue of the device's new Y:
    no rounding of the update can be blamed."""
    import mpmath
    z = np.load(GOLDEN)
    Y, dY, a = z["Y"], z["dY"], float(z["alpha_d"])
    w, V = np.linalg.eigh(z["Yn"])
    v = V[:, 0]
    with mpmath.workprec(400):
        am = mpmath.mpf(a)
        vm = [mpmath.mpf(float(t)) for t in v]
        q = mpmath.mpf(0)
        n = Y.shape[0]
        for i in range(n):
            row = mpmath.mpf(0)
            for k in range(n):
                row += (mpmath.mpf(float(Y[i, k])) + am * mpmath.mpf(float(dY[i, k]))) * vm[k]
            q += vm[i] * row
    assert q < 0, float(q)
    # and it is tiny against the block's scale: the new Y is singular at fp64 resolution
    assert abs(float(q)) < 1e-14 * float(np.abs(Y).max())
