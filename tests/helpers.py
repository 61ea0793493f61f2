"""Shared test helpers: instances, dense reconstructions of the constraint matrices, metrics."""
import math

import numpy as np


def dense_A(cl, bi, j, t_idx):
    """Dense block-diagonal (list over l) constraint matrix A_{j,(r,s,k)} (MPMP.jl:385-386)."""
    m, N = bi.m[j], bi.n_samples[j]
    loc = t_idx
    k = loc % N
    rs = loc // N
    r = 0
    while (r + 1) * (r + 2) // 2 <= rs:
        r += 1
    s = rs - r * (r + 1) // 2
    E = np.zeros((m, m))
    if r == s:
        E[r, r] = 1.0
    else:
        E[r, s] = E[s, r] = 0.5
    out = []
    for l in range(bi.L[j]):
        d = bi.Y_blocksizes[j][l] // m
        W = np.zeros((d, d))
        for v, lam in zip(cl.A[l][k], cl.H[l][k]):
            v = np.asarray(v, dtype=float)
            W += float(lam) * np.outer(v, v)
        out.append(np.kron(E, W))
    return out


def rand_spd(n, rng, shift=1.0):
    G = rng.standard_normal((n, n))
    return G @ G.T / n + shift * np.eye(n)


def rel_err(a, b, scale=0.0):
    """max|a-b| / max(max|b|, scale); exact (mpmath) when either side holds mpf objects."""
    a = np.asarray(a).ravel()
    b = np.asarray(b).ravel()
    if a.size == 0:
        return 0.0
    if a.dtype == object or b.dtype == object:
        import mpmath
        num = max(abs(mpmath.mpf(x) - mpmath.mpf(y)) for x, y in zip(a, b))
        den = max([abs(mpmath.mpf(y)) for y in b] + [mpmath.mpf(scale), mpmath.mpf(1e-300)])
        return float(num / den)
    a = a.astype(float)
    b = b.astype(float)
    return float(np.max(np.abs(a - b)) / max(1e-300, float(np.max(np.abs(b))), scale))


def poly_min_instance(pk, coef=(2.0, 1.0, -3.0, 0.0, 1.0)):
    """max y s.t. p(x) - y is a sum of squares (univariate): optimum = min_x p(x).
    One cluster, m = 1, v_k = (1, x_k, x_k^2), lambda = 1, B = 1, c_k = p(x_k), b = 1."""
    N = len(coef)
    deg = (len(coef) - 1) // 2
    xs = np.cos(np.pi * (2 * np.arange(N) + 1) / (2 * N)) * 2.0
    A = [[[np.array([x ** i for i in range(deg + 1)])] for x in xs]]
    H = [[[1.0] for _ in xs]]
    B = np.ones((N, 1))
    c = np.array([np.polyval(list(coef)[::-1], x) for x in xs])
    dcoef = [i * coef[i] for i in range(1, len(coef))]
    r = np.roots(dcoef[::-1])
    r = r[np.abs(r.imag) < 1e-12].real
    pmin = float(min(np.polyval(list(coef)[::-1], r)))
    return [pk.Cluster(A, B, c, H)], np.array([1.0]), pmin


def stage_reference(it, nxt, bi):
    """The oracle's stage outputs of one iteration (``oracle.iteration``'s intermediates ``it``
    and new state ``nxt``) as flat arrays in the C-ABI buffer layout, in stage order.  Names
    match :func:`stage_device`."""
    from clrsdp_amd import instance as inst
    fl = inst.blocks_to_flat
    ay = [it["A_Y"][j][l][r][s] for j in range(bi.J) for l in range(bi.L[j])
          for r in range(bi.m[j]) for s in range(r + 1)]
    out = {"mu": np.array([it["mu"]], dtype=object), "R": fl(it["R"]), "Xinv": fl(it["X_inv"]),
           "S": np.concatenate([s.reshape(-1, order="F") for s in it["dec"].S_raw]),
           "A_Y": np.concatenate(ay), "Q": it["dec"].Q_raw.reshape(-1, order="F"),
           "P": fl(it["P"]), "p": np.asarray(it["p"]), "d": np.asarray(it["d"])}
    for key in ("pred", "corr"):
        if key == "corr":
            out["beta_c"] = np.array([it["beta_c"]], dtype=object)
            out["R2"] = fl(it["R2"])
        dx, dX, dy, dY = it[key]
        out[key + "_dx"], out[key + "_dy"] = np.asarray(dx), np.asarray(dy)
        out[key + "_dX"], out[key + "_dY"] = fl(dX), fl(dY)
    out["alpha_p"] = np.array([it["alpha_p"]], dtype=object)
    out["alpha_d"] = np.array([it["alpha_d"]], dtype=object)
    out["x+"], out["X+"] = np.asarray(nxt[0]), fl(nxt[1])
    out["y+"], out["Y+"] = np.asarray(nxt[2]), fl(nxt[3])
    return out


def stage_device(dev, exact):
    """Run the ten stages of one iteration on a DeviceSolver whose state is set, reading every
    stage's buffers back (the C-ABI layout of :func:`stage_reference`)."""
    from clrsdp_amd import _lib as L
    from clrsdp_amd import instance as inst
    import _clrsdp_pkg
    pk = _clrsdp_pkg.load()
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    buf = lambda k: np.array(dev.buffer(k, exact), dtype=object if exact else float)
    o = {}
    dev.run_stage(L.STAGE_MU_R, P, False)
    o["mu"] = np.array([dev.scalar("mu", exact)], dtype=object)
    o["R"] = buf(L.BUF_R)
    dev.run_stage(L.STAGE_XINV, P, False)
    o["Xinv"] = buf(L.BUF_XINV)
    dev.run_stage(L.STAGE_SCHUR, P, False)
    o["S"], o["A_Y"] = buf(L.BUF_S), buf(L.BUF_AY)
    dev.run_stage(L.STAGE_FACTOR, P, False)
    o["Q"] = buf(L.BUF_Q)
    dev.run_stage(L.STAGE_RESIDUALS, P, False)
    o["P"], o["p"], o["d"] = buf(L.BUF_P), buf(L.BUF_PVEC), buf(L.BUF_DVEC)
    for stage, key in ((L.STAGE_PREDICTOR, "pred"), (L.STAGE_CORRECTOR, "corr")):
        if key == "corr":
            dev.run_stage(L.STAGE_CORRECTOR_R, P, False)
            o["beta_c"] = np.array([dev.scalar("beta_c", exact)], dtype=object)
            o["R2"] = buf(L.BUF_R)
        dev.run_stage(stage, P, False)
        o[key + "_dx"], o[key + "_dy"] = buf(L.BUF_DX), buf(L.BUF_DY)
        o[key + "_dX"], o[key + "_dY"] = buf(L.BUF_DXMAT), buf(L.BUF_DYMAT)
    dev.run_stage(L.STAGE_STEP, P, False)
    o["alpha_p"] = np.array([dev.scalar("alpha_p", exact)], dtype=object)
    o["alpha_d"] = np.array([dev.scalar("alpha_d", exact)], dtype=object)
    dev.run_stage(L.STAGE_UPDATE, P, False)
    xg, Xg, yg, Yg = dev.get_state(exact)
    o["x+"], o["X+"] = np.asarray(xg), inst.blocks_to_flat(Xg)
    o["y+"], o["Y+"] = np.asarray(yg), inst.blocks_to_flat(Yg)
    return o


def residual_scales(cons, b, X):
    """Scales for the residual buffers, which are themselves at round-off level once feasible:
    P against the X scale, p against b, d against c."""
    from clrsdp_amd import instance as inst
    Xscale = float(np.max(np.abs(np.array(inst.blocks_to_flat(X), dtype=float))))
    return {"P": Xscale, "p": float(np.max(np.abs(np.array(b, dtype=float)))),
            "d": float(max(np.max(np.abs(np.array(c.c, dtype=float))) for c in cons))}


# ---- sampled fixtures of large stage outputs (tests/golden/make_stage_fixtures.py) ----------
SKETCH_MULT = (0x9E3779B1, 0x85EBCA77)


def sketch_weights(n, which):
    """Deterministic +-1 weights for the linear sketch number ``which`` of an n-vector."""
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = (i + np.uint64(1)) * np.uint64(SKETCH_MULT[which]) & np.uint64(0xFFFFFFFF)
    return 1 - 2 * ((h >> np.uint64(13)) & np.uint64(1)).astype(np.int64)


def sample_indices(n, count=384, seed=2024):
    """Sorted sample of indices: the first and last 32 entries and ``count`` spread by a
    fixed multiplicative hash (no RNG, identical on every host)."""
    if n <= count + 64:
        return list(range(n))
    s = set(range(32)) | set(range(n - 32, n))
    k = 0
    while len(s) < count + 64:
        s.add(int((k * 2654435761 + seed * 40503) % n))
        k += 1
    return sorted(s)


def summarize(arr, digits):
    """Fixture record of a flat buffer: sampled entries, two +-1 sketches, the l1 norm and the
    max |entry| (decimal strings at ``digits`` significant digits)."""
    import mpmath
    a = [mpmath.mpf(v) for v in np.asarray(arr, dtype=object).ravel()]
    n = len(a)
    idx = sample_indices(n)
    st = lambda v: mpmath.nstr(v, digits, strip_zeros=False, min_fixed=1, max_fixed=0)
    rec = {"n": n, "idx": idx, "val": [st(a[i]) for i in idx],
           "l1": st(mpmath.fsum(abs(v) for v in a)), "amax": st(max([abs(v) for v in a] + [mpmath.mpf(0)]))}
    rec["sketch"] = [st(mpmath.fsum(int(w) * v for w, v in zip(sketch_weights(n, q), a))) for q in range(2)]
    return rec


def compare_summary(arr, rec, scale=0.0):
    """Scale-aware relative error of a device buffer against a fixture record: max over the
    sampled entries (relative to max(amax, scale)) and the sketches (relative to l1)."""
    import mpmath
    a = np.asarray(arr, dtype=object).ravel()
    assert len(a) == rec["n"], (len(a), rec["n"])
    # the fixture strings are parsed and the differences taken at 320 bits whatever the global
    # mpmath.mp.prec is (a test run that starts with this comparison has it at 53)
    with mpmath.workprec(320):
        den = max(mpmath.mpf(rec["amax"]), mpmath.mpf(scale), mpmath.mpf(1e-300))
        err = max([abs(mpmath.mpf(a[i]) - mpmath.mpf(v)) / den
                   for i, v in zip(rec["idx"], rec["val"])] + [mpmath.mpf(0)])
        l1 = max(mpmath.mpf(rec["l1"]), mpmath.mpf(scale) * len(a), mpmath.mpf(1e-300))
        for q, sv in enumerate(rec["sketch"]):
            s = mpmath.fsum(int(w) * mpmath.mpf(v) for w, v in zip(sketch_weights(len(a), q), a))
            err = max(err, abs(s - mpmath.mpf(sv)) / l1)
    return float(err)


CONFIGS_SMALL = [
    dict(J=2, delta=4, rank=1, n_y=4),                    # C1
    dict(J=2, delta=3, rank=1, n_y=3, m=2, L=2),          # polynomial-matrix clusters, 2 blocks
    dict(J=3, delta=4, rank=2, n_y=5),                    # rank 2
    dict(J=3, delta=5, rank=1, n_y=4, m=3, L=2),          # m = 3
    dict(J=1, delta=6, rank=1, n_y=1),                    # single cluster, n_y = 1
]
