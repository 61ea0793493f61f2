"""Host mirror of ``solverank1sdp`` (MPMP.jl:595-1025) driving the MI355X library.

The loop control, the termination test, the printed table and the returned 11-tuple follow
the reference exactly; every loop body (MPMP.jl:755-887) is one ``clrsdp_iterate`` call that
runs entirely on the GPU.  Numbers cross the boundary as planar limbs (``precision_words`` 1 =
fp64, 2 = double-double).
"""
from __future__ import annotations

import ctypes as C
import time
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .blockinfo import BlockInfo
from .instance import Flat, blocks_to_flat, concat_colmajor, flat_to_blocks, flatten, from_planes, \
    to_planes

DEFAULTS = dict(beta_infeasible="0.3", beta_feasible="0.1", gamma="0.7", omega_p="1e10",
                omega_d="1e10", duality_gap_threshold="1e-15", primal_error_threshold="1e-30",
                dual_error_threshold="1e-30")


def limbs(v, words=4):
    """A scalar (float, str, mpmath.mpf) as `words` limbs of an unevaluated sum."""
    import mpmath
    with mpmath.workprec(320):
        r = mpmath.mpf(v) if not isinstance(v, float) else mpmath.mpf(v)
        out = []
        for _ in range(words):
            h = float(r)
            out.append(h)
            r = r - h
    return out


def make_params(beta_infeasible, beta_feasible, gamma, b0) -> _lib.Params:
    p = _lib.Params()
    for name, v in (("beta_infeasible", beta_infeasible), ("beta_feasible", beta_feasible),
                    ("gamma", gamma), ("b0", b0)):
        arr = getattr(p, name)
        for i, x in enumerate(limbs(v)):
            arr[i] = x
    return p


def make_control(duality_gap_threshold, primal_error_threshold, dual_error_threshold,
                 need_primal_feasible=False, need_dual_feasible=False) -> _lib.Control:
    c = _lib.Control()
    for name, v in (("duality_gap_threshold", duality_gap_threshold),
                    ("primal_error_threshold", primal_error_threshold),
                    ("dual_error_threshold", dual_error_threshold)):
        arr = getattr(c, name)
        for i, x in enumerate(limbs(v)):
            arr[i] = x
    c.need_primal_feasible = 1 if need_primal_feasible else 0
    c.need_dual_feasible = 1 if need_dual_feasible else 0
    return c


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_lib.P_f64)


class DeviceSolver:
    """One handle of libclrsdp: constraint data resident on one GPU (the clusters of this rank)."""

    def __init__(self, constraints: Sequence, b, bi: BlockInfo, precision_words: int = 1,
                 C_blocks=None, device: int = 0, rank: int = 0, world: int = 1,
                 owned: Optional[Sequence[int]] = None, timing: bool = False):
        self.L = _lib.lib()
        self.bi = bi
        self.w = int(precision_words)
        self.rank, self.world = rank, world
        flat = flatten(constraints, bi)
        self.flat = flat
        self._keep = []
        desc = _lib.Desc()
        desc.J = bi.J
        desc.n_y = bi.n_y
        for name in ("m", "L", "n_samples", "delta", "ranks"):
            arr = np.ascontiguousarray(getattr(flat, name), dtype=np.int64)
            self._keep.append(arr)
            setattr(desc, name, arr.ctypes.data_as(_lib.P_i64))
        cfg = _lib.Config()
        cfg.precision_words = self.w
        cfg.device = device
        cfg.rank = rank
        cfg.world_size = world
        if owned is not None:
            own = np.ascontiguousarray(sorted(owned), dtype=np.int32)
            self._keep.append(own)
            cfg.owned = own.ctypes.data_as(_lib.P_i32)
            cfg.n_owned = len(own)
        cfg.timing = 1 if timing else 0
        self.timing = bool(timing)
        h = C.c_void_p()
        _lib.check(self.L.clrsdp_create(C.byref(desc), C.byref(cfg), C.byref(h)))
        self.h = h
        self.owned = sorted(owned) if owned is not None else list(range(bi.J))
        w = self.w
        Vp = to_planes(concat_colmajor(flat.V), w)
        lp = to_planes(np.concatenate(flat.lam), w)
        Bp = to_planes(concat_colmajor(flat.B), w)
        cp = to_planes(np.concatenate(flat.c), w)
        bp = to_planes(np.asarray(b), w)
        Cp = to_planes(blocks_to_flat(C_blocks), w) if C_blocks is not None else None
        self.check(self.L.clrsdp_upload_constraints(
            self.h, _ptr(Vp), _ptr(lp), _ptr(Bp), _ptr(cp), _ptr(bp),
            _ptr(Cp) if Cp is not None else None))
        self.n_x = sum(bi.dim_S)
        self.n_blk = sum(n * n for bj in bi.Y_blocksizes for n in bj)

    # ------------------------------------------------------------------ plumbing
    def check(self, rc):
        _lib.check(rc, self.h)

    def close(self):
        if getattr(self, "h", None):
            self.L.clrsdp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _from_planes(self, planes: np.ndarray, n: int, exact=False):
        if self.w == 1 or not exact:
            return planes[:n].copy()
        return from_planes(planes, n, self.w)

    # ------------------------------------------------------------------ state
    def set_state(self, x, X, y, Y):
        w = self.w
        xp = to_planes(np.asarray(x), w)
        Xp = to_planes(blocks_to_flat(X), w)
        yp = to_planes(np.asarray(y), w)
        Yp = to_planes(blocks_to_flat(Y), w)
        self.check(self.L.clrsdp_set_state(self.h, _ptr(xp), _ptr(Xp), _ptr(yp), _ptr(Yp)))

    def get_state(self, exact=False):
        w = self.w
        xp = np.zeros(w * self.n_x)
        Xp = np.zeros(w * self.n_blk)
        yp = np.zeros(w * self.bi.n_y)
        Yp = np.zeros(w * self.n_blk)
        self.check(self.L.clrsdp_get_state(self.h, _ptr(xp), _ptr(Xp), _ptr(yp), _ptr(Yp)))
        x = self._from_planes(xp, self.n_x, exact)
        y = self._from_planes(yp, self.bi.n_y, exact)
        X = flat_to_blocks(self._from_planes(Xp, self.n_blk, exact), self.bi)
        Y = flat_to_blocks(self._from_planes(Yp, self.n_blk, exact), self.bi)
        return x, X, y, Y

    def buffer(self, buf: int, exact=False) -> np.ndarray:
        cnt = C.c_int64()
        self.check(self.L.clrsdp_get_buffer(self.h, buf, None, C.byref(cnt)))
        n = cnt.value
        out = np.zeros(self.w * max(n, 1))
        self.check(self.L.clrsdp_get_buffer(self.h, buf, _ptr(out), C.byref(cnt)))
        return self._from_planes(out, n, exact)

    def global_P_d(self):
        """P (blocks) and d (vector) in the global layout of get_state: the device buffers hold
        the owned clusters only (in owned order); the other clusters' entries are zero, as in
        get_state, and live on the ranks that own them."""
        bi = self.bi
        Pl, dl = self.buffer(_lib.BUF_P), self.buffer(_lib.BUF_DVEC)
        if len(self.owned) == bi.J:
            return flat_to_blocks(Pl, bi), dl
        P = [[np.zeros((n, n)) for n in bj] for bj in bi.Y_blocksizes]
        d = np.zeros(self.n_x)
        xoff = np.concatenate([[0], np.cumsum(bi.dim_S)])
        po = lo = 0
        for j in self.owned:
            for l, n in enumerate(bi.Y_blocksizes[j]):
                P[j][l] = np.asarray(Pl[po:po + n * n]).reshape(n, n, order="F")
                po += n * n
            D = bi.dim_S[j]
            d[xoff[j]:xoff[j] + D] = dl[lo:lo + D]
            lo += D
        return P, d

    def scalar(self, name: str, exact=False):
        return self.buffer(_lib.BUF_SCALARS, exact)[_lib.SC[name]]

    # ------------------------------------------------------------------ iteration
    def initial_residuals(self, prm: _lib.Params) -> _lib.IterStats:
        st = _lib.IterStats()
        self.check(self.L.clrsdp_initial_residuals(self.h, C.byref(prm), C.byref(st)))
        return st

    def iterate(self, prm: _lib.Params, pd_feas: bool) -> _lib.IterStats:
        st = _lib.IterStats()
        self.check(self.L.clrsdp_iterate(self.h, C.byref(prm), 1 if pd_feas else 0, C.byref(st)))
        return st

    def set_control(self, ctl: _lib.Control):
        self.check(self.L.clrsdp_set_control(self.h, C.byref(ctl)))

    def iterate_async(self, prm: _lib.Params):
        """Enqueue one loop body (pd_feas / termination decided on the device); no wait."""
        self.check(self.L.clrsdp_iterate_async(self.h, C.byref(prm)))

    def iterate_wait(self):
        """Stats of the oldest loop body in flight and whether it ran (0: the device had
        terminated before it)."""
        st = _lib.IterStats()
        ran = C.c_int32(0)
        self.check(self.L.clrsdp_iterate_wait(self.h, C.byref(st), C.byref(ran)))
        return st, bool(ran.value)

    def run_stage(self, stage: int, prm: _lib.Params, pd_feas: bool):
        self.check(self.L.clrsdp_run_stage(self.h, stage, C.byref(prm), 1 if pd_feas else 0))

    def synchronize(self):
        self.check(self.L.clrsdp_synchronize(self.h))

    def set_timing(self, on):
        """Per-stage HIP-event timing: False/0 off, True/1 every stage (no graph), 2 only the
        SCHUR stage, from device-clock stamps inside the replayed loop-body graph (off or 2 + one rank:
        iterate replays a hipGraph)."""
        mode = 2 if on == 2 else (1 if on else 0)
        self.check(self.L.clrsdp_set_timing(self.h, mode))
        self.timing = mode == 1

    def save_state(self):
        """Device-side snapshot of x, X, y, Y and the scalar slots (clrsdp_save_state)."""
        self.check(self.L.clrsdp_save_state(self.h))

    def restore_state(self):
        """Restore the last snapshot, stream-ordered after the work already enqueued."""
        self.check(self.L.clrsdp_restore_state(self.h))

    def set_factorization(self, flags: int):
        """clrsdp_set_factorization: FACT_FALLBACK (default: pivoted LU once a Cholesky fails),
        FACT_LU_SQ (S_j and Q by pivoted LU, the reference's approx_lu!), FACT_LU_X (X^-1 by
        approx_inv!)."""
        self.check(self.L.clrsdp_set_factorization(self.h, int(flags)))

    @property
    def factorization(self) -> int:
        f = C.c_int32(0)
        self.check(self.L.clrsdp_get_factorization(self.h, C.byref(f)))
        return f.value

    def set_graph(self, on: bool):
        """clrsdp_set_graph: hipGraph replay of the loop body on/off (off: eager enqueue)."""
        self.check(self.L.clrsdp_set_graph(self.h, 1 if on else 0))

    def comm_info(self):
        """(ranks, backend) of the exchange: backend 'none', 'rccl' (native communicator, ranks
        from ncclCommCount) or 'callback' (clrsdp_set_exchange)."""
        n, b = C.c_int32(0), C.c_int32(0)
        self.check(self.L.clrsdp_comm_info(self.h, C.byref(n), C.byref(b)))
        return n.value, {0: "none", 1: "rccl", 2: "callback"}.get(b.value, str(b.value))

    def set_stream(self, stream_ptr: int):
        self.check(self.L.clrsdp_set_stream(self.h, C.c_void_p(stream_ptr)))

    def stream_ptr(self) -> int:
        """The hipStream_t every launch of this handle goes to."""
        return self.L.clrsdp_get_stream(self.h) or 0

    def exchange_bytes(self) -> int:
        b = C.c_int64()
        self.check(self.L.clrsdp_exchange_bytes(self.h, C.byref(b)))
        return b.value

    def comm_init(self, uid: bytes):
        """Attach the native RCCL communicator (clrsdp_comm_init): every rank passes the id rank 0
        got from :func:`comm_unique_id`; the exchanges are then all-gathers issued by the
        library on its stream.  With one rank they are captured into the replayed loop-body
        graph; with more ranks the body is enqueued eagerly unless CLRSDP_GRAPH_RCCL=1."""
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError("RCCL unique id must be %d bytes" % _lib.COMM_ID_BYTES)
        self.check(self.L.clrsdp_comm_init(self.h, bytes(uid)))

    def set_exchange(self, fn, send_ptr: int, recv_ptr: int):
        self._xfn = _lib.EXCHANGE_FN(fn)
        self.check(self.L.clrsdp_set_exchange(self.h, self._xfn, None, C.c_void_p(send_ptr),
                                              C.c_void_p(recv_ptr)))


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (clrsdp_comm_unique_id), to be created on rank 0 only."""
    buf = C.create_string_buffer(_lib.COMM_ID_BYTES)
    _lib.check(_lib.lib().clrsdp_comm_unique_id(buf))
    return buf.raw


def compute_step_length(M, dM, gamma, device: int = 0, return_eigs: bool = False):
    """compute_step_length(M, dM, gamma, blockinfo) of MPMP.jl:1829-1898 on the GPU (fp64,
    clrsdp_step_length): ``min(1, -gamma / lambda_min)`` over the blocks of L^-1 dM L^-T with
    M = L L^T.  ``M`` and ``dM`` are nested block lists (as X/Y) or flat lists of square
    arrays.  Returns ``(alpha, bigfloat_steplength)`` as the reference does (the flag is always
    False: there is no ball-arithmetic fallback), plus the per-block lambda_min with
    ``return_eigs``.  Raises ClrsdpError(E_STEP) when a block of M is not positive definite."""
    def flat(blocks):
        out = []
        for b in blocks:
            if isinstance(b, (list, tuple)):
                out.extend(flat(b))
            else:
                out.append(np.asarray(b, dtype=np.float64))
        return out
    Mb, dMb = flat(M), flat(dM)
    if len(Mb) != len(dMb) or not Mb:
        raise ValueError("M and dM need the same non-empty block structure")
    for a, b in zip(Mb, dMb):
        if a.ndim != 2 or a.shape[0] != a.shape[1] or a.shape != b.shape:
            raise ValueError("blocks must be square and M, dM blocks of equal size")
    n = np.array([a.shape[0] for a in Mb], dtype=np.int64)
    Mf = np.concatenate([a.ravel(order="F") for a in Mb])
    dMf = np.concatenate([b.ravel(order="F") for b in dMb])
    alpha = C.c_double(0.0)
    eig = np.zeros(len(Mb))
    _lib.check(_lib.lib().clrsdp_step_length(device, len(Mb), n.ctypes.data_as(_lib.P_i64),
                                              _ptr(Mf), _ptr(dMf), float(gamma), C.byref(alpha),
                                              _ptr(eig)))
    if return_eigs:
        return alpha.value, False, eig
    return alpha.value, False


def eigmin(blocks, precision_words: int = 1, device: int = 0):
    """lambda_min of each exactly symmetric block at fp64 / double-double / quad-double
    (clrsdp_eigmin; the eigenvalue part of compute_step_length, MPMP.jl:1857-1870).  Blocks are
    float arrays or object arrays of mpmath numbers (split exactly into limbs); returns floats
    (words 1) or mpmath numbers (the exact limb sums)."""
    w = int(precision_words)
    mats = [np.asarray(b) for b in blocks]
    for a in mats:
        if a.ndim != 2 or a.shape[0] != a.shape[1] or a.shape[0] < 1:
            raise ValueError("blocks must be square")
    n = np.array([a.shape[0] for a in mats], dtype=np.int64)
    flat = np.concatenate([a.reshape(-1, order="F") for a in mats])
    planes = to_planes(flat, w)
    out = np.zeros(w * len(mats))
    _lib.check(_lib.lib().clrsdp_eigmin(device, w, len(mats), n.ctypes.data_as(_lib.P_i64),
                                        _ptr(planes), _ptr(out)))
    if w == 1:
        return out
    return from_planes(out, len(mats), w)


def initial_point(bi: BlockInfo, omega_p, omega_d):
    """x = 0, X = omega_p I, y = 0, Y = omega_d I (MPMP.jl:660-686)."""
    x = np.zeros(sum(bi.dim_S))
    X = [[float(omega_p) * np.eye(n) for n in bj] for bj in bi.Y_blocksizes]
    y = np.zeros(bi.n_y)
    Y = [[float(omega_d) * np.eye(n) for n in bj] for bj in bi.Y_blocksizes]
    return x, X, y, Y


def device_threshold(v, words):
    """A threshold as the device holds it at `words` limbs (clrsdp_set_control sums the first
    `words` limbs of :func:`limbs` in the word type, exactly): a float at fp64, else the exact
    mpmath value, so host comparisons at dd/qd are the device's own."""
    lv = limbs(v)
    if words == 1:
        return lv[0]
    import mpmath
    s = mpmath.mpf(0)
    for x in lv[:words]:
        s = mpmath.fadd(s, x, exact=True)
    return s


def _terminate(gap, perr, derr, gthr, pthr, dthr, need_p, need_d, out):
    """MPMP.jl:1147-1173."""
    gap_opt, pf, df = gap < gthr, perr < pthr, derr < dthr
    if need_p and pf:
        out("Primal feasible solution found")
        return True
    if need_d and df:
        out("Dual feasible solution found")
        return True
    if pf and df and gap_opt:
        out("Optimal solution found")
        return True
    return False


def log_row(it, t, st, p_obj, d_obj, dual_gap):
    """One row of the iteration table (MPMP.jl:923-937).  Every column is a float (the leading
    double of the device's value) except the gap, which is the loop control's own value: a float
    at fp64, the full-width mpmath number at dd/qd (the value terminate() compared, MPMP.jl:
    942-945, 1147-1173); the other columns at full width are in RunInfo.exact (record_exact)."""
    gap = dual_gap if not isinstance(dual_gap, (float, int, np.floating)) else float(dual_gap)
    return (int(it), float(t), float(st.mu), float(p_obj), float(d_obj), gap,
            float(st.P_err), float(st.p_err), float(st.d_err), float(st.alpha_p),
            float(st.alpha_d), float(st.beta_c))


HEADER = "%5s %8s %11s %11s %11s %10s %10s %10s %10s %10s %10s %10s" % (
    "iter", "time(s)", "μ", "P-obj", "D-obj", "gap", "P-error", "p-error", "d-error", "α_p",
    "α_d", "beta")


@dataclass
class RunInfo:
    iterations: int
    log: list
    phase_ms: np.ndarray
    time_total: float
    time_loop_after2: float
    status: str
    exact: list = None   # per iteration, the device scalar slots at full precision (record_exact)
    factorization: int = 1  # clrsdp_get_factorization at the end (an LU fallback adds its flag)
    lu_switch: int = 0      # iteration whose loop body switched to LU (0: none)
    inner_ms: np.ndarray = None  # the reference's inner buckets summed from iteration 3 (ms)


def _stage_groups(ph):
    """The reference's timing groups (MPMP.jl:888-898) from the device stages (seconds)."""
    S = {n: ph[i] for i, n in enumerate(_lib.STAGE_NAMES)}
    return {"Decomp": S["schur"] + S["factor"], "predict_dir": S["predictor"],
            "correct_dir": S["corrector"], "alpha": S["step"], "Xinv": S["Xinv"],
            "R": S["mu_R"] + S["corrector_R"], "res": S["residuals"], "update": S["update"]}


def _first_iteration_times(ph):
    g = _stage_groups(ph)
    return ("decomp:%s. directions:%s. steplength:%s\nschur:%s factor (chol S, CinvB, Q, chol Q):%s\n"
            "X inv:%s. R:%s. residuals p,P,d:%s" % (
                g["Decomp"], g["predict_dir"] + g["correct_dir"], g["alpha"], ph[2], ph[3],
                g["Xinv"], g["R"], g["res"]))


def _time_spent(total, ph, inner=None):
    """MPMP.jl:973-1012.  Per-stage device times (sums over iterations 3, 4, ...) need the
    handle's HIP-event timing (DeviceSolver(timing=True)); without it only the total is known."""
    cols = ["total", "Decomp", "predict_dir", "correct_dir", "alpha", "Xinv", "R", "res"]
    lines = ["\nTime spent: (The total time may include compile time. The first few iterations "
             "are not included in the rest of the times)",
             ("%11s " * len(cols)).rstrip() % tuple(cols)]
    if ph is None:
        lines.append("%11.5e %s" % (total, "(per-stage times need DeviceSolver(timing=True))"))
        return "\n".join(lines) + "\n"
    g = _stage_groups(ph)
    lines.append(("%11.5e " * len(cols)).rstrip() % tuple([total] + [g[c] for c in cols[1:]]))
    if inner is None:
        lines.append("\nTime inside decomp:\n%11s %11s\n%11.5e %11.5e" % (
            "schur", "factor", ph[2], ph[3]))
        return "\n".join(lines) + "\n"
    # MPMP.jl:997-1012: the inner buckets (clrsdp_iter_stats.inner_ms, device time of each
    # bucket's launches; the direction buckets summed over predictor and corrector)
    lines.append("\nTime inside decomp:")
    lines.append(("%11s " * 5).rstrip() % ("schur", "chol_S", "comp CinvB", "comp Q", "chol_Q"))
    lines.append(("%11.5e " * 5).rstrip() % tuple(inner[:5]))
    lines.append("\nTime inside search directions (both predictor & corrector step)")
    lines.append(("%11s " * 5).rstrip() % ("calc Z", "calc rhs x", "solve system", "calc dX",
                                          "calc dY"))
    lines.append(("%11.5e " * 5).rstrip() % tuple(inner[5:10]))
    return "\n".join(lines) + "\n"


def solverank1sdp(constraints, b, blockinfo: BlockInfo, C=None, b0=0, maxiterations=500,
                  beta_infeasible=None, beta_feasible=None, gamma=None, omega_p=None,
                  omega_d=None, duality_gap_threshold=None, primal_error_threshold=None,
                  dual_error_threshold=None, need_primal_feasible=False, need_dual_feasible=False,
                  testing=True, initial_solutions=(), precision_words=1, device=0, verbose=True,
                  solver: Optional[DeviceSolver] = None, return_info=False, record_exact=False,
                  pipelined: Optional[bool] = None, factorization: Optional[int] = None):
    """Solve the clustered low-rank SDP on the GPU; same signature/semantics as MPMP.jl:595-614.

    Returns ``(x, X, y, Y, P, p, d, duality_gap, primal_objective, dual_objective, time)``
    (MPMP.jl:1014-1024); with ``return_info`` a :class:`RunInfo` is appended.

    ``pipelined`` (default: on when the clusters are sharded over ranks): the host stays one loop body behind
    the device (clrsdp_iterate_async / _wait) and pd_feas / terminate() are evaluated on the
    device with the same thresholds, so no host round trip separates two loop bodies.  The
    iterates, the log and the returned values are the same as the synchronous loop's.

    ``factorization``: clrsdp_set_factorization flags (default FACT_FALLBACK: Cholesky, and the
    reference's pivoted LU once a Cholesky fails, announced like MPMP.jl:776-778).  At
    double-double and quad-double the returned gap and objectives are mpmath numbers at the
    state's full precision (MPMP.jl:1021-1023), not leading limbs; at fp64 they are floats.  The
    log rows (RunInfo.log) are floats except the gap column, which is an mpmath number at dd/qd
    like the returned gap (:func:`log_row`).
    """
    kw = dict(beta_infeasible=beta_infeasible, beta_feasible=beta_feasible, gamma=gamma,
              omega_p=omega_p, omega_d=omega_d, duality_gap_threshold=duality_gap_threshold,
              primal_error_threshold=primal_error_threshold,
              dual_error_threshold=dual_error_threshold)
    prm_v = {k: (DEFAULTS[k] if v is None else v) for k, v in kw.items()}
    out = print if verbose else (lambda *a, **k: None)
    bi = blockinfo
    dev = solver or DeviceSolver(constraints, b, bi, precision_words=precision_words, C_blocks=C,
                                 device=device)
    prm = make_params(prm_v["beta_infeasible"], prm_v["beta_feasible"], prm_v["gamma"], b0)
    # loop control at the state's full width (MPMP.jl:942-945, 1067-1078, 1147-1185 run at the
    # working precision): at dd/qd the thresholds are the device's exact multi-word values and
    # the gap, errors and pd_feas are the device's own control_update results (all limbs), so a
    # threshold below fp64 resolution is decided at the word's precision, and the synchronous
    # and pipelined loops decide alike
    exact_ctl = dev.w > 1
    gthr = device_threshold(prm_v["duality_gap_threshold"], dev.w)
    pthr = device_threshold(prm_v["primal_error_threshold"], dev.w)
    dthr = device_threshold(prm_v["dual_error_threshold"], dev.w)
    if initial_solutions is not None and len(initial_solutions) == 4:
        x, X, y, Y = initial_solutions
    else:
        x, X, y, Y = initial_point(bi, float(prm_v["omega_p"]), float(prm_v["omega_d"]))
    dev.set_state(x, X, y, Y)
    if factorization is not None:
        dev.set_factorization(factorization)
    fact_seen = dev.factorization
    b0f = float(b0)
    if pipelined is None:
        # one GPU: the hipGraph replay leaves only a short host round trip between bodies and
        # the synchronous loop measured faster; sharded: enqueueing (exchange callbacks, no
        # graph) is host-heavy, so the host runs one body ahead
        pipelined = dev.world > 1 and not record_exact
    dev.set_control(make_control(prm_v["duality_gap_threshold"], prm_v["primal_error_threshold"],
                                 prm_v["dual_error_threshold"], need_primal_feasible,
                                 need_dual_feasible))
    out(HEADER)
    st = dev.initial_residuals(prm)
    p_obj, d_obj = st.p_obj, st.d_obj
    # compute_duality_gap(constraints, x, y, Y, C, b) excludes b0 (MPMP.jl:725, 1067-1074)
    dual_gap = abs((p_obj - b0f) - (d_obj - b0f)) / max(1.0, abs((p_obj - b0f) + (d_obj - b0f)))
    perr = max(st.p_err, st.P_err)
    derr = st.d_err

    def device_control(st):
        """(gap, primal error, dual error) of the device's control_update for the state after
        the body `st` reports, all limbs (exact mpmath sums)."""
        import mpmath

        def v(limbs_):
            r = mpmath.mpf(0)
            for x in list(limbs_)[:dev.w]:
                r = mpmath.fadd(r, x, exact=True)
            return r
        return v(st.gap_w), max(v(st.P_err_w), v(st.p_err_w)), v(st.d_err_w)

    if exact_ctl:
        dual_gap, perr, derr = device_control(st)
    pd_feas = perr < pthr and derr < dthr
    it = 1
    log = []
    phase = np.zeros(_lib.NUM_STAGES)
    inner = np.zeros(_lib.NUM_INNER)
    t_start = time.time()
    t_after2 = None
    status = "maxiterations"
    exact = []
    lu_switch = [0]

    timed = bool(getattr(dev, "timing", False))

    def record(st):
        nonlocal p_obj, d_obj, dual_gap, perr, derr, pd_feas, it, fact_seen
        f = dev.factorization
        if f != fact_seen:   # the device switched to LU for the rest of the solve
            if (f & ~fact_seen) & _lib.FACT_LU_X:
                out("The inverse of X could not be computed with the cholesky factorization. We "
                    "switch to using the LU decomposition.")
            if (f & ~fact_seen) & _lib.FACT_LU_SQ:
                out("The Cholesky factorization of S or Q failed. We switch to the pivoted LU "
                    "decomposition (approx_lu!) for S and Q.")
            fact_seen = f
            lu_switch[0] = lu_switch[0] or it
        if it > 2:
            phase[:] += np.array(st.phase_ms[:])
            inner[:] += np.array(st.inner_ms[:])
        elif testing and timed:  # MPMP.jl:899-920: the times of the first iterations
            out(_first_iteration_times(np.array(st.phase_ms[:]) / 1e3))
        row = log_row(it, time.time() - t_start, st, p_obj, d_obj, dual_gap)
        log.append(row)
        out("%5d %8.1f %11.3e %11.3e %11.3e %10.2e %10.2e %10.2e %10.2e %10.2e %10.2e %10.2e" % row)
        p_obj, d_obj = st.p_obj, st.d_obj
        if exact_ctl:   # the device's full-width values (dd/qd)
            dual_gap, perr, derr = device_control(st)
        else:
            dual_gap = abs(p_obj - d_obj) / max(1.0, abs(p_obj + d_obj))      # MPMP.jl:942
            perr = max(st.p_err, st.P_err)                                     # MPMP.jl:943
            derr = st.d_err
        it += 1
        pd_feas = perr < pthr and derr < dthr                                  # MPMP.jl:949-953

    def term():
        return _terminate(dual_gap, perr, derr, gthr, pthr, dthr, need_primal_feasible,
                          need_dual_feasible, out)

    if pipelined:
        # the host one loop body behind: body it+1 is enqueued before the log row of body it is
        # read; the device decides pd_feas and terminate() itself (same thresholds) and a body
        # enqueued after termination applies nothing (ran = False)
        inflight = 0
        halted = False
        if term():
            status = "terminated"
        elif it < maxiterations:
            dev.iterate_async(prm)
            inflight = 1
        try:
            while inflight:
                if it + 1 < maxiterations:
                    dev.iterate_async(prm)
                    inflight += 1
                if it == 3:
                    t_after2 = time.time()
                st, ran = dev.iterate_wait()
                inflight -= 1
                if not ran:
                    halted = True
                    break
                record(st)
        finally:
            while inflight:   # drain skipped bodies (or the one behind a failure)
                try:
                    dev.iterate_wait()
                except Exception:
                    pass
                inflight -= 1
        if it > 1 or halted:
            # the reference evaluates terminate() (which prints the reason) before iter < maxit
            if term() or halted:
                status = "terminated"
    while not pipelined:
        if term():
            status = "terminated"
            break
        if not it < maxiterations:
            break
        if it == 3:
            t_after2 = time.time()
        st = dev.iterate(prm, pd_feas)
        if record_exact:
            sc = dev.buffer(_lib.BUF_SCALARS, exact=True)
            exact.append({k: sc[v] for k, v in _lib.SC.items()})
        record(st)
    t_total = time.time() - t_start
    out(HEADER)
    out(_time_spent(t_total, phase / 1e3 if timed else None, inner / 1e3 if timed else None))
    xf, Xf, yf, Yf = dev.get_state()
    P, d = dev.global_P_d()
    p = dev.buffer(_lib.BUF_PVEC)
    gap_nob0 = abs((p_obj - b0f) - (d_obj - b0f)) / max(1.0, abs((p_obj - b0f) + (d_obj - b0f)))
    ret_p, ret_d = p_obj, d_obj
    if dev.w > 1:
        # MPMP.jl:1021-1023 at the state's precision: the device's objectives of the final state
        # (all limbs) and the gap without b0 from them
        import mpmath
        with mpmath.workprec(64 * dev.w + 64):
            sc = dev.buffer(_lib.BUF_SCALARS, exact=True)
            ret_p, ret_d = +sc[_lib.SC["p_obj"]], +sc[_lib.SC["d_obj"]]
            b0m = mpmath.mpf(b0)
            pp, dd_ = ret_p - b0m, ret_d - b0m
            gap_nob0 = abs(pp - dd_) / max(mpmath.mpf(1), abs(pp + dd_))
    res = (xf, Xf, yf, Yf, P, p, d, gap_nob0, ret_p, ret_d, t_total)
    if return_info:
        res = res + (RunInfo(it - 1, log, phase, t_total,
                             (time.time() - t_after2) if t_after2 else 0.0, status, exact,
                             dev.factorization, lu_switch[0], inner),)
    if solver is None:
        dev.close()
    return res
