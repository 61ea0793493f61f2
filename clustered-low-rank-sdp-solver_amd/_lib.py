"""ctypes binding of libclrsdp.so (include/clrsdp.h).

The library is built in-tree by ``__graft_entry__.build()``.  There is no fallback: if the
shared library is missing, :func:`lib` raises -- the solver never silently runs anywhere else.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libclrsdp.so")

OK = 0
E_ARG, E_HIP, E_NOT_PD_X, E_NOT_PD_S, E_NOT_PD_Q, E_STEP, E_EXCHANGE, E_STATE = range(1, 9)

STAGE_MU_R, STAGE_XINV, STAGE_SCHUR, STAGE_FACTOR, STAGE_RESIDUALS, STAGE_PREDICTOR, \
    STAGE_CORRECTOR_R, STAGE_CORRECTOR, STAGE_STEP, STAGE_UPDATE = range(10)
NUM_STAGES = 10
NUM_INNER = 10
# the reference's inner timing buckets (MPMP.jl:897-898, 997-1012), clrsdp_iter_stats.inner_ms
INNER_NAMES = ["schur", "chol_S", "comp CinvB", "comp Q", "chol_Q", "calc Z", "calc rhs x",
               "solve system", "calc dX", "calc dY"]
STAGE_NAMES = ["mu_R", "Xinv", "schur", "factor", "residuals", "predictor", "corrector_R",
               "corrector", "step", "update"]

(BUF_X, BUF_Y, BUF_XINV, BUF_R, BUF_S, BUF_AY, BUF_Q, BUF_P, BUF_PVEC, BUF_DVEC, BUF_DX,
 BUF_DXMAT, BUF_DY, BUF_DYMAT, BUF_XVEC, BUF_YVEC, BUF_SCALARS) = range(17)

SC = dict(mu=0, mu_p=1, r=2, beta=3, beta_c=4, mu_c=5, alpha_p=6, alpha_d=7, mineig_X=8,
          mineig_Y=9, p_obj=10, d_obj=11, err_P=12, err_p=13, err_d=14, dot_XY=15, dot_XdY=16,
          pd_feas=24, halt=25, gap=26)

EXPORTS = ["clrsdp_version", "clrsdp_last_error", "clrsdp_create", "clrsdp_upload_constraints",
           "clrsdp_set_state", "clrsdp_get_state", "clrsdp_initial_residuals", "clrsdp_iterate",
           "clrsdp_run_stage", "clrsdp_get_buffer", "clrsdp_exchange_bytes", "clrsdp_set_exchange",
           "clrsdp_set_stream", "clrsdp_get_stream", "clrsdp_synchronize", "clrsdp_set_timing",
           "clrsdp_destroy", "clrsdp_set_control", "clrsdp_iterate_async", "clrsdp_iterate_wait",
           "clrsdp_comm_unique_id", "clrsdp_comm_init", "clrsdp_save_state",
           "clrsdp_restore_state", "clrsdp_step_length", "clrsdp_set_factorization",
           "clrsdp_get_factorization", "clrsdp_set_graph", "clrsdp_comm_info", "clrsdp_eigmin"]
# clrsdp_set_factorization flags (include/clrsdp.h)
FACT_FALLBACK, FACT_LU_SQ, FACT_LU_X = 1, 2, 4
COMM_ID_BYTES = 128

P_i64 = C.POINTER(C.c_int64)
P_i32 = C.POINTER(C.c_int32)
P_f64 = C.POINTER(C.c_double)


class Desc(C.Structure):
    _fields_ = [("J", C.c_int64), ("n_y", C.c_int64), ("m", P_i64), ("L", P_i64),
                ("n_samples", P_i64), ("delta", P_i64), ("ranks", P_i64)]


class Config(C.Structure):
    _fields_ = [("precision_words", C.c_int32), ("device", C.c_int32), ("rank", C.c_int32),
                ("world_size", C.c_int32), ("owned", P_i32), ("n_owned", C.c_int32),
                ("timing", C.c_int32)]


class Params(C.Structure):
    _fields_ = [("beta_infeasible", C.c_double * 4), ("beta_feasible", C.c_double * 4),
                ("gamma", C.c_double * 4), ("b0", C.c_double * 4)]


class Control(C.Structure):
    _fields_ = [("duality_gap_threshold", C.c_double * 4), ("primal_error_threshold", C.c_double * 4),
                ("dual_error_threshold", C.c_double * 4), ("need_primal_feasible", C.c_int32),
                ("need_dual_feasible", C.c_int32)]


class IterStats(C.Structure):
    _fields_ = [("mu", C.c_double), ("P_err", C.c_double), ("p_err", C.c_double),
                ("d_err", C.c_double), ("alpha_p", C.c_double), ("alpha_d", C.c_double),
                ("beta_c", C.c_double), ("p_obj", C.c_double), ("d_obj", C.c_double),
                ("phase_ms", C.c_double * NUM_STAGES), ("status", C.c_int32),
                ("inner_ms", C.c_double * NUM_INNER), ("gap_w", C.c_double * 4),
                ("P_err_w", C.c_double * 4), ("p_err_w", C.c_double * 4),
                ("d_err_w", C.c_double * 4)]


EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.c_int64, C.c_void_p)

_lib = None


def lib():
    """Load libclrsdp.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: the HIP library has not been built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'`).")
    L = C.CDLL(LIB_PATH)
    L.clrsdp_version.restype = C.c_int32
    L.clrsdp_last_error.restype = C.c_char_p
    L.clrsdp_last_error.argtypes = [C.c_void_p]
    L.clrsdp_create.argtypes = [C.POINTER(Desc), C.POINTER(Config), C.POINTER(C.c_void_p)]
    L.clrsdp_upload_constraints.argtypes = [C.c_void_p] + [P_f64] * 6
    L.clrsdp_set_state.argtypes = [C.c_void_p] + [P_f64] * 4
    L.clrsdp_get_state.argtypes = [C.c_void_p] + [P_f64] * 4
    L.clrsdp_initial_residuals.argtypes = [C.c_void_p, C.POINTER(Params), C.POINTER(IterStats)]
    L.clrsdp_iterate.argtypes = [C.c_void_p, C.POINTER(Params), C.c_int32, C.POINTER(IterStats)]
    L.clrsdp_run_stage.argtypes = [C.c_void_p, C.c_int32, C.POINTER(Params), C.c_int32]
    L.clrsdp_get_buffer.argtypes = [C.c_void_p, C.c_int32, P_f64, P_i64]
    L.clrsdp_exchange_bytes.argtypes = [C.c_void_p, P_i64]
    L.clrsdp_set_exchange.argtypes = [C.c_void_p, EXCHANGE_FN, C.c_void_p, C.c_void_p, C.c_void_p]
    L.clrsdp_set_stream.argtypes = [C.c_void_p, C.c_void_p]
    L.clrsdp_get_stream.restype = C.c_void_p
    L.clrsdp_get_stream.argtypes = [C.c_void_p]
    L.clrsdp_synchronize.argtypes = [C.c_void_p]
    L.clrsdp_set_timing.argtypes = [C.c_void_p, C.c_int32]
    L.clrsdp_destroy.argtypes = [C.c_void_p]
    L.clrsdp_set_control.argtypes = [C.c_void_p, C.POINTER(Control)]
    L.clrsdp_iterate_async.argtypes = [C.c_void_p, C.POINTER(Params)]
    L.clrsdp_iterate_wait.argtypes = [C.c_void_p, C.POINTER(IterStats), P_i32]
    L.clrsdp_comm_unique_id.argtypes = [C.c_char_p]
    L.clrsdp_comm_init.argtypes = [C.c_void_p, C.c_char_p]
    L.clrsdp_save_state.argtypes = [C.c_void_p]
    L.clrsdp_restore_state.argtypes = [C.c_void_p]
    L.clrsdp_set_factorization.argtypes = [C.c_void_p, C.c_int32]
    L.clrsdp_get_factorization.argtypes = [C.c_void_p, P_i32]
    L.clrsdp_set_graph.argtypes = [C.c_void_p, C.c_int32]
    L.clrsdp_comm_info.argtypes = [C.c_void_p, P_i32, P_i32]
    L.clrsdp_eigmin.argtypes = [C.c_int32, C.c_int32, C.c_int64, P_i64, P_f64, P_f64]
    L.clrsdp_step_length.argtypes = [C.c_int32, C.c_int64, P_i64, P_f64, P_f64, C.c_double, P_f64,
                                     P_f64]
    for name in EXPORTS:
        if name not in ("clrsdp_last_error", "clrsdp_get_stream"):
            getattr(L, name).restype = C.c_int32
    _lib = L
    return L


class ClrsdpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"clrsdp error {code}: {msg}")
        self.code = code


def check(rc, handle=None):
    if rc != OK:
        msg = lib().clrsdp_last_error(handle).decode(errors="replace")
        raise ClrsdpError(rc, msg)
