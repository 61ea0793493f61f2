/*
 * clrsdp.h -- C ABI of the MI355X-native interior-point step for clustered low-rank SDPs.
 *
 * This is the drop-in boundary for the hot path of nanleij/Clustered-Low-Rank-SDP-solver
 * (MPMP.jl).  The reference has no FFI of its own: its seam is a set of Julia
 * calls inside the `solverank1sdp` loop (MPMP.jl:742-954).  Every entry point below names the
 * reference function(s) it replaces.  A host (the Python mirror in
 * clustered-low-rank-sdp-solver_amd/solver.py, or the Julia `ccall` shim in INTEGRATION.md)
 * keeps `solvempmp` / `prepareabc` / `solverank1sdp` and calls these.
 *
 * Conventions
 *   - plain C types; sizes are int64_t; matrices are column-major.
 *   - multi-word numbers (precision_words w = 2 double-double, 4 quad-double) are passed as
 *     PLANAR limbs: an array of n values is w consecutive planes of n doubles, plane 0 = the
 *     leading (hi) limb.  w = 1 is plain IEEE binary64.
 *   - every call returns an int status (CLRSDP_OK = 0); no exception crosses the ABI; the
 *     message of the last failure is returned by clrsdp_last_error().
 *   - host pointers are borrowed for the duration of a call only; the handle owns all device
 *     memory (constraint data stays resident across iterations).
 *   - calls are synchronous w.r.t. the host, not re-entrant per handle, safe across handles.
 */
#ifndef CLRSDP_H
#define CLRSDP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (the reference's failure outcomes) ---------------------- */
#define CLRSDP_OK 0
#define CLRSDP_E_ARG 1        /* invalid argument / shape                                     */
#define CLRSDP_E_HIP 2        /* HIP runtime failure (no device, out of memory, ...)         */
#define CLRSDP_E_NOT_PD_X 3   /* spd_inv! failed on a block of X      (MPMP.jl:774-797)       */
#define CLRSDP_E_NOT_PD_S 4   /* "S was not decomposed succesfully"   (MPMP.jl:1439)          */
#define CLRSDP_E_NOT_PD_Q 5   /* "Q was not decomposed correctly"     (MPMP.jl:1503)          */
#define CLRSDP_E_STEP 6       /* step length failed: cho!(X or Y)     (MPMP.jl:1846-1882)      */
#define CLRSDP_E_EXCHANGE 7   /* the multi-rank exchange callback failed                     */
#define CLRSDP_E_STATE 8      /* call out of order (e.g. iterate before upload)              */

/* ---- stages of one iteration (MPMP.jl:755-887); clrsdp_iterate runs them in this order ---- */
#define CLRSDP_STAGE_MU_R 0        /* mu = <X,Y>/dim, mu_p, R = mu_p I - XY   (755-761, 1189)   */
#define CLRSDP_STAGE_XINV 1        /* X^-1 per block (spd_inv!)               (762-801)         */
#define CLRSDP_STAGE_SCHUR 2       /* S_j and A_Y        (compute_S_integrated, 1218-1414)      */
#define CLRSDP_STAGE_FACTOR 3      /* chol(S_j), L^-1 B_j, Q, chol(Q)         (1429-1505)       */
#define CLRSDP_STAGE_RESIDUALS 4   /* P, p, d            (compute_residuals, 1107-1144)         */
#define CLRSDP_STAGE_PREDICTOR 5   /* dx, dX, dy, dY     (compute_search_direction, 818)        */
#define CLRSDP_STAGE_CORRECTOR_R 6 /* r, beta_c, mu_c, R = mu_c I - XY - dXdY (832-842, 1203)   */
#define CLRSDP_STAGE_CORRECTOR 7   /* corrector direction                     (846-857)         */
#define CLRSDP_STAGE_STEP 8        /* alpha_p, alpha_d   (compute_step_length, 863-874)         */
#define CLRSDP_STAGE_UPDATE 9      /* x,y,X,Y += alpha d*, new objectives     (877-887, 940-941) */
#define CLRSDP_NUM_STAGES 10

/* Inner buckets of the reference's timing table (MPMP.jl:897-898: "Time inside decomp" and
 * "Time inside search directions", printed at 997-1012) */
#define CLRSDP_INNER_SCHUR 0       /* compute_S_integrated                                       */
#define CLRSDP_INNER_CHOL_S 1      /* factorisation of S_j (Cholesky + L^-1, or approx_lu!)      */
#define CLRSDP_INNER_CINVB 2       /* L_j^-1 B_j (and B_j^T U_j^-1)                               */
#define CLRSDP_INNER_Q 3           /* Q = sum_j W_j^T W_j (+ the exchange)                        */
#define CLRSDP_INNER_CHOL_Q 4      /* factorisation of Q                                          */
#define CLRSDP_INNER_Z 5           /* Z = sym(X^-1 (P Y - R)) and its trace_A products            */
#define CLRSDP_INNER_RHS_X 6       /* rhs_x = -d - Tr(A_* Z)                                      */
#define CLRSDP_INNER_SOLVE 7       /* the block solve for dx, dy                                  */
#define CLRSDP_INNER_DX 8          /* dX = P + sum dx_i A_i                                        */
#define CLRSDP_INNER_DY 9          /* dY = sym(X^-1 (R - dX Y))                                    */
#define CLRSDP_NUM_INNER 10

/* ---- device buffers readable with clrsdp_get_buffer (stage-level parity tests) ----------- */
#define CLRSDP_BUF_X 0        /* block-diagonal state X, blocks concatenated, column-major   */
#define CLRSDP_BUF_Y 1
#define CLRSDP_BUF_XINV 2     /* X^-1 after STAGE_XINV                                       */
#define CLRSDP_BUF_R 3        /* R after STAGE_MU_R / STAGE_CORRECTOR_R                      */
#define CLRSDP_BUF_S 4        /* S_j (full symmetric) after STAGE_SCHUR, clusters concatenated */
#define CLRSDP_BUF_AY 5       /* A_Y: per block, per (r,s) with r>=s, K values               */
#define CLRSDP_BUF_Q 6        /* Q = sum_j B_j^T S_j^-1 B_j before its factorisation           */
#define CLRSDP_BUF_P 7        /* primal residual P (blocks)                                  */
#define CLRSDP_BUF_PVEC 8     /* p (n_y)                                                      */
#define CLRSDP_BUF_DVEC 9     /* d (local sum dim_S)                                           */
#define CLRSDP_BUF_DX 10      /* dx (local)                                                   */
#define CLRSDP_BUF_DXMAT 11   /* dX (blocks)                                                  */
#define CLRSDP_BUF_DY 12      /* dy (n_y)                                                     */
#define CLRSDP_BUF_DYMAT 13   /* dY (blocks)                                                  */
#define CLRSDP_BUF_XVEC 14    /* x (local)                                                    */
#define CLRSDP_BUF_YVEC 15    /* y (n_y)                                                      */
#define CLRSDP_BUF_SCALARS 16 /* clrsdp_scalar slots (see CLRSDP_SC_*)                          */
#define CLRSDP_NUM_BUFS 17

/* slots of CLRSDP_BUF_SCALARS */
#define CLRSDP_SC_MU 0
#define CLRSDP_SC_MU_P 1
#define CLRSDP_SC_R 2
#define CLRSDP_SC_BETA 3
#define CLRSDP_SC_BETA_C 4
#define CLRSDP_SC_MU_C 5
#define CLRSDP_SC_ALPHA_P 6
#define CLRSDP_SC_ALPHA_D 7
#define CLRSDP_SC_MINEIG_X 8
#define CLRSDP_SC_MINEIG_Y 9
#define CLRSDP_SC_POBJ 10
#define CLRSDP_SC_DOBJ 11
#define CLRSDP_SC_ERR_P_MAT 12
#define CLRSDP_SC_ERR_P_VEC 13
#define CLRSDP_SC_ERR_D_VEC 14
#define CLRSDP_SC_DOT_XY 15
#define CLRSDP_SC_DOT_XDY 16
#define CLRSDP_NUM_SCALARS 24

/* Problem description: the fields of BlockInfo (MPMP.jl:467-513) the device needs.
 * Global over ALL clusters (every rank passes the same description). */
typedef struct {
  int64_t J;                 /* number of clusters                                          */
  int64_t n_y;               /* number of free variables y                                  */
  const int64_t* m;          /* [J]  polynomial-matrix size m_j                              */
  const int64_t* L;          /* [J]  blocks per cluster                                      */
  const int64_t* n_samples;  /* [J]  N_j                                                     */
  const int64_t* delta;      /* [sum_j L_j] vector length of block (j,l), (j,l) order         */
  const int64_t* ranks;      /* [sum_{j,l} N_j] rank of (j,l,k), (j,l,k) order               */
} clrsdp_desc;

typedef struct {
  int32_t precision_words;   /* 1 = fp64, 2 = double-double, 4 = quad-double                 */
  int32_t device;            /* HIP device ordinal                                            */
  int32_t rank;              /* this process's rank, 0 <= rank < world_size                   */
  int32_t world_size;        /* number of processes (one per GPU)                             */
  const int32_t* owned;      /* clusters owned by this rank (ascending); NULL = all clusters  */
  int32_t n_owned;
  int32_t timing;            /* nonzero: record per-phase HIP events into clrsdp_iter_stats   */
} clrsdp_config;

/* solverank1sdp keyword arguments used inside the loop body (MPMP.jl:599-613); each value is
 * given as up to 4 limbs (unused limbs 0). */
typedef struct {
  double beta_infeasible[4];
  double beta_feasible[4];
  double gamma[4];
  double b0[4];
} clrsdp_params;

/* Loop-control thresholds of terminate() and check_pd_feasibility() (MPMP.jl:606-611,
 * 1147-1185), up to 4 limbs each; used by the pipelined loop (clrsdp_iterate_async). */
typedef struct {
  double duality_gap_threshold[4];
  double primal_error_threshold[4];
  double dual_error_threshold[4];
  int32_t need_primal_feasible;
  int32_t need_dual_feasible;
} clrsdp_control;

/* What one loop body produces for the host's log row and termination test (MPMP.jl:923-953).
 * All values are the leading limb. */
typedef struct {
  double mu;        /* mu at the start of the iteration                           (755)      */
  double P_err;     /* max |P_ij| of the residual computed this iteration         (931)      */
  double p_err;     /* max |p_i|                                                  (932)      */
  double d_err;     /* max |d_i|                                                  (933)      */
  double alpha_p;   /* primal step                                                (934)      */
  double alpha_d;   /* dual step                                                  (935)      */
  double beta_c;    /* corrector beta                                             (936)      */
  double p_obj;     /* <c,x> + b0 after the update                                (940)      */
  double d_obj;     /* <C,Y> + <b,y> + b0 after the update                        (941)      */
  double phase_ms[CLRSDP_NUM_STAGES]; /* per-stage device time when config.timing != 0       */
  int32_t status;
  /* timing mode 1 only: the reference's inner timings (MPMP.jl:897-898, 997-1012), device time
   * of the launches of each bucket (side-stream work included, measured on its own stream):
   * CLRSDP_INNER_* below; the direction buckets are predictor + corrector */
  double inner_ms[CLRSDP_NUM_INNER];
  /* the loop control of the state after this body at the word's full width (up to 4 limbs, hi
   * first; unused limbs 0): the duality gap (MPMP.jl:942; for clrsdp_initial_residuals the gap
   * without b0, 725) and the errors of the residuals computed in this body (943-944), as the
   * device's terminate()/check_pd_feasibility() compares them (1147-1185) */
  double gap_w[4];
  double P_err_w[4];
  double p_err_w[4];
  double d_err_w[4];
} clrsdp_iter_stats;

/* Multi-rank exchange: gather `bytes` bytes from `send_dev` on every rank into `recv_dev`
 * (rank r's bytes at offset r*bytes).  send_dev/recv_dev are the device buffers registered
 * with clrsdp_set_exchange.  Called on the host, in the middle of a stage, with the library's
 * work on `stream` enqueued but not necessarily finished; the callee must order its transfer
 * after that work and before anything enqueued later on `stream`.  Return 0 on success. */
typedef int (*clrsdp_exchange_fn)(void* ctx, int32_t tag, int64_t bytes, void* stream);

typedef struct clrsdp_handle clrsdp_handle;

int32_t clrsdp_version(void);
const char* clrsdp_last_error(const clrsdp_handle* h);  /* h may be NULL: last global error */

/* Allocate device state for the clusters owned by this rank.
 * Replaces: the allocations of solverank1sdp (MPMP.jl:660-721) and BlockInfo (MPMP.jl:480). */
int32_t clrsdp_create(const clrsdp_desc* desc, const clrsdp_config* cfg, clrsdp_handle** out);

/* Copy the constraint data (the (A, B, c, H) tuples of prepareabc, MPMP.jl:385-406).
 *  V:      per (j,l) the delta_jl x K_jl matrix of all vectors v_{j,l,k,rnk} (columns in (k,rnk)
 *          order, MPMP.jl:1249-1254), all (j,l) concatenated: sum delta_jl*K_jl values.
 *  lambda: per (j,l) the K_jl eigenvalues H[l,k][rnk], concatenated.
 *  B:      per j the dim_S_j x n_y matrix, concatenated.   c: per j dim_S_j values.
 *  b:      n_y values.   C: NULL (C = 0, MPMP.jl:691-695) or the blocks of C concatenated.
 * Each array is w planes (see conventions); data of clusters not owned is skipped. */
int32_t clrsdp_upload_constraints(clrsdp_handle* h, const double* V, const double* lambda,
                                  const double* B, const double* c, const double* b,
                                  const double* C);

/* State (x, X, y, Y) in the global layout: x has sum_j dim_S_j entries, X and Y all blocks
 * concatenated (column-major), y has n_y.  set: the owned parts are read.  get: the owned
 * parts of x/X/Y are written (others untouched); y is replicated.
 * Replaces: initial_solutions / the returned state (MPMP.jl:613, 660-690, 1014-1024). */
int32_t clrsdp_set_state(clrsdp_handle* h, const double* x, const double* X, const double* y,
                         const double* Y);
int32_t clrsdp_get_state(clrsdp_handle* h, double* x, double* X, double* y, double* Y);

/* Residuals, errors and objectives at the current state, before the loop (MPMP.jl:723-736):
 * fills P_err, p_err, d_err, p_obj, d_obj (with b0) of `st`. */
int32_t clrsdp_initial_residuals(clrsdp_handle* h, const clrsdp_params* prm,
                                 clrsdp_iter_stats* st);

/* One full loop body (MPMP.jl:755-887 + the objective update 940-941).  pd_feas is the host's
 * check_pd_feasibility result from the previous iteration (MPMP.jl:949-953). */
int32_t clrsdp_iterate(clrsdp_handle* h, const clrsdp_params* prm, int32_t pd_feas,
                       clrsdp_iter_stats* st);

/* Pipelined loop (replaces the same loop, MPMP.jl:743-954, with the host one body behind):
 * clrsdp_set_control sets the thresholds; clrsdp_iterate_async enqueues one loop body whose
 * pd_feas and termination are decided on the device from the previous body's results
 * (after clrsdp_initial_residuals for the first) and returns at once; clrsdp_iterate_wait
 * waits for the oldest body in flight and returns its log row.  At most two bodies are in
 * flight.  A body enqueued after the device decided to terminate applies nothing and returns
 * *ran = 0; P, p, d (clrsdp_get_buffer) are then those of the last body that ran. */
int32_t clrsdp_set_control(clrsdp_handle* h, const clrsdp_control* ctl);
int32_t clrsdp_iterate_async(clrsdp_handle* h, const clrsdp_params* prm);
int32_t clrsdp_iterate_wait(clrsdp_handle* h, clrsdp_iter_stats* st, int32_t* ran);

/* Run one stage (CLRSDP_STAGE_*) only; stages must be run in order within an iteration. */
int32_t clrsdp_run_stage(clrsdp_handle* h, int32_t stage, const clrsdp_params* prm,
                         int32_t pd_feas);

/* Read a device buffer (CLRSDP_BUF_*) as w planes of doubles.  *count receives the number of
 * values per plane; host may be NULL to query the size. */
int32_t clrsdp_get_buffer(clrsdp_handle* h, int32_t buf, double* host, int64_t* count);

/* Register the multi-rank exchange (required when world_size > 1).  send_dev / recv_dev are
 * device buffers of at least clrsdp_exchange_bytes() and world_size times that. */
int32_t clrsdp_exchange_bytes(const clrsdp_handle* h, int64_t* bytes);
int32_t clrsdp_set_exchange(clrsdp_handle* h, clrsdp_exchange_fn fn, void* ctx, void* send_dev,
                            void* recv_dev);

/* Native RCCL exchange (the per-cluster partials all-gathered over xGMI, SURVEY.md §8e;
 * replaces the reference's shared-memory reductions across cluster threads, e.g. the Q sum
 * MPMP.jl:1486-1494 and the dy partials 1758-1761).  Rank 0 calls clrsdp_comm_unique_id and
 * hands the CLRSDP_COMM_ID_BYTES bytes to every rank (any host channel); every rank then calls
 * clrsdp_comm_init with them.  The handle creates an RCCL communicator of world_size ranks on
 * its device (RCCL is loaded at run time) and from then on issues every exchange itself as an
 * ncclAllGather on its stream; the exchange callback is no longer used.  With world_size > 1
 * the loop body is enqueued eagerly (the pipelined loop hides the enqueue), or replayed as one
 * hipGraph with the all-gathers captured in it when CLRSDP_GRAPH_RCCL is set.  With
 * world_size 1 the all-gathers are still issued (in place, one rank) inside the graph, which
 * exercises the capture path. */
#define CLRSDP_COMM_ID_BYTES 128
int32_t clrsdp_comm_unique_id(uint8_t* id);
int32_t clrsdp_comm_init(clrsdp_handle* h, const uint8_t* id);

/* Device-side snapshot of the iterate: clrsdp_save_state copies x, X, y, Y and the scalar
 * slots into a buffer of the handle, clrsdp_restore_state copies them back; both are enqueued
 * on the handle's stream (no host synchronisation), so a benchmark can replay a window of loop
 * bodies indefinitely without converging into the fp64 breakdown regime.  (No reference
 * counterpart; initial_solutions, MPMP.jl:613, restarts from the host.) */
int32_t clrsdp_save_state(clrsdp_handle* h);
int32_t clrsdp_restore_state(clrsdp_handle* h);

/* Run all work on `stream` (a hipStream_t; NULL = the handle's own stream). */
int32_t clrsdp_set_stream(clrsdp_handle* h, void* stream);
void* clrsdp_get_stream(const clrsdp_handle* h);
int32_t clrsdp_synchronize(clrsdp_handle* h);

/* Per-stage HIP-event timing (clrsdp_iter_stats.phase_ms): 0 = off, 1 = every stage (the loop
 * body is enqueued stage by stage, no graph), 2 = only phase_ms[CLRSDP_STAGE_SCHUR]: the sum of
 * the three Schur launches' first-workgroup-start..last-workgroup-end on the 100 MHz device clock,
 * stamped by the kernels inside the replayed loop-body graph (fp64 fast path; 0 elsewhere).
 * With timing 0 or 2 and world_size 1 (or a
 * native RCCL communicator), clrsdp_iterate replays a captured hipGraph of the loop body. */
int32_t clrsdp_set_timing(clrsdp_handle* h, int32_t on);

/* Loop-body hipGraph replay on (default) or off (on = 0: every body is enqueued eagerly from the
 * host, launch by launch, as the sharded path without CLRSDP_GRAPH_RCCL does; a measurement
 * switch, e.g. for the host enqueue time of one body).  No reference counterpart. */
int32_t clrsdp_set_graph(clrsdp_handle* h, int32_t on);

/* The exchange this handle's loop body uses: *backend 0 = none (one rank),
 * 1 = the native RCCL communicator of clrsdp_comm_init (*nranks = ncclCommCount of it),
 * 2 = the clrsdp_set_exchange callback (*nranks = world_size).  Replaces nothing in the
 * reference (shared-memory threads, MPMP.jl:1486-1494, 1758-1761). */
int32_t clrsdp_comm_info(const clrsdp_handle* h, int32_t* nranks, int32_t* backend);

/* Factorisations of S_j, Q and X (flags, default CLRSDP_FACT_FALLBACK).  The device factorises
 * S_j and Q by Cholesky (they are SPD) and X^-1 by the Cholesky inverse (spd_inv!).  The
 * reference factorises S_j and Q by partially pivoted LU (approx_lu!, MPMP.jl:1433-1442,
 * 1499-1505) and switches X^-1 to LU when spd_inv! fails (approx_inv!, MPMP.jl:774-786):
 *   CLRSDP_FACT_FALLBACK  when a Cholesky fails, set the matching LU flag and re-run the loop
 *                         body (its update was not applied); LU then stays on for the solve
 *   CLRSDP_FACT_LU_SQ     S_j and Q by pivoted LU now (the reference's own factorisation)
 *   CLRSDP_FACT_LU_X      X^-1 by pivoted LU now (approx_inv!)
 * clrsdp_get_factorization reports the current flags (a fallback adds its LU flag).
 * A failed LU is the reference's error (CLRSDP_E_NOT_PD_S / _Q / _X). */
#define CLRSDP_FACT_FALLBACK 1
#define CLRSDP_FACT_LU_SQ 2
#define CLRSDP_FACT_LU_X 4
int32_t clrsdp_set_factorization(clrsdp_handle* h, int32_t flags);
int32_t clrsdp_get_factorization(const clrsdp_handle* h, int32_t* flags);
int32_t clrsdp_destroy(clrsdp_handle* h);

/* Stand-alone step length of a block-diagonal pair, fp64 (replaces compute_step_length,
 * MPMP.jl:1829-1898, without a handle): M_b = L_b L_b^T and lambda_b = lambda_min(L_b^-1 dM_b
 * L_b^-T) per block, then *alpha = 1 if min_b lambda_b > -gamma, else -gamma / min_b lambda_b
 * (1893-1897).  The nblocks blocks of sizes n[] are concatenated column-major in M and dM (host
 * memory); min_eig (may be NULL) receives the nblocks lambda_b.  CLRSDP_E_STEP when some M_b is
 * not positive definite (cho! fails, 1846-1848 / 1882). */
int32_t clrsdp_step_length(int32_t device, int64_t nblocks, const int64_t* n, const double* M,
                           const double* dM, double gamma, double* alpha, double* min_eig);

/* lambda_min of each symmetric block at fp64 (words 1), double-double (2) or quad-double (4):
 * the eigenvalue part of compute_step_length (MPMP.jl:1857-1870, approx_eig_qr! of L^-1 dM L^-T),
 * Householder tridiagonalisation + Sturm multisection (+ the multi-word Newton tail) as the
 * loop body runs it.  A: the nblocks blocks of sizes n[] concatenated column-major, as `words`
 * planes of doubles (hi limb first; the blocks must be exactly symmetric); min_eig: `words` planes of nblocks values. */
int32_t clrsdp_eigmin(int32_t device, int32_t words, int64_t nblocks, const int64_t* n,
                      const double* A, double* min_eig);

#ifdef __cplusplus
}
#endif
#endif /* CLRSDP_H */
