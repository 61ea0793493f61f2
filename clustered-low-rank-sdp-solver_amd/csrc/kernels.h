// kernels.h -- gfx950 kernels of one interior-point iteration, templated on the word type T.
//
// Every kernel is *batched over a descriptor array*: one launch covers all (j,l) blocks (or
// all clusters) of a phase, whatever their sizes -- the reference's `Threads.@threads for
// (j,l) in jl_pairs` loops become the grid.  Layout in HBM: every matrix
// column-major; block matrices of X, Y, ... concatenated in (j,l) order.
//
//   gemm_f64_mfma   C = alpha op(A) op(B) + beta Cin     fp64 matrix cores (v_mfma_f64_16x16x4)
//   gemm_valu       same for multi-word T                VALU
//   potrf_batched   in-place lower Cholesky              (spd_inv!/cho!/approx_lu! replacements)
//   trsm_batched    B <- L^-1 B  or  L^-T B              (approx_solve_tril!/triu!)
//   eigmin_batched  lambda_min of a symmetric block      (approx_eig_qr! replacement)
//   schur_assemble  S_j from the pairings BX, BY         (MPMP.jl:1335-1409)
//   + small elementwise / reduction kernels
#pragma once
#include <hip/hip_runtime.h>
#include "mwfloat.h"

namespace clrsdp {

using mw::Num;
using mw::sel;

typedef double d4 __attribute__((ext_vector_type(4)));

// workgroup -> (problem, tile).  The batched launches order their workgroups tile-major
// (problem fastest), so with a problem count divisible by 8 every tile of one problem lands on
// the same XCD (workgroups go round-robin over the 8 XCDs) and shares its L2.
struct TileRef {
  int p, t;
};

template <class T> struct GemmDesc {
  const T* A;
  const T* B;
  const T* Cin;
  T* C;
  int M, N, K, lda, ldb, ldcin, ldc;
  int tn;     // tiles along N
  int tile0;  // (unused by the TileRef kernels)
  int flags;  // gemm_f64_dyn: bit 0 op(A) = A^T, bit 1 op(B) = B^T, bit 2 alpha/beta below,
              // bit 3 raised wave priority
  double alpha, beta;  // gemm_f64_dyn with flags bit 2 (else the launch's)
  const T* sa;  // SCA launches: column k of op(A) is scaled by sa[k] * sl[k] (weighted A)
  const T* sl;
};

template <class T> struct MatDesc {
  T* A;
  int n, lda;
};

template <class T> struct TrsmDesc {
  const T* L;
  T* B;
  int n, nrhs, ldl, ldb;
  int tile0;  // first column-tile index of this problem in the launch
  int pad;    // trsv_wave / trsv_wave128: 1 = the right-hand sides are the identity's columns
  const T* src;  // trsv_wave / trsv_wave128: right-hand sides read from here (ld ldb), not B
};
// the right-hand side entry (row, column c) of a vector solve: the identity, src, or B in place
template <class T>
__device__ __forceinline__ T trsv_rhs(const TrsmDesc<T>& d, const T* B, int row, int c) {
  if (d.pad == 1) return T(row == c ? 1.0 : 0.0);
  return d.src ? d.src[row + (size_t)c * d.ldb] : B[row];
}

// Load through an explicitly global pointer.  A pointer read from a descriptor is generic, and
// hipcc then emits flat_load, which also counts on lgkmcnt: the first LDS wait of the MFMA loop
// then drains every prefetch load in flight (no overlap of the next slab with the MFMAs).
typedef const __attribute__((address_space(1))) double* gdptr;
__device__ inline double gload(const double* p) { return *(gdptr)p; }

namespace lds_gemm {
// Staging of one R x BK slab of an operand (NTH threads, R*BK/NTH elements per thread; R = 64,
// or 32 for the small-tile GEMM).  kcontig: element (i, k) at P[k + i*ld], kept in LDS as
// S[i*(BK+1) + k]; else at P[i + k*ld], kept as S[k*LM + i] (LM = R + 16: the four k-rows of a
// fragment read start 32 banks apart).  Rows i beyond `rows` are clamped (their products are
// never stored); k beyond K is zeroed.
// The k-contiguous pitch is odd (round 6; BK + 2 before): hipcc reads two k-steps of a fragment
// with one ds_read2_b64 (k, k + 4), whose 16-lane groups bank by dword mod 32, and an even pitch
// put rows i and i + 8 of a group on one bank (2-way: the 0.15 / 0.30 SQ_LDS_BANK_CONFLICT
// shares of gemm_f64_uni / gemm_f64_dyn in round 5)
constexpr int LSM = 80;
template <int BK, int NTH = 256, int R = 64> struct Slab {
  static constexpr int PER = R * BK / NTH, LSK = BK + 1, LM = R + 16;
  static_assert(PER * NTH == R * BK, "slab split");
  static constexpr int SZ = R * LSK > BK * LM ? R * LSK : BK * LM;  // doubles per image
  template <bool kcontig>
  __device__ static inline void kk(int tid, int q, int& i, int& k) {
    if (!kcontig) { i = tid % R; k = tid / R + (NTH / R) * q; }
    else { k = tid & (BK - 1); i = tid / BK + (NTH / BK) * q; }
  }
  // Unconditional loads from clamped addresses; the k >= K tail is zeroed in store(), after
  // the MFMAs (a select right after the load would make the compiler wait for it there, and a
  // load under a condition makes hipcc branch around every element).
  template <bool kcontig>
  __device__ static inline void load(double (&r)[PER], const double* __restrict__ P, int ld,
                                     int i0, int rows, int k0, int K, int tid) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      int i, k;
      kk<kcontig>(tid, q, i, k);
      const int gi = min(i0 + i, rows - 1), gkc = min(k0 + k, K - 1);
      r[q] = gload(P + (kcontig ? gkc + (size_t)gi * ld : gi + (size_t)gkc * ld));
    }
  }
  template <bool kcontig>
  __device__ static inline void store(const double (&r)[PER], double* __restrict__ S, int tid,
                                      int k0, int K) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      int i, k;
      kk<kcontig>(tid, q, i, k);
      const double v = k0 + k < K ? r[q] : 0.0;
      if (!kcontig) S[k * LM + i] = v;
      else S[i * LSK + k] = v;
    }
  }
  // MFMA fragment: element (i, k) of the staged image
  template <bool kcontig>
  __device__ static inline double frag(const double* __restrict__ S, int i, int k) {
    return kcontig ? S[i * LSK + k] : S[k * LM + i];
  }
};
// 64x64 output tile staged in LDS (pitch TP) so the global stores are coalesced: the MFMA
// accumulator layout puts 16 consecutive lanes on 16 different columns.
constexpr int TP = 65;
__device__ inline int acc_row(int wm, int mi, int lk, int r) { return wm * 32 + mi * 16 + lk + 4 * r; }
__device__ inline int acc_col(int wn, int ni, int lr, int wcols = 32) { return wn * wcols + ni * 16 + lr; }
}  // namespace lds_gemm

// TAG only names the instantiation (a profile can tell the Schur-stage launch from the others).
// TS = 64: NW = 8 (2x4 waves, 32x16 each) or 4 (2x2 waves, 32x32 each).  TS = 32 (small
// batches, where 64x64 tiles leave most CUs idle and each CU latency-bound): NW = 2, 1x2 waves
// of 32x16.
// SYM: square problems whose product is symmetric in exact arithmetic (L^-1 dM L^-T): the launch
// covers the lower tiles only, each writes its tile and the mirror image, and a diagonal tile
// mirrors its lower triangle -- the result is exactly symmetric (beta = 0, no diagonal term).
template <int BK, int NW, bool DB = false, int TS = 64>
constexpr int gemm_f64_smem() {
  return (DB ? 4 : 2) * lds_gemm::Slab<BK, 64 * NW, TS>::SZ > TS * lds_gemm::TP
             ? (DB ? 4 : 2) * lds_gemm::Slab<BK, 64 * NW, TS>::SZ
             : TS * lds_gemm::TP;
}
// one TS x TS output tile t of problem d (the body of every fp64 GEMM launch)
// SCA (op(A) = A only): A(i, k) * (sa[k] * sl[k]) -- compute_weighted_A's V diag(x lambda)
// (MPMP.jl:1659) formed while the slab is staged, with scale_cols's operation order
// DB: double-buffered slabs (two LDS images per operand): the next slab is stored into the
// other image while no wave reads it, so each k-step needs one barrier instead of two
// (round 6: the opt-in two-slab prefetch, CLRSDP_GEMM_PF=2, measured within noise in round 5
// and is gone)
template <bool TA, bool TB, int BK, int NW, bool SYM, bool SCA = false, bool DB = false, int TS = 64>
__device__ __forceinline__ void gemm_f64_tile(const GemmDesc<double>& d, int t, double* smem,
                                              double alpha, double beta,
                                              const double* __restrict__ dscal, double dmult) {
  using namespace lds_gemm;
  constexpr int NTH = 64 * NW, WM = TS / 32, WN = NW / WM, NI = TS / (16 * WN), WC = TS / WN;
  static_assert(WM * WN == NW && NI * 16 * WN == TS, "wave layout");
  using SL = Slab<BK, NTH, TS>;
  constexpr int PER = SL::PER;
  double* As = smem;
  double* Bs = smem + SL::SZ;
  const int m0 = (t / d.tn) * TS, n0 = (t % d.tn) * TS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN, lr = lane & 15, lk = lane >> 4;
  const int M = d.M, N = d.N, K = d.K;
  // A is (i, k) with i along M: contiguous along k iff TA.  B is (j, k): contiguous along k iff !TB.
  constexpr bool AK = TA, BKc = !TB;
  double ra[PER], rb[PER];
  d4 acc[2][NI];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NI; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  static_assert(!SCA || !TA, "scaled A: op(A) = A only");
  double wa[SCA ? PER : 1], wl[SCA ? PER : 1];  // the slab's column factors (loaded with it)
  auto load_w = [&](int k0) {
    if constexpr (SCA) {
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        int i, k;
        SL::template kk<AK>(tid, q, i, k);
        const int kc = min(k0 + k, K - 1);
        wa[q] = gload(d.sa + kc);
        wl[q] = gload(d.sl + kc);
      }
    }
  };
  auto scale_a = [&]() {
    if constexpr (SCA) {
#pragma unroll
      for (int q = 0; q < PER; ++q) ra[q] = ra[q] * (wa[q] * wl[q]);
    }
  };
  auto mfma_slab = [&](const double* Ac, const double* Bc) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      double af[2], bf[NI];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) af[mi] = SL::template frag<AK>(Ac, wm * 32 + mi * 16 + lr, kk + lk);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) bf[ni] = SL::template frag<BKc>(Bc, wn * WC + ni * 16 + lr, kk + lk);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
    }
  };
  SL::template load<AK>(ra, d.A, d.lda, m0, M, 0, K, tid);
  SL::template load<BKc>(rb, d.B, d.ldb, n0, N, 0, K, tid);
  load_w(0);
  // the epilogue's C_in (beta != 0) and diagonal scalar, loaded now, behind the first slab: in
  // the epilogue each C_in load sat between stores to C that may alias it (R -= dX dY is in
  // place), so the compiler waited for every one of them in turn (CPT serial round trips)
  const int rl = tid % TS, row = m0 + rl, c0 = tid / TS;
  constexpr int CPT = TS * TS / NTH, CST = NTH / TS;
  double cin[SYM ? 1 : CPT];
  double dsv = 0.0;
  if constexpr (!SYM) {
    if (beta != 0.0) {
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int col = min(n0 + c0 + CST * c, N - 1);
        cin[c] = gload(d.Cin + min(row, M - 1) + (size_t)col * d.ldcin);
      }
    }
    if (dscal) dsv = gload(dscal);
  }
  {
  scale_a();
  SL::template store<AK>(ra, As, tid, 0, K);
  SL::template store<BKc>(rb, Bs, tid, 0, K);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) {
      SL::template load<AK>(ra, d.A, d.lda, m0, M, k0 + BK, K, tid);
      SL::template load<BKc>(rb, d.B, d.ldb, n0, N, k0 + BK, K, tid);
      load_w(k0 + BK);
    }
    const double* Ac = DB ? smem + cur * 2 * SL::SZ : As;
    const double* Bc = DB ? smem + cur * 2 * SL::SZ + SL::SZ : Bs;
    mfma_slab(Ac, Bc);
    if (!more) break;
    if constexpr (DB) {
      // the other image was last read before the previous barrier
      cur ^= 1;
      scale_a();
      SL::template store<AK>(ra, smem + cur * 2 * SL::SZ, tid, k0 + BK, K);
      SL::template store<BKc>(rb, smem + cur * 2 * SL::SZ + SL::SZ, tid, k0 + BK, K);
      __syncthreads();
    } else {
      __syncthreads();
      scale_a();
      SL::template store<AK>(ra, As, tid, k0 + BK, K);
      SL::template store<BKc>(rb, Bs, tid, k0 + BK, K);
      __syncthreads();
    }
  }
  }
  __syncthreads();  // LDS slabs -> output tile
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        smem[acc_row(wm, mi, lk, r) * TP + acc_col(wn, ni, lr, WC)] = acc[mi][ni][r];
  __syncthreads();
  // thread -> row rl of the tile (consecutive threads, consecutive rows: coalesced), columns
  // cl = tid / TS + (NTH / TS) c
  if constexpr (SYM) {
#pragma unroll 4
    for (int c = 0; c < CPT; ++c) {
      const int cl = c0 + CST * c;
      if (row < M && n0 + cl < N) {
        const double v = (m0 != n0 || cl <= rl) ? smem[rl * TP + cl] : smem[cl * TP + rl];
        d.C[row + (size_t)(n0 + cl) * d.ldc] = alpha * v;
      }
      // the mirror tile: element (m0 + cl, n0 + rl) to (n0 + rl, m0 + cl)
      if (m0 != n0 && m0 + cl < M && n0 + rl < N)
        d.C[(n0 + rl) + (size_t)(m0 + cl) * d.ldc] = alpha * smem[cl * TP + rl];
    }
    return;
  }
  if constexpr (!SYM) {
    if (row < M) {
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int cl = c0 + CST * c, col = n0 + cl;
        if (col < N) {
          double v = alpha * smem[rl * TP + cl];
          if (beta != 0.0) v += beta * cin[c];
          if (dscal && row == col) v += dmult * dsv;  // fused "+ s I" (square diagonal blocks)
          d.C[row + (size_t)col * d.ldc] = v;
        }
      }
    }
  }
}

// stamp (TAG 1 and 3, the Schur-stage V^T X^-1 and V^T Y launches): stamp[0] = the earliest
// workgroup start and stamp[1] = the latest workgroup end on the 100 MHz clock
template <bool TA, bool TB, int TAG = 0, int BK = 32, int NW = 8, bool SYM = false, bool SCA = false>
__global__ __launch_bounds__(64 * NW) void gemm_f64_lds(const GemmDesc<double>* __restrict__ descs,
                                                        const TileRef* __restrict__ t2d,
                                                        double alpha, double beta,
                                                        const double* __restrict__ dscal = nullptr,
                                                        double dmult = 0.0,
                                                        unsigned long long* stamp = nullptr) {
  if constexpr (TAG == 1 || TAG == 3)
    if (stamp && threadIdx.x == 0) atomicMin(stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  __shared__ double smem[gemm_f64_smem<BK, NW>()];
  const TileRef tr = t2d[blockIdx.x];
  const GemmDesc<double> d = descs[tr.p];
  gemm_f64_tile<TA, TB, BK, NW, SYM, SCA>(d, tr.t, smem, alpha, beta, dscal, dmult);
  if constexpr (TAG == 1 || TAG == 3)
    if (stamp) {
      __syncthreads();
      if (threadIdx.x == 0) atomicMax(stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

// Uniform batch: every problem has the same shape and leading dimensions, and problem p's
// operands sit at a fixed stride from problem 0's (the block and cluster arenas).  The batch is
// passed by value in the kernel arguments, and workgroup b takes tile b / P of problem b % P
// (tile-major, problem fastest, as tile_major()), so no descriptor or tile table is read before
// the first operand load (the t2d -> desc -> operands chain cost ~2 us per launch).
struct UniGemm {
  const double* A;
  const double* B;
  const double* Cin;
  double* C;
  const double* sa;
  const double* sl;
  long long sA, sB, sCin, sC, sSa, sSl;  // per-problem strides (elements)
  int M, N, K, lda, ldb, ldcin, ldc, tn, P, tsym;  // tsym: SYM, lower tiles per problem
  int prio;  // raised wave priority (critical-path batches beside side-stream work)
};
// lower tile q (row-major over the lower triangle) -> (tm, tn)
__device__ inline void lower_tile(int q, int& tm, int& tn) {
  tm = 0;
  while ((tm + 1) * (tm + 2) / 2 <= q) ++tm;
  tn = q - tm * (tm + 1) / 2;
}
template <bool TA, bool TB, int TAG = 0, int BK = 32, int NW = 8, bool SYM = false, bool SCA = false,
          bool DB = true, int TS = 64>
__global__ __launch_bounds__(64 * NW) void gemm_f64_uni(const UniGemm u, double alpha, double beta,
                                                        const double* __restrict__ dscal = nullptr,
                                                        double dmult = 0.0,
                                                        unsigned long long* stamp = nullptr) {
  if constexpr (TAG == 1 || TAG == 3)
    if (stamp && threadIdx.x == 0) atomicMin(stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  __shared__ double smem[gemm_f64_smem<BK, NW, DB, TS>()];
  if (u.prio) __builtin_amdgcn_s_setprio(2);
  const int p = blockIdx.x % u.P, q = blockIdx.x / u.P;
  GemmDesc<double> d;
  d.A = u.A + p * u.sA;
  d.B = u.B + p * u.sB;
  d.Cin = u.Cin ? u.Cin + p * u.sCin : nullptr;
  d.C = u.C + p * u.sC;
  d.M = u.M; d.N = u.N; d.K = u.K;
  d.lda = u.lda; d.ldb = u.ldb; d.ldcin = u.ldcin; d.ldc = u.ldc; d.tn = u.tn;
  d.sa = SCA ? u.sa + p * u.sSa : nullptr;
  d.sl = SCA ? u.sl + p * u.sSl : nullptr;
  int t = q;
  if constexpr (SYM) {
    int tm, tc;
    lower_tile(q, tm, tc);
    t = tm * u.tn + tc;
  }
  gemm_f64_tile<TA, TB, BK, NW, SYM, SCA, DB, TS>(d, t, smem, alpha, beta, dscal, dmult);
  if constexpr (TAG == 1 || TAG == 3)
    if (stamp) {
      __syncthreads();
      if (threadIdx.x == 0) atomicMax(stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

// ------------------------------------------------------------------------------------------
// chain_f64: two dependent products of one block as ONE launch, by column strips,
//     T = a1 A1 op(B1)[:, S] + b1 C1[:, S]        (stage 1, n x NS, kept on chip)
//     O[:, S] = A2 T                              (stage 2)
// for every problem p of a uniform batch (n x n blocks, n <= 128, all at constant strides; a
// second pointer set for problems p >= P1, so the X and the Y blocks of the step length share
// one launch).  Each strip S of NS = 32 columns depends on its own strip of T only, so the
// intermediate never goes to HBM and the second product does not wait for a whole launch:
//   Z  = X^-1 (P Y - R)          (compute_search_direction, MPMP.jl:1698-1716)
//   dY = X^-1 (R - dX Y)         (MPMP.jl:1789-1805; symmetrised afterwards)
//   L^-1 dM L^-T = L^-1 (dM (L^-1[S, :])^T)   (compute_step_length, MPMP.jl:1853-1856), SYM:
//        the strip's lower part and its mirror image are written, so the result is exactly
//        symmetric; stage 1 stops at k = s0 + NS (L^-1 is lower triangular) and stage 2 skips
//        the row tiles above the strip.
// 512 threads: wave w owns rows 16w..16w+15 of the strip (two 16x16 MFMA tiles).  The wave's
// rows of A1 and A2 are loaded straight into registers in A-fragment order (32 k-steps x one
// double per lane each: no LDS and no barrier for the A operands), and every load of the launch
// -- A1, A2, the op(B1) strip and C1 -- is issued at the start, so the kernel sees one memory
// latency instead of one per k-slab.  op(B1)[:, S] (n x NS) is staged in LDS once, T goes from
// the accumulators to LDS in B-fragment order, and the output tile is staged in LDS so every
// store writes whole 128-row column segments.  Workgroup b takes strip b / P of problem b % P,
// so all strips of a problem share one XCD's L2 (P a multiple of 8).
// ------------------------------------------------------------------------------------------
// TRACE (one stage, the trace_A of the search direction for m = L = rank = 1, MPMP.jl:1537-1578
// with 1733-1739): U = Z V[:, S] (A1 = Z, B1 = V, n x NC) and, in the epilogue, for every
// column t of the strip  rout[t] = c_agg lam[t] (U[:, t] . V[:, t]) + c_in din[t]  -- no U in HBM
// and no separate column-sum launch.
struct ChainGemm {
  const double* A1[2];
  const double* B1[2];
  const double* C1[2];
  const double* A2[2];
  double* O[2];
  long long sA1, sB1, sC1, sA2, sO;  // per-problem strides (elements) within a pointer set
  int n, lda1, ldb1, ldc1, lda2, ldo;
  int P, P1;  // problems; p >= P1 uses pointer set 1 at index p - P1
  // TRACE only: B1 has NC columns; lam at stride sLam, din / rout at stride sX per problem
  int NC;
  const double* lam;
  const double* din;
  double* rout;
  long long sLam, sX;
  double c_in, c_agg;
  // optional (two-stage, !SYM): sum over the strip of (DA + DdA) .* (DB + O) -> dot_part[block],
  // the <X + dX, Y + dY> of the corrector's mu (same strides as O); nullptr: off
  const double* DA[2];
  const double* DdA[2];
  const double* DB[2];
  double* dot_part;
};
namespace chain {
constexpr int NS = 32, KT = 32;            // strip width; k-steps of 4 for n <= 128
constexpr int LBK = NS + 16;               // k-major B image pitch (TB1, and T)
constexpr int LBJ = 128 + 2;               // j-major B image pitch (!TB1)
constexpr int SP = NS + 1;                 // output staging pitch
constexpr int BREG = 128 * LBK;            // the op(B1) image (either layout fits)
static_assert(NS * LBJ <= BREG && 128 * SP <= BREG, "chain LDS regions");
constexpr int TOFF = BREG, END = 2 * BREG;  // op(B1) image | T image (the staging reuses the first)
constexpr size_t LDS = sizeof(double) * END;  // 96 KB
constexpr size_t LDS_TRACE = sizeof(double) * BREG;
}  // namespace chain

// DBG (timing experiments only, tools/micro/chain_bench.hip): 1 = no MFMAs, 2 = no A loads
template <bool TB1, bool SYM, bool TRACE = false, int DBG = 0>
__global__ __launch_bounds__(512) void chain_f64(const ChainGemm u, double a1, double b1) {
  using namespace chain;
  extern __shared__ __attribute__((aligned(16))) double sm_chain[];
  const int P = u.P, p = blockIdx.x % P, s = blockIdx.x / P;
  const int hs = p >= u.P1 ? 1 : 0, pl = p - hs * u.P1;
  const double* A1 = u.A1[hs] + pl * u.sA1;
  const double* B1 = u.B1[hs] + pl * u.sB1;
  const double* C1 = u.C1[hs] ? u.C1[hs] + pl * u.sC1 : nullptr;
  const double* A2 = TRACE ? nullptr : u.A2[hs] + pl * u.sA2;
  double* O = TRACE ? nullptr : u.O[hs] + pl * u.sO;
  const int n = u.n, s0 = NS * s, NC = TRACE ? u.NC : n;  // NC: columns of op(B1)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, lk = lane >> 4;
  double* Bs = sm_chain;
  double* Tm = sm_chain + TOFF;
  // stage 1 stops where L^-1[s0 + j, k] vanishes (SYM); stage 2 skips rows above the strip
  const int K1 = SYM ? min(n, s0 + NS) : n;
  const bool live1 = 16 * w < n, live2 = live1 && (!SYM || 16 * w + 15 >= s0);
  const int arow = min(16 * w + lr, n - 1);
  // ---------------- every load up front, in the order they are consumed (vmcnt retires in
  // order, so stage 1 starts when the op(B1) strip and its first A fragments are in): the
  // op(B1) strip, A1's rows (A fragments), C1, A2's rows
  double rb[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = tid + 512 * q;
    const int k = TB1 ? e >> 5 : e & 127, j = TB1 ? e & 31 : e >> 7;
    const int gk = min(k, n - 1), gj = min(s0 + j, NC - 1);
    rb[q] = gload(B1 + (TB1 ? gj + (size_t)gk * u.ldb1 : gk + (size_t)gj * u.ldb1));
  }
  double fa1[KT], fa2[TRACE ? 1 : KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int k = min(4 * t + lk, n - 1);
    fa1[t] = (DBG & 2) ? 1e-3 * (t + lane) : gload(A1 + arow + (size_t)k * u.lda1);
  }
  double cr[2][4];
#pragma unroll
  for (int u2 = 0; u2 < 2; ++u2)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = min(16 * w + lk + 4 * r, n - 1), gj = min(s0 + 16 * u2 + lr, NC - 1);
      cr[u2][r] = (!TRACE && C1) ? gload(C1 + gi + (size_t)gj * u.ldc1) : 0.0;
    }
  if constexpr (!TRACE) {
#pragma unroll
    for (int t = 0; t < KT; ++t)
      fa2[t] = (DBG & 2) ? 1e-3 * (t - lane) : gload(A2 + arow + (size_t)min(4 * t + lk, n - 1) * u.lda2);
  }
  // op(B1) strip into LDS (k-major for TB1, j-major otherwise: conflict-free stores and reads);
  // k >= n zeroed (the A fragments beyond n are clamped copies, their products must vanish)
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = tid + 512 * q;
    const int k = TB1 ? e >> 5 : e & 127, j = TB1 ? e & 31 : e >> 7;
    Bs[TB1 ? k * LBK + j : j * LBJ + k] = k < K1 ? rb[q] : 0.0;
  }
  auto fragB = [&](int k, int j) { return TB1 ? Bs[k * LBK + j] : Bs[j * LBJ + k]; };
  __syncthreads();
  // ---------------- stage 1: acc = A1 op(B1)[:, S] (k < K1)
  d4 acc[2];
  acc[0] = acc[1] = d4{0.0, 0.0, 0.0, 0.0};
  if (live1 && !(DBG & 1)) {
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if (4 * t >= K1) break;  // (uniform)
      const double b0 = fragB(4 * t + lk, lr), b1v = fragB(4 * t + lk, 16 + lr);
      acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa1[t], b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa1[t], b1v, acc[1], 0, 0, 0);
    }
  }
  if constexpr (TRACE) {
    // column dot products U[:, t] . V[:, t] (V = op(B1), in LDS): the wave's 16 rows (4
    // registers x the 4 lane groups lk), then the 8 waves in a fixed order
    __shared__ double part[8 * NS];
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * w + lk + 4 * r;
        if (row < n) v += acc[u2][r] * fragB(row, 16 * u2 + lr);
      }
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lk == 0) part[w * NS + 16 * u2 + lr] = v;
    }
    __syncthreads();
    if (tid < NS && s0 + tid < NC) {
      double v = part[tid];
#pragma unroll
      for (int q = 1; q < 8; ++q) v += part[q * NS + tid];
      const long long g = (long long)pl * u.sX + s0 + tid;
      double o = u.lam[(long long)pl * u.sLam + s0 + tid] * v * u.c_agg;
      if (u.din) o += u.din[g] * u.c_in;
      u.rout[g] = o;
    }
    return;
  } else {
    // T = a1 acc + b1 C1 -> LDS as the B operand of stage 2 (rows >= n zero)
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * w + lk + 4 * r;
        Tm[row * LBK + 16 * u2 + lr] = row < n ? a1 * acc[u2][r] + b1 * cr[u2][r] : 0.0;
      }
    __syncthreads();
    // the dot epilogue's operands, loaded while stage 2 runs (the store loop's element order)
    const bool dot = !SYM && u.dot_part != nullptr;
    double dv[NS / 4][3];
    if (dot) {
      const double* DA = u.DA[hs] + pl * u.sO;
      const double* DdA = u.DdA[hs] + pl * u.sO;
      const double* DB = u.DB[hs] + pl * u.sO;
      const int row = min(tid & 127, n - 1);
#pragma unroll
      for (int c = 0; c < NS / 4; ++c) {
        const size_t e = row + (size_t)min(s0 + (tid >> 7) + 4 * c, n - 1) * u.ldo;
        dv[c][0] = gload(DA + e);
        dv[c][1] = gload(DdA + e);
        dv[c][2] = gload(DB + e);
      }
    }
    // ---------------- stage 2: O[:, S] = A2 T
    acc[0] = acc[1] = d4{0.0, 0.0, 0.0, 0.0};
    if (live2 && !(DBG & 1)) {
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        if (4 * t >= n) break;  // (uniform)
        const double* tb = Tm + (4 * t + lk) * LBK + lr;
        acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa2[t], tb[0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa2[t], tb[16], acc[1], 0, 0, 0);
      }
    }
    // the output tile through LDS (over the op(B1) image: every wave is past its last read of
    // it, the barrier above), so the stores are 128-row column segments
    double* St = Bs;
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2)
#pragma unroll
      for (int r = 0; r < 4; ++r) St[(16 * w + lk + 4 * r) * SP + 16 * u2 + lr] = acc[u2][r];
    __syncthreads();
    {  // columns of the strip as 128-row segments (SYM: the rows on and below the diagonal)
      const int row = tid & 127;
      double dacc = 0.0;
#pragma unroll
      for (int c = 0; c < NS / 4; ++c) {
        const int cl = (tid >> 7) + 4 * c, col = s0 + cl;
        const double v = St[row * SP + cl];
        if (row < n && col < n && (!SYM || row >= col)) O[row + (size_t)col * u.ldo] = v;
        if (dot && row < n && col < n) dacc = fma(dv[c][0] + dv[c][1], dv[c][2] + v, dacc);
      }
      if (dot) {  // fixed tree: the wave (xor butterfly), then the 8 waves in order
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) dacc += __shfl_xor(dacc, o);
        __shared__ double dred[8];
        if (lane == 0) dred[w] = dacc;
        __syncthreads();
        if (tid == 0)
          u.dot_part[blockIdx.x] = ((dred[0] + dred[1]) + (dred[2] + dred[3])) + ((dred[4] + dred[5]) + (dred[6] + dred[7]));
      }
    }
    if constexpr (SYM) {  // mirror: O[col][row] for row > col, as NS-long row segments
      const int cl = tid & (NS - 1), col = s0 + cl;
#pragma unroll
      for (int c = 0; c < 128 / (512 / NS); ++c) {
        const int row = (tid / NS) + (512 / NS) * c;
        if (row < n && col < n && row > col) O[col + (size_t)row * u.ldo] = St[row * SP + cl];
      }
    }
  }
}

// Mixed batch: op(A), op(B) and (flags bit 2) alpha/beta per problem, so independent products of
// different shapes share one launch (one uniform branch per workgroup picks the instantiation).
template <int BK = 32, int NW = 8>
__global__ __launch_bounds__(64 * NW) void gemm_f64_dyn(const GemmDesc<double>* __restrict__ descs,
                                                        const TileRef* __restrict__ t2d,
                                                        double alpha, double beta) {
  __shared__ double smem[gemm_f64_smem<BK, NW>()];
  const TileRef tr = t2d[blockIdx.x];
  const GemmDesc<double> d = descs[tr.p];
  if (d.flags & 8) __builtin_amdgcn_s_setprio(2);
  const double al = (d.flags & 4) ? d.alpha : alpha, be = (d.flags & 4) ? d.beta : beta;
  // flags bit 4: "+ s I" on the diagonal of a square problem, s = *d.sa (the descriptor's scaled-A
  // pointer, unused by these unscaled products): R = mu_p I - XY in XINV's mixed batch
  const double* ds = (d.flags & 16) ? d.sa : nullptr;
  const double dm = (d.flags & 16) ? 1.0 : 0.0;
  switch (d.flags & 3) {
    case 0: gemm_f64_tile<false, false, BK, NW, false>(d, tr.t, smem, al, be, ds, dm); break;
    case 1: gemm_f64_tile<true, false, BK, NW, false>(d, tr.t, smem, al, be, ds, dm); break;
    case 2: gemm_f64_tile<false, true, BK, NW, false>(d, tr.t, smem, al, be, ds, dm); break;
    default: gemm_f64_tile<true, true, BK, NW, false>(d, tr.t, smem, al, be, ds, dm); break;
  }
}

// ------------------------------------------------------------------------------------------
// GEMM on the VALU for multi-word T: 16x16 tile, 256 threads, one output per thread.
// ------------------------------------------------------------------------------------------
template <class T, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_valu(const GemmDesc<T>* __restrict__ descs,
                                                 const TileRef* __restrict__ t2d, double alpha,
                                                 double beta) {
  // 16x16 output tile, one output per thread with two accumulation chains (even / odd k): the
  // multi-word FMA is a long dependent sequence, so the tile is small enough for a batch of
  // 64x64 blocks to put two workgroups on every CU (the 32x32 tile with 2x2 outputs per thread
  // left half the CUs idle at one wave per SIMD)
  constexpr int BM = 16, BN = 16, BK = 16;
  __shared__ T As[BK][BM + 1];
  __shared__ T Bs[BK][BN + 1];
  const TileRef tr = t2d[blockIdx.x];
  const GemmDesc<T> d = descs[tr.p];
  const int t = tr.t;
  const int m0 = (t / d.tn) * BM, n0 = (t % d.tn) * BN;
  const int tid = threadIdx.x;
  const int ti = tid & 15, tj = tid >> 4;
  T acc0 = T(0.0), acc1 = T(0.0);
  for (int k0 = 0; k0 < d.K; k0 += BK) {
    {  // A tile 16 x 16: i contiguous in memory unless TA
      const int i = TA ? (tid >> 4) : (tid & 15), k = TA ? (tid & 15) : (tid >> 4);
      const int gi = m0 + i, gk = k0 + k;
      // (an unconditional load from a clamped index and a component-wise select: a multi-word
      // value assigned under a branch stayed in scratch memory)
      const bool in = gi < d.M && gk < d.K;
      const size_t ia = in ? (TA ? gk + (size_t)gi * d.lda : gi + (size_t)gk * d.lda) : 0;
      As[k][i] = sel(in, d.A[ia], T(0.0));
    }
    {  // B tile 16 x 16: j contiguous in memory iff TB
      const int j = TB ? (tid & 15) : (tid >> 4), k = TB ? (tid >> 4) : (tid & 15);
      const int gj = n0 + j, gk = k0 + k;
      const bool in = gj < d.N && gk < d.K;
      const size_t ib = in ? (TB ? gj + (size_t)gk * d.ldb : gk + (size_t)gj * d.ldb) : 0;
      Bs[k][j] = sel(in, d.B[ib], T(0.0));
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BK; k += 2) {
      acc0 += As[k][ti] * Bs[k][tj];
      acc1 += As[k + 1][ti] * Bs[k + 1][tj];
    }
    __syncthreads();
  }
  const int row = m0 + ti, col = n0 + tj;
  if (row < d.M && col < d.N) {
    T v = (acc0 + acc1) * T(alpha);
    if (beta != 0.0) v += d.Cin[row + (size_t)col * d.ldcin] * T(beta);
    d.C[row + (size_t)col * d.ldc] = v;
  }
}

// gemm_valu_ks: the same product with 8 x 8 output tiles and K split four ways inside the
// workgroup (wave s takes k = s mod 4 of every 32-k chunk, two accumulation chains each; the
// four partial sums meet in LDS).  A multi-word FMA is ~20 (dd) to ~225 (qd) fp64 instructions,
// so one wave issuing a whole 16-long k-chunk per output was both issue- and chain-bound on the
// few workgroups of the small-block configs; here every thread carries a quarter of K and a
// launch has four times the workgroups.
template <class T, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_valu_ks(const GemmDesc<T>* __restrict__ descs,
                                                    const TileRef* __restrict__ t2d, double alpha,
                                                    double beta) {
  constexpr int BM = 8, BN = 8, BK = 32;
  __shared__ T As[BK][BM + 1];
  __shared__ T Bs[BK][BN + 1];
  __shared__ T red[4][64];
  const TileRef tr = t2d[blockIdx.x];
  const GemmDesc<T> d = descs[tr.p];
  const int t = tr.t;
  const int m0 = (t / d.tn) * BM, n0 = (t % d.tn) * BN;
  const int tid = threadIdx.x, o = tid & 63, s = tid >> 6;
  const int ti = o & 7, tj = o >> 3;
  T acc0 = T(0.0), acc1 = T(0.0);
  for (int k0 = 0; k0 < d.K; k0 += BK) {
    {  // A tile 8 x 32 (the contiguous index fastest)
      const int i = TA ? (tid >> 5) : (tid & 7), k = TA ? (tid & 31) : (tid >> 3);
      const int gi = m0 + i, gk = k0 + k;
      // (an unconditional load from a clamped index and a component-wise select: a multi-word
      // value assigned under a branch stayed in scratch memory)
      const bool in = gi < d.M && gk < d.K;
      const size_t ia = in ? (TA ? gk + (size_t)gi * d.lda : gi + (size_t)gk * d.lda) : 0;
      As[k][i] = sel(in, d.A[ia], T(0.0));
    }
    {  // B tile 32 x 8
      const int j = TB ? (tid & 7) : (tid >> 5), k = TB ? (tid >> 3) : (tid & 31);
      const int gj = n0 + j, gk = k0 + k;
      const bool in = gj < d.N && gk < d.K;
      const size_t ib = in ? (TB ? gj + (size_t)gk * d.ldb : gk + (size_t)gj * d.ldb) : 0;
      Bs[k][j] = sel(in, d.B[ib], T(0.0));
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < BK / 4; u += 2) {
      acc0 += As[s + 4 * u][ti] * Bs[s + 4 * u][tj];
      acc1 += As[s + 4 * u + 4][ti] * Bs[s + 4 * u + 4][tj];
    }
    __syncthreads();
  }
  red[s][o] = acc0 + acc1;
  __syncthreads();
  if (s != 0) return;
  const int row = m0 + ti, col = n0 + tj;
  if (row < d.M && col < d.N) {
    T v = ((red[0][o] + red[1][o]) + (red[2][o] + red[3][o])) * T(alpha);
    if (beta != 0.0) v += d.Cin[row + (size_t)col * d.ldcin] * T(beta);
    d.C[row + (size_t)col * d.ldc] = v;
  }
}

// ------------------------------------------------------------------------------------------
// Batched GEMV (the N = 1 problems of a GemmDesc batch): y = alpha op(A) x + beta y_in.
// One 256-thread workgroup per 64 outputs.  TA = false: 64 rows x 4 k-classes (coalesced along
// the rows, LDS combine of the 4 partials in a fixed order).  TA = true: each wave owns 16
// outputs (columns of A) and sweeps each with 64 lanes along k + a fixed butterfly.
// ------------------------------------------------------------------------------------------
// In-register cross-lane sums of doubles (no LDS round trip, unlike __shfl_xor which is a
// ds_bpermute): DPP quad permutes and row mirrors for lane distances 1..8, v_permlane16/32_swap
// (CDNA4) for 16 and 32.  Every lane ends with the same, order-independent result.
template <int CTRL>
__device__ inline double dpp_d(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ inline double xsum16(double x) {  // x + x[lane ^ 16]
  const auto rl = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false);
  return __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
}
__device__ inline double xsum32(double x) {  // x + x[lane ^ 32]
  const auto rl = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(x), false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(x), false, false);
  return __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
}
__device__ inline double row16_sum(double x) {  // sum over the 16 lanes of a DPP row
  x += dpp_d<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp_d<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_d<0x141>(x);  // row_half_mirror
  x += dpp_d<0x140>(x);  // row_mirror
  return x;
}
__device__ inline double wave_sum_dpp(double x) { return xsum32(xsum16(row16_sum(x))); }
__device__ inline double readlane_d(double x, int l) {  // l must be wave-uniform
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ inline double swap16_d(double x) {  // value of lane ^ 16
  const auto rl = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false);
  // lanes 0-15 / 32-47 keep their value in [0] and receive the partner's in [1]; the odd rows
  // the other way round
  const bool low = ((__lane_id() >> 4) & 1) == 0;
  return low ? __hiloint2double(rh[1], rl[1]) : __hiloint2double(rh[0], rl[0]);
}

template <class T>
__device__ __forceinline__ T shfl_xor_t(T v, int o) {
  if constexpr (sizeof(T) == 8) {
    return __shfl_xor(v, o);
  } else {
    T t;
    double* td = reinterpret_cast<double*>(&t);
    const double* vd = reinterpret_cast<const double*>(&v);
#pragma unroll
    for (int q = 0; q < (int)(sizeof(T) / 8); ++q) td[q] = __shfl_xor(vd[q], o);
    return t;
  }
}

template <class T>
__device__ __forceinline__ T shfl_t(T v, int src) {  // the value of lane src (of the wave)
  T t;
  double* td = reinterpret_cast<double*>(&t);
  const double* vd = reinterpret_cast<const double*>(&v);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(T) / 8); ++q) td[q] = __shfl(vd[q], src);
  return t;
}

// sum over the 16 lanes of a row (lanes 16r..16r+15)
template <class T>
__device__ __forceinline__ T row16_sum_t(T v) {
  if constexpr (sizeof(T) == 8) {
    return row16_sum(v);
  } else {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += shfl_xor_t(v, o);
    return v;
  }
}

// y = alpha op(A) x + beta y for every problem; 64 outputs per 256-thread workgroup.
//  !TA: thread (row r = tid & 63, k-group g = tid >> 6) sums k = g, g+4, ... with 8 loads in
//       flight; the 4 k-groups are combined through LDS.
//   TA: wave w owns 16 outputs (columns); lane (k-offset kk = lane & 15, column c4 = lane >> 4)
//       streams 4 columns at once (16 consecutive k per column per load instruction), 4 column
//       groups x 2 k-steps of loads in flight; each column sum is a 16-lane DPP reduction.
//       Multi-word with DEEP: thread per column and k-group as !TA (the quad-double default).
template <class T, bool TA, bool DEEP = true>
__global__ __launch_bounds__(256) void gemv_batched(const GemmDesc<T>* __restrict__ descs,
                                                    const TileRef* __restrict__ t2d, double alpha,
                                                    double beta) {
  const TileRef tr = t2d[blockIdx.x];
  const GemmDesc<T> d = descs[tr.p];
  const int o0 = tr.t * 64;
  const int tid = threadIdx.x;
  const T* __restrict__ A = d.A;
  const T* __restrict__ x = d.B;
  const int K = d.K;
  if (!TA) {
    __shared__ T part[4][64];
    const int r = tid & 63, g = tid >> 6, i = o0 + r;
    const int ic = min(i, d.M - 1);
    T acc0 = T(0.0), acc1 = T(0.0);
    if constexpr (sizeof(T) == 8 && DEEP) {
      // fp64: 32 elements of the row in flight per thread (a GEMV is a stream: the bytes in
      // flight per CU, not the FMAs, set its rate), the tail by clamped loads times zero
      for (int k0 = g; k0 < K; k0 += 128) {
        T a[32], xv[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
          const int k = min(k0 + 4 * u, K - 1);
          a[u] = A[ic + (size_t)k * d.lda];
          xv[u] = k0 + 4 * u < K ? x[k] : T(0.0);
        }
#pragma unroll
        for (int u = 0; u < 32; u += 2) {
          acc0 += a[u] * xv[u];
          acc1 += a[u + 1] * xv[u + 1];
        }
      }
    } else {
      int k = g;
      for (; k + 28 < K; k += 32) {
        T a[8], xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          a[u] = A[ic + (size_t)(k + 4 * u) * d.lda];
          xv[u] = x[k + 4 * u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
          acc0 += a[u] * xv[u];
          acc1 += a[u + 1] * xv[u + 1];
        }
      }
      for (; k < K; k += 4) acc0 += A[ic + (size_t)k * d.lda] * x[k];
    }
    part[g][r] = acc0 + acc1;
    __syncthreads();
    if (g == 0 && i < d.M) {
      T v = ((part[0][r] + part[1][r]) + (part[2][r] + part[3][r])) * T(alpha);
      if (beta != 0.0) v += d.Cin[i] * T(beta);
      d.C[i] = v;
    }
  } else if constexpr (sizeof(T) > 8 && DEEP) {
    // multi-word: thread (column r, k-group g) walks down its column (k = g, g+4, ...; the
    // column is contiguous), the 4 k-groups combined through LDS -- the 16-lane cross-lane
    // reduction of the fp64 layout costs four multi-word additions and 4 x words shuffles per
    // column there, more than the products themselves at these sizes (K ~ 50)
    __shared__ T part[4][64];
    const int r = tid & 63, g = tid >> 6, j = o0 + r;
    const T* col = A + (size_t)min(j, d.M - 1) * d.lda;
    T acc0 = T(0.0), acc1 = T(0.0);
    int k = g;
    for (; k + 4 < K; k += 8) {
      acc0 += col[k] * x[k];
      acc1 += col[k + 4] * x[k + 4];
    }
    if (k < K) acc0 += col[k] * x[k];
    part[g][r] = acc0 + acc1;
    __syncthreads();
    if (g == 0 && j < d.M) {
      T v = ((part[0][r] + part[1][r]) + (part[2][r] + part[3][r])) * T(alpha);
      if (beta != 0.0) v += d.Cin[j] * T(beta);
      d.C[j] = v;
    }
  } else {
    const int lane = tid & 63, w = tid >> 6, kk = lane & 15, c4 = lane >> 4;
    const int jb = o0 + w * 16;  // this wave's 16 columns: jb + 4q + c4, q = 0..3
    const T* col[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) col[q] = A + (size_t)min(jb + 4 * q + c4, d.M - 1) * d.lda;
    T acc[4] = {T(0.0), T(0.0), T(0.0), T(0.0)};
    int k = kk;
    if constexpr (sizeof(T) == 8 && DEEP) {  // fp64: 8 k-steps (32 column elements) in flight per lane
      for (; k + 112 < K; k += 128) {
        T av[4][8], xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          xv[u] = x[k + 16 * u];
#pragma unroll
          for (int q = 0; q < 4; ++q) av[q][u] = col[q][k + 16 * u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] += av[q][u] * xv[u] + av[q][u + 1] * xv[u + 1];
      }
    }
    for (; k + 16 < K; k += 32) {
      T a0[4], a1[4];
      const T x0 = x[k], x1 = x[k + 16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a0[q] = col[q][k];
        a1[q] = col[q][k + 16];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += a0[q] * x0 + a1[q] * x1;
    }
    if (k < K) {
      const T x0 = x[k];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += col[q][k] * x0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const T s = row16_sum_t(acc[q]);
      const int j = jb + 4 * q + c4;
      if (kk == 0 && j < d.M) {
        T v = s * T(alpha);
        if (beta != 0.0) v += d.Cin[j] * T(beta);
        d.C[j] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Flat 2-level reductions over a contiguous range (deterministic: fixed chunking + fixed tree)
//   op 0: sum a.*b    op 1: sum (a+da).*(b+db)    op 2: max |a|
// ------------------------------------------------------------------------------------------
// acc + a b as one fused operation for fp64 (spelled out, so that flat_reduce and update_state
// produce bitwise the same partial sums)
template <class T>
__device__ __forceinline__ T madd(T acc, T a, T b) {
  if constexpr (sizeof(T) == 8) return fma(a, b, acc);
  else return acc + a * b;
}

// flat_reduce's chunk of workgroup `blk` out of `nblk` over [0, n)
__device__ __forceinline__ void flat_chunk(long long n, int blk, int nblk, long long& lo,
                                           long long& hi) {
  const long long chunk = (n + nblk - 1) / nblk;
  lo = (long long)blk * chunk;
  hi = lo + chunk < n ? lo + chunk : n;
}

// The state update of a loop body (MPMP.jl:877-887): X += alpha_p dX, Y += alpha_d dY,
// x += alpha_p dx, y += alpha_d dy -- all skipped when a status word info[0..ninfo) is set (a
// failed factorisation or a halted loop) -- with the sums the next steps need folded in: per
// workgroup the partial <X,Y> of the new state (the next iteration's mu, with flat_reduce's
// chunking, per-thread order and tree, so it is bitwise flat_reduce's partial), <c,x> and <b,y>
// (the objectives, MPMP.jl:940-941).  part = [<X,Y> | <c,x> | <b,y>], gridDim.x partials each.
// The step lengths folded into the update (one rank, a loop body): every workgroup forms
// lambda_min of X and Y as the minimum over the blocks (scalar_kernel's fold: lane l takes
// blocks l, l+64, ..., then the xor butterfly; min is exact, so the order is immaterial) and
// alpha = min(1, -gamma / lambda_min), the pd-feasible alpha_p = alpha_d = min of the two
// (MPMP.jl:863-874, 1893-1897; scalar_kernel which == 2); workgroup 0 writes the four slots.
template <class T> struct StepAlpha {
  const T* eigX;
  const T* eigY;
  int nb;       // blocks (0: alpha from the slots, as computed by the STEP stage)
  int pd_feas;  // 0/1 from the host, -1: sc[pdslot] (decided on the device)
  T gamma;
  T* sc;
  int sx, sy, sap, sad, pdslot;
};
template <class T>
__device__ __forceinline__ T min_fold64(const T* v, int cnt, int lane) {
  T acc = v[0];
  bool have = false;
  for (int i = lane; i < cnt; i += 64) {
    const T e = v[i];
    if (!have) { acc = e; have = true; }
    else if (e < acc) acc = e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const T e = shfl_xor_t(acc, o);
    if (e < acc) acc = e;
  }
  return acc;
}
template <class T>
__global__ __launch_bounds__(256) void update_state(T* __restrict__ X, const T* __restrict__ dX,
                                                    T* __restrict__ Y, const T* __restrict__ dY,
                                                    long long nb, T* __restrict__ x,
                                                    const T* __restrict__ dx, long long nx,
                                                    const T* __restrict__ cv, T* __restrict__ y,
                                                    const T* __restrict__ dy, long long ny,
                                                    const T* __restrict__ bv, const T* alpha_p,
                                                    const T* alpha_d, const int* info, int ninfo,
                                                    T* __restrict__ part, StepAlpha<T> sa) {
  __shared__ T red[3][256];
  __shared__ T alph[2];
  const int tid = threadIdx.x, G = gridDim.x, g = blockIdx.x;
  long long lo, hi;
  flat_chunk(nb, g, G, lo, hi);
  // the first PF elements of X, Y, dX, dY are in flight while the step lengths and the status
  // words are formed (wave 0: alpha; waves 1-3: the status words, OR-ed by the barrier)
  constexpr int PF = 4;
  T px[PF], py[PF], pdx[PF], pdy[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const long long e = lo + tid + 256 * u;
    px[u] = py[u] = pdx[u] = pdy[u] = T(0.0);
    if (e < hi) {
      px[u] = X[e];
      py[u] = Y[e];
      pdx[u] = dX[e];
      pdy[u] = dY[e];
    }
  }
  int flag = 0;
  if (sa.nb > 0 && tid < 64) {
    const T mx = min_fold64(sa.eigX, sa.nb, tid), my = min_fold64(sa.eigY, sa.nb, tid);
    if (tid == 0) {
      const T gm = sa.gamma;
      T ap = T(1.0), ad = T(1.0);
      if (!(mx > -gm)) ap = -gm / mx;
      if (!(my > -gm)) ad = -gm / my;
      const bool pdf = sa.pd_feas < 0 ? sa.sc[sa.pdslot] > T(0.5) : sa.pd_feas != 0;
      if (pdf) {
        if (ad < ap) ap = ad;
        else ad = ap;
      }
      alph[0] = ap;
      alph[1] = ad;
      if (g == 0) {
        sa.sc[sa.sx] = mx;
        sa.sc[sa.sy] = my;
        sa.sc[sa.sap] = ap;
        sa.sc[sa.sad] = ad;
      }
    }
  } else {
    const int t0 = sa.nb > 0 ? tid - 64 : tid, ts = sa.nb > 0 ? 192 : 256;
    for (int i = t0; i < ninfo; i += ts) flag |= info[i] != 0;
  }
  const bool upd = !__syncthreads_or(flag);
  const T ap = sa.nb > 0 ? alph[0] : *alpha_p, ad = sa.nb > 0 ? alph[1] : *alpha_d;
  T axy = T(0.0), acx = T(0.0), aby = T(0.0);
  auto step = [&](long long e, T xv, T yv, T dxv, T dyv) {
    if (upd) {
      xv = xv + ap * dxv;
      yv = yv + ad * dyv;
      X[e] = xv;
      Y[e] = yv;
    }
    axy = madd(axy, xv, yv);
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const long long e = lo + tid + 256 * u;
    if (e < hi) step(e, px[u], py[u], pdx[u], pdy[u]);
  }
#pragma unroll 4
  for (long long e = lo + tid + 256 * PF; e < hi; e += 256) step(e, X[e], Y[e], dX[e], dY[e]);
  flat_chunk(nx, g, G, lo, hi);
  for (long long e = lo + tid; e < hi; e += 256) {
    T v = x[e];
    if (upd) { v = v + ap * dx[e]; x[e] = v; }
    acx = madd(acx, cv[e], v);
  }
  flat_chunk(ny, g, G, lo, hi);
  for (long long e = lo + tid; e < hi; e += 256) {
    T v = y[e];
    if (upd) { v = v + ad * dy[e]; y[e] = v; }
    aby = madd(aby, bv[e], v);
  }
  red[0][tid] = axy;
  red[1][tid] = acx;
  red[2][tid] = aby;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s)
#pragma unroll
      for (int q = 0; q < 3; ++q) red[q][tid] = red[q][tid] + red[q][tid + s];
    __syncthreads();
  }
  if (tid < 3) part[tid * G + g] = red[tid][0];
}
template <class T>
__global__ __launch_bounds__(256) void flat_reduce(const T* __restrict__ a, const T* __restrict__ b,
                                                   const T* __restrict__ da,
                                                   const T* __restrict__ db, long long n, int op,
                                                   T* __restrict__ partial) {
  __shared__ T red[256];
  const long long chunk = (n + gridDim.x - 1) / gridDim.x;
  const long long lo = (long long)blockIdx.x * chunk;
  const long long hi = lo + chunk < n ? lo + chunk : n;
  T acc = T(0.0);
  // one loop per operation (uniform), unrolled so the loads of several elements are in flight;
  // the per-thread accumulation order is unchanged
  if (op == 0) {
#pragma unroll 4
    for (long long e = lo + threadIdx.x; e < hi; e += blockDim.x) acc = madd(acc, a[e], b[e]);
  } else if (op == 1) {
#pragma unroll 4
    for (long long e = lo + threadIdx.x; e < hi; e += blockDim.x) acc += (a[e] + da[e]) * (b[e] + db[e]);
  } else {
#pragma unroll 4
    for (long long e = lo + threadIdx.x; e < hi; e += blockDim.x) {
      const T v = Num<T>::abs_(a[e]);
      if (v > acc) acc = v;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      if (op == 2) { if (red[threadIdx.x + s] > red[threadIdx.x]) red[threadIdx.x] = red[threadIdx.x + s]; }
      else red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}


// ------------------------------------------------------------------------------------------
// Block reductions (deterministic: fixed tree over a fixed thread->element map)
// ------------------------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] = red[tid] + red[tid + s];
    __syncthreads();
  }
  T r = red[0];
  __syncthreads();
  return r;
}
template <class T>
__device__ __forceinline__ T block_max(T v, T* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (tid < s) { if (red[tid + s] > red[tid]) red[tid] = red[tid + s]; }
    __syncthreads();
  }
  T r = red[0];
  __syncthreads();
  return r;
}

// ------------------------------------------------------------------------------------------
// Cholesky A = L L^T in place (lower triangle), one 256-thread workgroup per matrix, blocked
// right-looking with NB-column panels; the panel lives in LDS, the trailing matrix in global
// memory (L2-resident at the sizes of this solver).  info[b] = 0 on success, else the 1-based
// column at which a non-positive pivot appeared (the reference's status 0 of spd_inv!/cho!).
// ------------------------------------------------------------------------------------------
// sqrt(d) and 1/sqrt(d) of a positive pivot.  Double-double: the hardware reciprocal square root
// refined by two fp64 Newton steps and one double-double Newton step, then s = d r -- no IEEE
// division or square-root sequence on the factorisations' serial pivot chain.
template <class T>
__device__ inline void pivot_sqrt(const T& d, T& s, T& r) {
  s = Num<T>::sqrt_(d);
  r = T(1.0) / s;
}
template <>
__device__ inline void pivot_sqrt<mw::dd>(const mw::dd& d, mw::dd& s, mw::dd& r) {
  double r0 = __builtin_amdgcn_rsq(d.hi);
  r0 = r0 * fma(-0.5 * d.hi, r0 * r0, 1.5);
  r0 = r0 * fma(-0.5 * d.hi, r0 * r0, 1.5);
  const mw::dd rr(r0);
  const mw::dd e = mw::dd(1.0) - d * (rr * rr);
  r = rr + (rr * e) * 0.5;
  s = d * r;
}

template <>
__device__ inline void pivot_sqrt<mw::qd>(const mw::qd& d, mw::qd& s, mw::qd& r) {
  // Newton on 1/sqrt(d), r += r (1 - d r^2) / 2, with precision doubling: fp64 (hardware rsq and
  // two fp64 steps, ~53 bits), one double-double step (~104 bits), then two steps whose residual
  // e = 1 - d r^2 is quad-double and whose correction r e / 2 (|e| < 2^-100) is double-double.
  // The second quad-double step also absorbs the double-double rounding of the first.  Four
  // quad-double products and s = d r on the factorisations' serial pivot chain, against nine
  // and s for three full quad-double steps (CLRSDP_QD_PIVOT_FULL: those, for A/B).
#ifdef CLRSDP_QD_PIVOT_FULL
  const mw::qd h = d * 0.5;
  r = mw::qd(1.0 / sqrt(d.x[0]));
  for (int it = 0; it < 3; ++it) r = r + r * (mw::qd(0.5) - h * (r * r));
#else
  double r0 = __builtin_amdgcn_rsq(d.x[0]);
  r0 = r0 * fma(-0.5 * d.x[0], r0 * r0, 1.5);
  r0 = r0 * fma(-0.5 * d.x[0], r0 * r0, 1.5);
  const mw::dd d2(d.x[0], d.x[1]);
  mw::dd r2(r0);
  r2 = r2 + (r2 * (mw::dd(1.0) - d2 * (r2 * r2))) * 0.5;
  r = mw::qd(r2);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const mw::qd e = mw::qd(1.0) - d * (r * r);
    r = r + mw::qd((mw::dd(r.x[0], r.x[1]) * mw::dd(e.x[0], e.x[1])) * 0.5);
  }
#endif
  s = d * r;
}
// 1/q: double-double from the hardware reciprocal (two fp64 Newton steps) and one
// double-double Newton step
template <class T>
__device__ inline T recip_fast(const T& q) { return T(1.0) / q; }
template <>
__device__ inline mw::dd recip_fast<mw::dd>(const mw::dd& q) {
  double r0 = __builtin_amdgcn_rcp(q.hi);
  r0 = fma(fma(-q.hi, r0, 1.0), r0, r0);
  r0 = fma(fma(-q.hi, r0, 1.0), r0, r0);
  const mw::dd rr(r0);
  const mw::dd e = mw::dd(1.0) - q * rr;
  return rr + rr * e;
}
// 1/q at quad-double: the double-double reciprocal of the leading limbs, then two Newton steps
// r += r (1 - q r) with a quad-double residual and a double-double correction (as pivot_sqrt):
// two quad-double products against the long division's chain of quad-double x double steps
template <>
__device__ inline mw::qd recip_fast<mw::qd>(const mw::qd& q) {
#ifdef CLRSDP_QD_PIVOT_FULL
  return mw::qd(1.0) / q;
#else
  mw::qd r(recip_fast(mw::dd(q.x[0], q.x[1])));
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const mw::qd e = mw::qd(1.0) - q * r;
    r = r + mw::qd(mw::dd(r.x[0], r.x[1]) * mw::dd(e.x[0], e.x[1]));
  }
  return r;
#endif
}

// a (quad-double) x b (double-double): the truncated quad-double product with b's words 2, 3 zero
// written out (the O(eps^3) terms a2 b1 + a3 b0 kept, as in operator*): ~70 operations against
// ~115 for the full product
__device__ inline mw::qd qd_mul_dd(const mw::qd& a, const mw::dd& b) {
  MW_EXACT
  double q0, q1, q2, q4, q5;
  const double p0 = mw::two_prod(a.x[0], b.hi, q0);
  double p1 = mw::two_prod(a.x[0], b.lo, q1);
  double p2 = mw::two_prod(a.x[1], b.hi, q2);
  const double p4 = mw::two_prod(a.x[1], b.lo, q4);
  const double p5 = mw::two_prod(a.x[2], b.hi, q5);
  mw::three_sum(p1, p2, q0);
  mw::three_sum(p2, q1, q2);
  double e4, t0, t1;
  const double p3 = mw::two_sum(p4, p5, e4);
  const double s0 = mw::two_sum(p2, p3, t0);
  double s1 = mw::two_sum(q1, e4, t1);
  double s2 = q2;
  s1 = mw::two_sum(s1, t0, t0);
  s2 += (t0 + t1);
  s1 += a.x[2] * b.lo + a.x[3] * b.hi + q0 + q4 + q5;
  return mw::qd_renorm(p0, p1, s0, s1, s2);
}
// 1/q at quad-double with ONE Newton step from the double-double reciprocal r (the LDL pivot of
// chol_lookahead with opts bit 1, round 6 form): e = 1 - q r to double-double (|e| ~ 2^-104:
// 1 - q0 r exact, the rest by two-sums, ~2^-210 absolute), then r + r e as the four words
// (r.hi, r.lo, (r e).hi, (r e).lo) renormalised -- ~2^-208 relative as before, but ~160
// operations on the serial pivot chain against ~330 (a quad-double product, two quad-double
// additions)
__device__ inline mw::qd recip_qd_newton1(const mw::qd& q) {
  MW_EXACT
  const mw::dd r = recip_fast(mw::dd(q.x[0], q.x[1]));
  const mw::qd p = qd_mul_dd(q, r);
  double e1, e2;
  const double eh = mw::two_sum(1.0 - p.x[0], -p.x[1], e1);  // (1 - p0 exact: p0 = 1 to ~2^-104)
  const double s = mw::two_sum(eh, -p.x[2], e2);
  double el;
  const double eq = mw::quick_two_sum(s, (e1 + e2) - p.x[3], el);
  const mw::dd d = r * mw::dd(eq, el);
  return mw::qd_renorm(r.hi, r.lo, d.hi, d.lo, 0.0);
}

template <class T, int NB, int NT = 256>
__global__ __launch_bounds__(NT) void potrf_batched(const MatDesc<T>* __restrict__ descs,
                                                     int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* D = reinterpret_cast<T*>(smem_raw);  // NB x NB diagonal block (column-major)
  T* P = D + NB * NB;                      // panel: P[q * pm + i]
  __shared__ int fail;
  __shared__ T rdg[NB];  // reciprocals of the block's pivots (one division each, by thread 0)
  const MatDesc<T> d = descs[blockIdx.x];
  T* A = d.A;
  const int n = d.n, lda = d.lda, tid = threadIdx.x;
  if (tid == 0) fail = 0;
  __syncthreads();
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int nb = min(NB, n - k0);
    for (int e = tid; e < nb * nb; e += blockDim.x) {
      const int i = e % nb, j = e / nb;
      D[i + j * NB] = A[(k0 + i) + (size_t)(k0 + j) * lda];
    }
    __syncthreads();
    for (int j = 0; j < nb; ++j) {
      if (tid == 0) {
        const T djj = D[j + j * NB];
        if (!(djj > T(0.0))) {
          fail = k0 + j + 1;
        } else {
          T sj, rj;
          pivot_sqrt(djj, sj, rj);
          D[j + j * NB] = sj;
          rdg[j] = rj;
        }
      }
      __syncthreads();
      if (fail) break;
      const T rpiv = rdg[j];
      for (int i = j + 1 + tid; i < nb; i += blockDim.x) D[i + j * NB] = D[i + j * NB] * rpiv;
      __syncthreads();
      const int r = nb - j - 1;
      for (int e = tid; e < r * r; e += blockDim.x) {
        const int i = j + 1 + e % r, c = j + 1 + e / r;
        if (i >= c) D[i + c * NB] = D[i + c * NB] - D[i + j * NB] * D[c + j * NB];
      }
      __syncthreads();
    }
    if (fail) break;
    for (int e = tid; e < nb * nb; e += blockDim.x) {
      const int i = e % nb, j = e / nb;
      if (i >= j) A[(k0 + i) + (size_t)(k0 + j) * lda] = D[i + j * NB];
    }
    const int k1 = k0 + nb, pm = n - k1;
    if (pm <= 0) break;
    // panel L21 = A21 L11^-T, one row per thread
    // (row[] in registers: the loops run to the compile-time NB with a uniform guard, so every
    // index is static -- a runtime bound put the array in scratch memory)
    for (int i = tid; i < pm; i += blockDim.x) {
      T row[NB];
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        if (q < nb) {
          T x = A[(k1 + i) + (size_t)(k0 + q) * lda];
#pragma unroll
          for (int p = 0; p < q; ++p) x = x - row[p] * D[q + p * NB];
          x = x * rdg[q];
          row[q] = x;
          P[q * pm + i] = x;
          A[(k1 + i) + (size_t)(k0 + q) * lda] = x;
        }
      }
    }
    __syncthreads();
    // trailing update A22 -= L21 L21^T (lower triangle)
    for (int e = tid; e < pm * pm; e += blockDim.x) {
      const int i = e % pm, j = e / pm;
      if (i >= j) {
        T s = T(0.0);
        for (int q = 0; q < nb; ++q) s += P[q * pm + i] * P[q * pm + j];
        A[(k1 + i) + (size_t)(k1 + j) * lda] = A[(k1 + i) + (size_t)(k1 + j) * lda] - s;
      }
    }
    __syncthreads();
  }
  if (tid == 0) info[blockIdx.x] = fail;
}

// ------------------------------------------------------------------------------------------
// Triangular solves with a lower triangular L (potrf's, non-unit), in place on B:
//   TRANS = false:  B <- L^-1 B     (forward substitution)
//   TRANS = true :  B <- L^-T B     (backward substitution)
// UNIT: L has a unit diagonal (the L factor of getrf_batched, approx_solve_tril!(.., 1)).
// STORE_T: L is read transposed from upper storage, L(i, j) = A[j + i*ld] -- with the U factor
// of getrf_batched: forward U^T x = b (B^T U^-1, MPMP.jl:1457-1460) and, with TRANS, backward
// U x = b (approx_solve_triu!, MPMP.jl:1772).
// One workgroup per (matrix, NC-column tile of B); NB-row blocks; L panel staged in LDS.  The
// diagonal enters as reciprocals (one per row, not per right-hand side: a multi-word division
// is an order of magnitude dearer than a product; multi-word words take recip_fast's Newton
// form).  Multi-word words also pre-scale the diagonal block's off-diagonal entries by those
// reciprocals (column q by 1/l_qq; transposed: row q), so that the serial chain of the block
// solve carries one product per row (v_r -= l_rq/l_qq v_q) and x_q = v_q/l_qq leaves it.
// ------------------------------------------------------------------------------------------
template <class T, bool TRANS, int NB, int NC, int NT = 256, bool UNIT = false, bool STORE_T = false>
__global__ __launch_bounds__(NT) void trsm_batched(const TrsmDesc<T>* __restrict__ descs,
                                                    const int* __restrict__ t2d) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* D = reinterpret_cast<T*>(smem_raw);  // NB x NB diagonal block of L (column-major)
  T* Xs = D + NB * NB;                     // NB x NC solved rows
  T* P = Xs + NB * NC;                     // panel NB x n
  __shared__ T rdg[NB];                    // reciprocals of the block's diagonal
  const TrsmDesc<T> d = descs[t2d[blockIdx.x]];
  const int c0 = (blockIdx.x - d.tile0) * NC;
  const int nc = min(NC, d.nrhs - c0);
  const int n = d.n, tid = threadIdx.x;
  const T* L = d.L;
  const size_t ldl = d.ldl;
  auto lat = [&](int i, int j) -> T { return STORE_T ? L[j + (size_t)i * ldl] : L[i + (size_t)j * ldl]; };
  constexpr bool PS = !UNIT && !std::is_same<T, double>::value;  // pre-scaled diagonal block
  T* B = d.B + (size_t)c0 * d.ldb;
  const int nblk = (n + NB - 1) / NB;
  for (int bi = 0; bi < nblk; ++bi) {
    const int i0 = TRANS ? (nblk - 1 - bi) * NB : bi * NB;
    const int nb = min(NB, n - i0);
    for (int e = tid; e < nb * nb; e += blockDim.x) {
      const int i = e % nb, j = e / nb;
      D[i + j * NB] = lat(i0 + i, i0 + j);
    }
    if (tid < nb) {
      if (UNIT) rdg[tid] = T(1.0);
      else rdg[tid] = recip_fast(lat(i0 + tid, i0 + tid));
    }
    if constexpr (PS) {
      __syncthreads();
      for (int e = tid; e < nb * nb; e += blockDim.x) {
        const int i = e % nb, j = e / nb;
        if (i > j) D[i + j * NB] = D[i + j * NB] * rdg[TRANS ? i : j];
      }
    }
    // panel of the rows still to be updated
    const int pr0 = TRANS ? 0 : i0 + nb;
    const int pm = TRANS ? i0 : n - i0 - nb;
    for (int e = tid; e < nb * pm; e += blockDim.x) {
      const int i = e % pm, q = e / pm;
      // non-trans: P[q][i] = L[pr0 + i, i0 + q];  trans: P[q][i] = L[i0 + q, i]
      P[q * pm + i] = TRANS ? lat(i0 + q, i) : lat(pr0 + i, i0 + q);
    }
    __syncthreads();
    // the diagonal block, column-oriented: lane r of a 16-lane group holds row r of one
    // right-hand side; per q the owner of row q finalises x_q (times 1/l_qq), the group reads it
    // by a shuffle and rows beyond it subtract l_rq x_q -- 16 short steps instead of one
    // thread's serial chain of nb(nb+1)/2 multi-word products per column (forward: the same
    // operation order per row as the row-oriented form)
    for (int cb = 0; cb < nc; cb += NT / 16) {  // uniform: NT/16 right-hand sides per pass
      const int r = tid & 15, c = cb + (tid >> 4), base = tid & 48;
      const bool act = r < nb && c < nc;
      T v = T(0.0);
      if (act) v = B[(i0 + r) + (size_t)c * d.ldb];
      T xr = T(0.0);
      if constexpr (PS) {
        // v_q is final once the steps before q have run: broadcast it, scale it off the chain
#pragma unroll
        for (int qq = 0; qq < NB; ++qq) {
          const int q = TRANS ? NB - 1 - qq : qq;
          if (q < nb) {
            const T vq = shfl_t(v, base + q);
            if (r == q) xr = v * rdg[q];
            if (TRANS ? r < q : r > q) v = v - (TRANS ? D[q + r * NB] : D[r + q * NB]) * vq;
          }
        }
      } else if (!TRANS) {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          if (q < nb) {
            if (r == q) { if (UNIT) xr = v; else xr = v * rdg[q]; }
            const T xq = shfl_t(xr, base + q);
            if (r > q) v = v - D[r + q * NB] * xq;
          }
        }
      } else {
#pragma unroll
        for (int q = NB - 1; q >= 0; --q) {
          if (q < nb) {
            if (r == q) { if (UNIT) xr = v; else xr = v * rdg[q]; }
            const T xq = shfl_t(xr, base + q);
            if (r < q) v = v - D[q + r * NB] * xq;
          }
        }
      }
      if (act) {
        B[(i0 + r) + (size_t)c * d.ldb] = xr;
        Xs[r * NC + c] = xr;
      }
    }
    __syncthreads();
    for (int e = tid; e < pm * nc; e += blockDim.x) {
      const int i = e % pm, c = e / pm;
      T s = T(0.0);
      for (int q = 0; q < nb; ++q) s += P[q * pm + i] * Xs[q * NC + c];
      T* bp = B + (pr0 + i) + (size_t)c * d.ldb;
      *bp = *bp - s;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// trsv_wave: the multi-word vector solves of potrf's L (n <= 64, a few right-hand sides:
// t_j = L_j^-1 rhs_j, the two solves with L_Q, dx_j = L_j^-T (...), MPMP.jl:1751-1773), one wave
// per right-hand side with lane r holding row r.  The workgroup first stages L with its
// off-diagonal entries scaled by the reciprocal pivots into LDS, in the order the wave reads
// them (Ls[r + 64 q] = l_rq / l_qq, transposed: l_qr / l_qq), so each of the n serial steps is
// one broadcast (v_readlane) and one multi-word product and subtraction per lane:
//   v_r -= Ls[r, q] v_q   (r > q; transposed r < q),   and at the end x_r = v_r / l_rr.
// trsm_batched's 16-row blocks carried, per block, a 16-step diagonal chain AND a 16-long
// dependent dot product per row of the panel update on a mostly idle workgroup.
// One workgroup per (matrix, NW right-hand sides), t2d as for trsm_batched with NC = NW.
// ------------------------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ T readlane_t(const T& v, int src) {  // src wave-uniform
  T t;
  int* ti = reinterpret_cast<int*>(&t);
  const int* vi = reinterpret_cast<const int*>(&v);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(T) / 4); ++q) ti[q] = __builtin_amdgcn_readlane(vi[q], src);
  return t;
}
// one step's update v - c vq of the vector solves: double-double with fms_fast (one two-sum, the
// low words added plainly: its absolute error ~2u^2(|v| + |c vq|) is the componentwise bound the
// backward analysis of a triangular solve asks of each update, as for the factorisations' trailing
// updates), the accurate operations otherwise
template <class T> __device__ __forceinline__ T trsv_fms(const T& v, const T& c, const T& vq) {
  return v - c * vq;
}
template <> __device__ __forceinline__ mw::dd trsv_fms(const mw::dd& v, const mw::dd& c, const mw::dd& vq) {
  return mw::fms_fast(v, c, vq);
}
// two rows' fms_fast against one broadcast value with the two dependent chains interleaved
// operation by operation (left to itself the scheduler issues one chain after the other, and a
// lone chain waits out every fp64 latency); the same operations as mw::fms_fast per row
template <class T>
__device__ __forceinline__ void trsv_fms2(T& w0, const T& a0, const T& b0, T& w1, const T& a1,
                                          const T& b1, const T& c) {
  w0 = trsv_fms(a0, b0, c);
  w1 = trsv_fms(a1, b1, c);
}
template <>
__device__ __forceinline__ void trsv_fms2(mw::dd& w0, const mw::dd& a0, const mw::dd& b0, mw::dd& w1,
                                          const mw::dd& a1, const mw::dd& b1, const mw::dd& c) {
  MW_EXACT
#define TSB __builtin_amdgcn_sched_barrier(0);
  const double p1a = b0.hi * c.hi, p1b = b1.hi * c.hi;
  TSB double p2a = fma(b0.hi, c.hi, -p1a), p2b = fma(b1.hi, c.hi, -p1b);
  TSB p2a = fma(b0.hi, c.lo, p2a); p2b = fma(b1.hi, c.lo, p2b);
  TSB p2a = fma(b0.lo, c.hi, p2a); p2b = fma(b1.lo, c.hi, p2b);
  // two_sum(a.hi, -p1)
  TSB const double sa = a0.hi + (-p1a), sb = a1.hi + (-p1b);
  TSB const double ba = sa - a0.hi, bb = sb - a1.hi;
  TSB const double ta = sa - ba, tb = sb - bb;
  TSB const double ua = a0.hi - ta, ub = a1.hi - tb;
  TSB const double va = (-p1a) - ba, vb = (-p1b) - bb;
  TSB double ea = ua + va, eb = ub + vb;
  TSB const double la = a0.lo - p2a, lb = a1.lo - p2b;
  TSB ea = ea + la; eb = eb + lb;
  // quick_two_sum(s, e)
  TSB const double ra = sa + ea, rb = sb + eb;
  TSB const double za = ra - sa, zb = rb - sb;
  TSB w0 = mw::dd(ra, ea - za);
  w1 = mw::dd(rb, eb - zb);
#undef TSB
}
template <class T> constexpr size_t trsv_wave_lds() { return sizeof(T) * (64 * 64 + 64); }
// PF (round 6, late): the staging loads of L are all issued before the pivots' reciprocals and
// before any of them is used (the loop with a runtime trip count waited on each load in turn:
// ~n^2 / (128 NW) dependent global-load latencies); the values and their order are unchanged.
template <class T, bool TRANS, int NW = 4, bool PF = true>
__global__ __launch_bounds__(64 * NW) void trsv_wave(const TrsmDesc<T>* __restrict__ descs,
                                                     const int* __restrict__ t2d) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Ls = reinterpret_cast<T*>(smem_raw);  // 64 x 64, Ls[r + 64 q]
  T* rdg = Ls + 64 * 64;                    // 1 / l_qq
  const TrsmDesc<T> d = descs[t2d[blockIdx.x]];
  const int n = d.n, tid = threadIdx.x, lane = tid & 63;
  const T* L = d.L;
  const size_t ldl = d.ldl;
  constexpr int NT = 64 * NW, IT = PF ? (64 * 64 + NT - 1) / NT : 1;
  T lv[IT];
  if constexpr (PF) {
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int e = tid + NT * u, i = e % n, j = e / n;
      lv[u] = (e < n * n && i > j) ? L[i + (size_t)j * ldl] : T(0.0);
    }
  }
  if (tid < n) rdg[tid] = recip_fast(L[tid + (size_t)tid * ldl]);
  __syncthreads();
  // column q of L (rows > q) scaled by 1/l_qq; transposed: row q (columns < q), read as column
  if constexpr (PF) {
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int e = tid + NT * u, i = e % n, j = e / n;
      if (e < n * n && i > j) {
        const T v = lv[u] * rdg[TRANS ? i : j];
        if (TRANS) Ls[j + 64 * i] = v;
        else Ls[i + 64 * j] = v;
      }
    }
  } else {
    for (int e = tid; e < n * n; e += 64 * NW) {
      const int i = e % n, j = e / n;  // coalesced: i runs over the rows of L
      if (i > j) {
        const T v = L[i + (size_t)j * ldl] * rdg[TRANS ? i : j];
        if (TRANS) Ls[j + 64 * i] = v;
        else Ls[i + 64 * j] = v;
      }
    }
  }
  __syncthreads();
  const int c = (blockIdx.x - d.tile0) * NW + (tid >> 6);
  if (c >= d.nrhs) return;  // (whole waves; no barrier follows)
  T* B = d.B + (size_t)c * d.ldb;
  T v = T(0.0);
  if (lane < n) v = trsv_rhs(d, B, lane, c);
  if constexpr (PF) {
    // branch-free steps with the next step's coefficient read ahead of this step's arithmetic
    // (the exec-masked form waited on each LDS read); inactive lanes keep v by a select, so
    // every active lane runs the same operations in the same order
    if (!TRANS) {
      T c = Ls[lane];
      for (int q = 0; q + 1 < n; ++q) {
        T nx = c;
        if (q + 2 < n) nx = Ls[lane + 64 * (q + 1)];
        const T vq = readlane_t(v, q);
        const T w = trsv_fms(v, c, vq);
        v = sel(lane > q && lane < n, w, v);
        c = nx;
      }
    } else {
      T c = Ls[lane + 64 * (n - 1)];
      for (int q = n - 1; q > 0; --q) {
        T nx = c;
        if (q > 1) nx = Ls[lane + 64 * (q - 1)];
        const T vq = readlane_t(v, q);
        const T w = trsv_fms(v, c, vq);
        v = sel(lane < q, w, v);
        c = nx;
      }
    }
  } else if (!TRANS) {
    for (int q = 0; q + 1 < n; ++q) {
      const T vq = readlane_t(v, q);
      if (lane > q && lane < n) v = v - Ls[lane + 64 * q] * vq;
    }
  } else {
    for (int q = n - 1; q > 0; --q) {
      const T vq = readlane_t(v, q);
      if (lane < q) v = v - Ls[lane + 64 * q] * vq;
    }
  }
  if (lane < n) B[lane] = v * rdg[lane];
}

// trsv_wave128: the same for 64 < n <= 128 (the double-double S_j of config 4): lane r holds
// rows r and r + 64, and the scaled L passes through LDS in chunks of 32 steps (the whole matrix
// would not fit), staged by the workgroup between two barriers per chunk.
template <class T> constexpr size_t trsv_wave128_lds() { return sizeof(T) * (32 * 128 + 128); }
// PF (round 6, late): the next chunk's loads are issued into registers before the current
// chunk's steps, so they arrive under its chain (the staging loop waited on each load in turn);
// the values and their order are unchanged.
template <class T, bool TRANS, int NW = 4, bool PF = true>
__global__ __launch_bounds__(64 * NW) void trsv_wave128(const TrsmDesc<T>* __restrict__ descs,
                                                        const int* __restrict__ t2d) {
  constexpr int CH = 32;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Ls = reinterpret_cast<T*>(smem_raw);  // Ls[i + 128 qq]: row i at step q0 + qq
  T* rdg = Ls + CH * 128;
  const TrsmDesc<T> d = descs[t2d[blockIdx.x]];
  const int n = d.n, tid = threadIdx.x, lane = tid & 63;
  const T* L = d.L;
  const size_t ldl = d.ldl;
  for (int i = tid; i < n; i += 64 * NW) rdg[i] = recip_fast(L[i + (size_t)i * ldl]);
  const int c = (blockIdx.x - d.tile0) * NW + (tid >> 6);
  const bool act = c < d.nrhs;  // (wave-uniform; every wave stays for the barriers)
  T* B = d.B + (size_t)(act ? c : 0) * d.ldb;
  T v0 = T(0.0), v1 = T(0.0);
  if (act && lane < n) v0 = trsv_rhs(d, B, lane, c);
  if (act && lane + 64 < n) v1 = trsv_rhs(d, B, lane + 64, c);
  const int nch = (n + CH - 1) / CH;
  // (the register image of a chunk only where it fits beside the step loop's operands: not for
  // quad-double at 1024 threads, 128 VGPRs)
  constexpr bool SPF = PF && (sizeof(T) <= 16 || NW <= 4);
  constexpr int NT = 64 * NW, IT = SPF ? (CH * 128 + NT - 1) / NT : 1;
  T lv[IT];
  auto loadc = [&](int ci) {  // chunk ci's entries of L into registers
    const int q0 = (TRANS ? nch - 1 - ci : ci) * CH, qn = min(CH, n - q0);
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int e = tid + NT * u;
      int i, qq;
      if (TRANS) { qq = e % qn; i = e / qn; } else { i = e % n; qq = e / n; }
      const int q = q0 + qq;
      lv[u] = (e < qn * n && (TRANS ? i < q : i > q))
                  ? (TRANS ? L[q + (size_t)i * ldl] : L[i + (size_t)q * ldl]) : T(0.0);
    }
  };
  if constexpr (SPF) loadc(0);
  for (int ci = 0; ci < nch; ++ci) {
    const int q0 = (TRANS ? nch - 1 - ci : ci) * CH, qn = min(CH, n - q0);
    __syncthreads();  // the previous chunk is consumed (first pass: rdg is written)
    if constexpr (SPF) {
#pragma unroll
      for (int u = 0; u < IT; ++u) {
        const int e = tid + NT * u;
        int i, qq;
        if (TRANS) { qq = e % qn; i = e / qn; } else { i = e % n; qq = e / n; }
        const int q = q0 + qq;
        if (e < qn * n) Ls[i + 128 * qq] = (TRANS ? i < q : i > q) ? lv[u] * rdg[q] : T(0.0);
      }
    } else {
      for (int e = tid; e < qn * n; e += 64 * NW) {
        int i, qq;
        if (TRANS) { qq = e % qn; i = e / qn; } else { i = e % n; qq = e / n; }  // (coalesced)
        const int q = q0 + qq;
        T val = T(0.0);
        if (TRANS ? i < q : i > q) val = (TRANS ? L[q + (size_t)i * ldl] : L[i + (size_t)q * ldl]) * rdg[q];
        Ls[i + 128 * qq] = val;
      }
    }
    __syncthreads();
    if constexpr (SPF) {
      if (ci + 1 < nch) loadc(ci + 1);  // in flight under this chunk's chain
    }
    if (act && PF) {
      // both rows of the lane every step, branch-free (their two chains interleave), with the
      // next step's coefficients read ahead; inactive rows keep their value by a select
      int qq = TRANS ? qn - 1 : 0;
      T c0 = Ls[lane + 128 * qq], c1 = Ls[lane + 64 + 128 * qq];
      for (int u = 0; u < qn; ++u) {
        const int q = q0 + qq, qn1 = TRANS ? qq - 1 : qq + 1;
        T n0 = c0, n1 = c1;
        if (u + 1 < qn) {
          n0 = Ls[lane + 128 * qn1];
          n1 = Ls[lane + 64 + 128 * qn1];
        }
        const T vq = readlane_t(sel(q < 64, v0, v1), q & 63);
        T w0, w1;
        trsv_fms2(w0, v0, c0, w1, v1, c1, vq);
        v0 = sel(TRANS ? lane < q : (lane > q && lane < n), w0, v0);
        v1 = sel(TRANS ? lane + 64 < q : (lane + 64 > q && lane + 64 < n), w1, v1);
        c0 = n0;
        c1 = n1;
        qq = qn1;
      }
    } else if (act) {
      for (int u = 0; u < qn; ++u) {
        const int qq = TRANS ? qn - 1 - u : u, q = q0 + qq;
        const T vq = readlane_t(sel(q < 64, v0, v1), q & 63);
        if (TRANS ? lane < q : (lane > q && lane < n)) v0 = v0 - Ls[lane + 128 * qq] * vq;
        if (TRANS ? lane + 64 < q : (lane + 64 > q && lane + 64 < n)) v1 = v1 - Ls[lane + 64 + 128 * qq] * vq;
      }
    }
  }
  if (act) {
    if (lane < n) B[lane] = v0 * rdg[lane];
    if (lane + 64 < n) B[lane + 64] = v1 * rdg[lane + 64];
  }
}

// ------------------------------------------------------------------------------------------
// LU with partial pivoting in place, A[perm] = L U (L unit lower, U upper): approx_lu!
// (MPMP.jl:1436, 1501) on midpoints, and the factor of approx_inv! (MPMP.jl:781, 788).  The
// fallback of the Cholesky-based factorisations: taken once a Cholesky status
// word fires, then for the rest of the solve, as the reference switches spd_inv! off.
// One NT-thread workgroup per matrix, right-looking with NB-column panels.  The panel (rows
// k0..n-1) is factorised in LDS column by column; the pivot is the first row of maximal |a_ik|
// (approx_lu!'s and LAPACK's choice), found by a wave shuffle reduction and one LDS step.  The
// panel's interchanges are then applied to the other columns, U12 = L11^-1 A12 is solved into
// LDS and the trailing matrix is updated in global memory (L2-resident at these sizes).
// perm[k] is the original row at position k (the reference's 1-based perms minus one);
// info[b] = 0, or the 1-based column of a zero pivot (approx_lu!'s status 0).
// ------------------------------------------------------------------------------------------
template <class T> struct LuDesc {
  T* A;
  int* perm;
  int n, lda;
};
template <class T, int NB> constexpr size_t getrf_lds_bytes(int n) { return 2 * sizeof(T) * (size_t)NB * n; }

template <class T, int NB, int NT = 256>
__global__ __launch_bounds__(NT) void getrf_batched(const LuDesc<T>* __restrict__ descs,
                                                     int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int NWV = NT / 64;
  const LuDesc<T> d = descs[blockIdx.x];
  const int n = d.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const size_t lda = d.lda;
  T* A = d.A;
  T* P = reinterpret_cast<T*>(smem_raw);  // panel, P[q * pm + i]                 (NB x pm)
  T* U = P + (size_t)NB * n;                // U12 of the panel, U[c * NB + q]     (NB x (n - k1))
  __shared__ T wbest[NWV];
  __shared__ int wrow[NWV];
  __shared__ int piv[NB];
  __shared__ T rpv;
  __shared__ int fail;
  if (tid == 0) fail = 0;
  for (int i = tid; i < n; i += NT) d.perm[i] = i;
  __syncthreads();
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int nb = min(NB, n - k0), pm = n - k0, k1 = k0 + nb;
    for (int e = tid; e < nb * pm; e += NT) {
      const int i = e % pm, q = e / pm;
      P[q * pm + i] = A[(k0 + i) + (size_t)(k0 + q) * lda];
    }
    __syncthreads();
    for (int j = 0; j < nb; ++j) {
      // pivot: first row i >= j of maximal |P(i, j)| (ties to the smaller row)
      T best = T(-1.0);
      int brow = pm;
      for (int i = j + tid; i < pm; i += NT) {
        const T a = Num<T>::abs_(P[j * pm + i]);
        const bool gt = a > best;  // (component-wise selects: a multi-word value assigned under
        best = sel(gt, a, best);   // a branch stayed in scratch memory)
        brow = gt ? i : brow;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const T ob = shfl_xor_t(best, o);
        const int orow = __shfl_xor(brow, o);
        const bool tk = ob > best || (!(ob < best) && orow < brow);
        best = sel(tk, ob, best);
        brow = tk ? orow : brow;
      }
      if (lane == 0) { wbest[wv] = best; wrow[wv] = brow; }
      __syncthreads();
      if (tid == 0) {
        T b = wbest[0];
        int r = wrow[0];
        for (int w = 1; w < NWV; ++w) {
          const T bw = wbest[w];
          const bool tk = bw > b || (!(bw < b) && wrow[w] < r);
          b = sel(tk, bw, b);
          r = tk ? wrow[w] : r;
        }
        if (!(b > T(0.0))) {
          fail = k0 + j + 1;
        } else {
          piv[j] = k0 + r;
          if (r != j) {  // interchange rows j and r of the panel, and of perm
            for (int q = 0; q < nb; ++q) {
              const T t = P[q * pm + j];
              P[q * pm + j] = P[q * pm + r];
              P[q * pm + r] = t;
            }
            const int t = d.perm[k0 + j];
            d.perm[k0 + j] = d.perm[k0 + r];
            d.perm[k0 + r] = t;
          }
          rpv = recip_fast(P[j * pm + j]);
        }
      }
      __syncthreads();
      if (fail) break;
      const T rp = rpv;
      for (int i = j + 1 + tid; i < pm; i += NT) P[j * pm + i] = P[j * pm + i] * rp;
      __syncthreads();
      const int r = pm - j - 1;
      for (int e = tid; e < r * (nb - j - 1); e += NT) {
        const int i = j + 1 + e % r, c = j + 1 + e / r;
        P[c * pm + i] = P[c * pm + i] - P[j * pm + i] * P[c * pm + j];
      }
      __syncthreads();
    }
    if (fail) break;
    for (int e = tid; e < nb * pm; e += NT) {
      const int i = e % pm, q = e / pm;
      A[(k0 + i) + (size_t)(k0 + q) * lda] = P[q * pm + i];
    }
    // the panel's interchanges on the columns left and right of it (sequential per column)
    for (int c = tid; c < n - nb; c += NT) {
      const int col = c < k0 ? c : c + nb;
      for (int j = 0; j < nb; ++j) {
        const int r = piv[j];
        if (r != k0 + j) {
          T* a0 = A + (k0 + j) + (size_t)col * lda;
          T* a1 = A + r + (size_t)col * lda;
          const T t = *a0;
          *a0 = *a1;
          *a1 = t;
        }
      }
    }
    __syncthreads();
    const int nr = n - k1;
    if (nr <= 0) break;
    // U12 = L11^-1 A12 (unit lower), one column per thread (compile-time indexed: registers)
    for (int c = tid; c < nr; c += NT) {
      T x[NB];
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        if (q < nb) {
          T v = A[(k0 + q) + (size_t)(k1 + c) * lda];
#pragma unroll
          for (int p = 0; p < q; ++p) v = v - P[p * pm + q] * x[p];
          x[q] = v;
          U[c * NB + q] = v;
          A[(k0 + q) + (size_t)(k1 + c) * lda] = v;
        }
      }
    }
    __syncthreads();
    // trailing update A22 -= L21 U12
    for (int e = tid; e < nr * nr; e += NT) {
      const int i = e % nr, c = e / nr;
      T s = T(0.0);
      for (int q = 0; q < nb; ++q) s += P[q * pm + nb + i] * U[c * NB + q];
      T* a = A + (k1 + i) + (size_t)(k1 + c) * lda;
      *a = *a - s;
    }
    __syncthreads();
  }
  if (tid == 0) info[blockIdx.x] = fail;
}

// out = rows perm of in (out[i, c] = in[perm[i], c]): B_j[perms[j], :] (MPMP.jl:1463) and
// rhs[perm] (MPMP.jl:1752, 1764).  grid (chunks, problems).  ident: in is the identity
// (approx_inv!'s right-hand side P I).
template <class T> struct PermDesc {
  const T* in;
  T* out;
  const int* perm;
  int n, ncol, ldi, ldo;
};
template <class T>
__global__ __launch_bounds__(256) void perm_rows(const PermDesc<T>* __restrict__ descs, int ident) {
  const PermDesc<T> d = descs[blockIdx.y];
  const long long tot = (long long)d.n * d.ncol;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < tot; e += 256LL * gridDim.x) {
    const int i = (int)(e % d.n), c = (int)(e / d.n);
    const int pi = d.perm[i];
    if (ident) d.out[i + (size_t)c * d.ldo] = T(pi == c ? 1.0 : 0.0);
    else d.out[i + (size_t)c * d.ldo] = d.in[pi + (size_t)c * d.ldi];
  }
}

// ------------------------------------------------------------------------------------------
// Smallest eigenvalue of a symmetric matrix (destroys it): symmetrise, Householder
// tridiagonalisation (full symmetric storage, one workgroup per matrix), then Sturm-count
// multisection by one wave (64 shifts per round).  Replaces the complex QR eigen-solver of
// compute_step_length (MPMP.jl:1857-1870), which returns the same spectrum for the
// (mathematically symmetric) L^-1 dM L^-T.
// ------------------------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ int sturm_count(const T* dg, const T* e2, int n, T sigma) {
  int cnt = 0;
  T q = dg[0] - sigma;
  if (q < T(0.0)) ++cnt;
  for (int i = 1; i < n; ++i) {
    if (q == T(0.0)) q = T(1e-300);
    q = dg[i] - sigma - e2[i - 1] / q;
    if (q < T(0.0)) ++cnt;
  }
  return cnt;
}

template <class T>
__global__ __launch_bounds__(256) void eigmin_batched(const MatDesc<T>* __restrict__ descs,
                                                      T* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const MatDesc<T> d = descs[blockIdx.x];
  const int n = d.n, lda = d.lda, tid = threadIdx.x;
  T* v = reinterpret_cast<T*>(smem_raw);  // n
  T* p = v + n;                            // n
  T* dg = p + n;                           // n   diagonal
  T* e2 = dg + n;                          // n   squared off-diagonal
  T* red = e2 + n;                         // blockDim.x
  T* A = d.A;
  // symmetrise: A = (A + A^T) / 2
  for (int e = tid; e < n * n; e += blockDim.x) {
    const int i = e % n, j = e / n;
    if (i > j) {
      const T s = (A[i + (size_t)j * lda] + A[j + (size_t)i * lda]) * T(0.5);
      A[i + (size_t)j * lda] = s;
      A[j + (size_t)i * lda] = s;
    }
  }
  __syncthreads();
  for (int k = 0; k + 2 < n; ++k) {
    const int m = n - k - 1;
    T* Ak = A + (k + 1) + (size_t)(k + 1) * lda;  // trailing m x m
    for (int i = tid; i < m; i += blockDim.x) v[i] = A[(k + 1 + i) + (size_t)k * lda];
    __syncthreads();
    T s = T(0.0);
    for (int i = tid; i < m; i += blockDim.x) s += v[i] * v[i];
    s = block_sum(s, red);
    const T x0 = v[0];
    const T nrm = Num<T>::sqrt_(s);
    const T alpha = sel(x0 > T(0.0), -nrm, nrm);
    if (tid == 0) dg[k] = A[k + (size_t)k * lda];
    T tail = s - x0 * x0;
    if (!(tail > T(0.0))) {  // already tridiagonal in this column
      if (tid == 0) e2[k] = x0 * x0;
      __syncthreads();
      continue;
    }
    if (tid == 0) {
      e2[k] = alpha * alpha;
      v[0] = x0 - alpha;
    }
    __syncthreads();
    // v^T v = tail + (x0 - alpha)^2
    const T v0 = x0 - alpha;
    const T beta = T(2.0) / (tail + v0 * v0);
    // p = beta A' v
    for (int i = tid; i < m; i += blockDim.x) {
      T acc = T(0.0);
      for (int j = 0; j < m; ++j) acc += Ak[i + (size_t)j * lda] * v[j];
      p[i] = acc * beta;
    }
    __syncthreads();
    T pv = T(0.0);
    for (int i = tid; i < m; i += blockDim.x) pv += p[i] * v[i];
    pv = block_sum(pv, red);
    const T Kc = beta * pv * T(0.5);
    for (int i = tid; i < m; i += blockDim.x) p[i] = p[i] - Kc * v[i];
    __syncthreads();
    for (int e = tid; e < m * m; e += blockDim.x) {
      const int i = e % m, j = e / m;
      Ak[i + (size_t)j * lda] = Ak[i + (size_t)j * lda] - (v[i] * p[j] + p[i] * v[j]);
    }
    __syncthreads();
  }
  if (tid == 0) {
    if (n >= 2) {
      dg[n - 2] = A[(n - 2) + (size_t)(n - 2) * lda];
      dg[n - 1] = A[(n - 1) + (size_t)(n - 1) * lda];
      const T e = A[(n - 1) + (size_t)(n - 2) * lda];
      e2[n - 2] = e * e;
    } else {
      dg[0] = A[0];
    }
  }
  __syncthreads();
  if (tid < 64) {
    // Gershgorin interval
    T lo = T(0.0), hi = T(0.0);
    if (tid == 0) {
      for (int i = 0; i < n; ++i) {
        T r = T(0.0);
        if (i > 0) r += Num<T>::sqrt_(e2[i - 1]);
        if (i + 1 < n) r += Num<T>::sqrt_(e2[i]);
        const T a = dg[i] - r, b = dg[i] + r;
        if (i == 0 || a < lo) lo = a;
        if (i == 0 || b > hi) hi = b;
      }
      red[0] = lo;
      red[1] = hi;
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    lo = red[0];
    hi = red[1];
    const T span = hi - lo;
    lo = lo - span * T(1e-3) - T(1e-300);
    hi = hi + span * T(1e-3) + T(1e-300);
    const int rounds = Num<T>::BITS / 6 + 3;
    for (int it = 0; it < rounds; ++it) {
      const T width = hi - lo;
      const T sigma = lo + width * T((double)(tid + 1) / 65.0);
      const int c = sturm_count(dg, e2, n, sigma);
      const unsigned long long mask = __ballot(c >= 1);
      T nlo = lo, nhi = hi;
      if (mask == 0ull) {
        nlo = lo + width * T(64.0 / 65.0);
      } else {
        const int f = __ffsll((long long)mask) - 1;
        nhi = lo + width * T((double)(f + 1) / 65.0);
        if (f > 0) nlo = lo + width * T((double)f / 65.0);
      }
      lo = nlo;
      hi = nhi;
    }
    if (tid == 0) out[blockIdx.x] = (lo + hi) * T(0.5);
  }
}

// ------------------------------------------------------------------------------------------
// Schur complement assembly from the pairings (MPMP.jl:1335-1409).  One thread per upper
// entry (ver <= hor) of one cluster; sums the l blocks and rank pairs in the reference's order
// and writes both triangles.
//   BX_b, BY_b:  (m K) x (m K) pairings of block b (column-major, ld m K)
//   S_c: D x D.   tuple t(r,s,k) = k + (s + r(r+1)/2) N
// ------------------------------------------------------------------------------------------
struct SchurClusterDesc {
  int m, N, D;
  int blk0, nblk;    // local blocks of this cluster
  int pair0;         // first upper-pair index of this cluster in the launch
  long long S_off;   // offset of S_c in the S arena
};
struct SchurBlockDesc {
  long long bx_off;   // offset of BX_b / BY_b in the pairing arenas
  int K;              // vectors of this block
  int rs_off;         // offset of rank_sums of this block in the int arena (N + 1 entries)
  int lam_off;        // offset of lambda_b
  int pad;
};

template <class T>
__global__ __launch_bounds__(256) void schur_assemble(const SchurClusterDesc* __restrict__ cd,
                                                      int ncl, const SchurBlockDesc* __restrict__ bd,
                                                      const int* __restrict__ rank_sums,
                                                      const T* __restrict__ lam,
                                                      const T* __restrict__ BX,
                                                      const T* __restrict__ BY,
                                                      T* __restrict__ S, long long npairs,
                                                      int upper = 0) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= npairs) return;
  int lo = 0, hi = ncl - 1;  // find the cluster: last c with pair0 <= g
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cd[mid].pair0 <= g) lo = mid; else hi = mid - 1;
  }
  const SchurClusterDesc c = cd[lo];
  long long u = g - c.pair0;  // index into the upper triangle, column by column
  // hor = column h, ver = row v <= h :  u = h(h+1)/2 + v
  int h = (int)((sqrt(8.0 * (double)u + 1.0) - 1.0) * 0.5);
  while ((long long)h * (h + 1) / 2 > u) --h;
  while ((long long)(h + 1) * (h + 2) / 2 <= u) ++h;
  const int v = (int)(u - (long long)h * (h + 1) / 2);
  const int N = c.N;
  // decode tuples: hor = (r1, s1, k1), ver = (r2, s2, k2)
  const int k1 = h % N, rs1 = h / N, k2 = v % N, rs2 = v / N;
  int r1 = 0;
  while ((r1 + 1) * (r1 + 2) / 2 <= rs1) ++r1;
  const int s1 = rs1 - r1 * (r1 + 1) / 2;
  int r2 = 0;
  while ((r2 + 1) * (r2 + 2) / 2 <= rs2) ++r2;
  const int s2 = rs2 - r2 * (r2 + 1) / 2;
  T tot = T(0.0);
  for (int b = c.blk0; b < c.blk0 + c.nblk; ++b) {
    const SchurBlockDesc B = bd[b];
    const int K = B.K, ld = c.m * K;
    const int* rsum = rank_sums + B.rs_off;
    const T* bx = BX + B.bx_off;
    const T* by = BY + B.bx_off;
    const T* lb = lam + B.lam_off;
    for (int p1 = rsum[k1]; p1 < rsum[k1 + 1]; ++p1) {
      for (int p2 = rsum[k2]; p2 < rsum[k2 + 1]; ++p2) {
        if (upper) {  // m = 1 with BX, BY symmetric and only their upper triangles formed
          const int lo = min(p1, p2), hi = max(p1, p2);
          tot += bx[lo + (size_t)hi * ld] * by[lo + (size_t)hi * ld] * lb[p1] * lb[p2];
          continue;
        }
        const int r1s = p1 + K * r1, s1s = p1 + K * s1, r2s = p2 + K * r2, s2s = p2 + K * s2;
        T t = bx[s1s + (size_t)r2s * ld] * by[s2s + (size_t)r1s * ld];
        t += bx[r1s + (size_t)r2s * ld] * by[s2s + (size_t)s1s * ld];
        t += bx[s1s + (size_t)s2s * ld] * by[r2s + (size_t)r1s * ld];
        t += bx[r1s + (size_t)s2s * ld] * by[r2s + (size_t)s1s * ld];
        tot += t * lb[p1] * lb[p2] * T(0.25);
      }
    }
  }
  T* Sc = S + c.S_off;
  Sc[v + (size_t)h * c.D] = tot;
  Sc[h + (size_t)v * c.D] = tot;
}

// ------------------------------------------------------------------------------------------
// Fused Schur pairing for blocks with m = 1 (fp64 matrix cores).  With V the delta x K vectors of
// block b and the transposed products TXt = V^T X^-1, TYt = V^T Y (K x delta, ld K), one 64x64
// upper tile (I <= J) of
//     G[p, q] = lambda_p lambda_q (V^T X^-1 V)[p, q] (V^T Y V)[q, p]
// per 256-thread workgroup: both contractions over delta share the staged V^T slab (three
// LDS slabs, k-major, pipelined like gemm_f64_lds), the Hadamard product and the lambda scaling
// are applied in registers and G is written to both triangles.  Diagonal tiles also write
// AY[p] = (V^T Y V)[p, p].  This is MPMP.jl:1291-1330 + 1373-1398 at m = 1 (the four pairing
// terms coincide) without materialising the K x K pairings BX, BY.
// ------------------------------------------------------------------------------------------
struct PairTileDesc {
  const double* Vt;   // K x delta, ld K  (V transposed, uploaded once)
  const double* TXt;  // K x delta, ld K
  const double* TYt;
  const double* lam;  // K
  double* G;          // K x K (ld ldG): S itself when L = 1 and every rank is 1
  double* AY;         // K
  int K, del, ldG, tile0;
  // grp = 2 (round 6): L = 1 and every sample of rank 2, the vectors ordered (k, rho): G is S
  // itself (ld ldG = D) and each 2 x 2 group of the tile is summed in the epilogue,
  // S[a, b] = sum_{rho1, rho2} G[2a + rho1, 2b + rho2] (MPMP.jl:1373-1398 at m = 1) -- no K x K
  // intermediate and no schur_gsum launch.  grp = 1: G written per (p, q) as before.
  int grp, pad;
};

template <int BK = 16>
// stamp[0] / stamp[1]: the earliest workgroup start / latest end of the launch on the 100 MHz
// clock (SCHUR-stage timing)
__global__ __launch_bounds__(256) void schur_pairs_f64(const PairTileDesc* __restrict__ descs,
                                                       const TileRef* __restrict__ t2d,
                                                       unsigned long long* stamp = nullptr) {
  if (stamp && threadIdx.x == 0) atomicMin(stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  using namespace lds_gemm;
  using SLB = Slab<BK>;
  constexpr int PER = SLB::PER, SL = BK * LSM;
  __shared__ double smem[3 * SL > 64 * TP + 128 ? 3 * SL : 64 * TP + 128];
  double* As = smem;
  double* Xs = smem + SL;
  double* Ys = smem + 2 * SL;
  const TileRef tr = t2d[blockIdx.x];
  const PairTileDesc d = descs[tr.p];
  const int u = tr.t;
  int J = 0;
  while ((J + 1) * (J + 2) / 2 <= u) ++J;
  const int I = u - J * (J + 1) / 2;
  const int p0 = I * 64, q0 = J * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1, lr = lane & 15, lk = lane >> 4;
  const int K = d.K, D = d.del;
  const bool diag_skip = I == J && wm > wn;  // wave-uniform
  double ra[PER], rx[PER], ry[PER];
  d4 ax[2][2], ay[2][2];
  // lambda of the tile's rows and columns (read before the K loop, used in the epilogue)
  const double lamv = tid < 128 ? d.lam[min((tid < 64 ? p0 : q0) + (tid & 63), K - 1)] : 0.0;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) ax[a][b] = ay[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  SLB::template load<false>(ra, d.Vt, K, p0, K, 0, D, tid);
  SLB::template load<false>(rx, d.TXt, K, q0, K, 0, D, tid);
  SLB::template load<false>(ry, d.TYt, K, q0, K, 0, D, tid);
  SLB::template store<false>(ra, As, tid, 0, D);
  SLB::template store<false>(rx, Xs, tid, 0, D);
  SLB::template store<false>(ry, Ys, tid, 0, D);
  __syncthreads();
  for (int k0 = 0; k0 < D; k0 += BK) {
    const bool more = k0 + BK < D;
#ifndef CLRSDP_PAIRS_NO_LOAD
    if (more) {
      SLB::template load<false>(ra, d.Vt, K, p0, K, k0 + BK, D, tid);
      SLB::template load<false>(rx, d.TXt, K, q0, K, k0 + BK, D, tid);
      SLB::template load<false>(ry, d.TYt, K, q0, K, k0 + BK, D, tid);
    }
#endif
    // a diagonal tile (I == J) stores only p <= q: the wave of rows 32..63 x columns 0..31 lies
    // strictly below the diagonal and leaves its SIMD to the other workgroups on the CU
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      if (diag_skip) break;
      const int kr = (kk + lk) * LSM;
      const double a0 = As[kr + wm * 32 + lr], a1 = As[kr + wm * 32 + 16 + lr];
      const double x0 = Xs[kr + wn * 32 + lr], x1 = Xs[kr + wn * 32 + 16 + lr];
      const double y0 = Ys[kr + wn * 32 + lr], y1 = Ys[kr + wn * 32 + 16 + lr];
      ax[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, x0, ax[0][0], 0, 0, 0);
      ay[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, y0, ay[0][0], 0, 0, 0);
      ax[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, x1, ax[0][1], 0, 0, 0);
      ay[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, y1, ay[0][1], 0, 0, 0);
      ax[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, x0, ax[1][0], 0, 0, 0);
      ay[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, y0, ay[1][0], 0, 0, 0);
      ax[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, x1, ax[1][1], 0, 0, 0);
      ay[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, y1, ay[1][1], 0, 0, 0);
    }
    if (!more) break;
    __syncthreads();
    SLB::template store<false>(ra, As, tid, k0 + BK, D);
    SLB::template store<false>(rx, Xs, tid, k0 + BK, D);
    SLB::template store<false>(ry, Ys, tid, k0 + BK, D);
    __syncthreads();
  }
  __syncthreads();  // LDS slabs -> output tile T[p][q] = (V^T X^-1 V)(V^T Y V), lambdas at 64*TP
  double* Tt = smem;
  double* lamS = smem + 64 * TP;
  if (tid < 128) lamS[tid] = lamv;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pl = acc_row(wm, mi, lk, r), ql = acc_col(wn, ni, lr);
        const double yv = ay[mi][ni][r];
        Tt[pl * TP + ql] = ax[mi][ni][r] * yv;
        if (I == J && pl == ql && p0 + pl < K) d.AY[p0 + pl] = yv;
      }
  __syncthreads();
  if (d.grp == 2) {
    // the 32 x 32 tile of S at (p0 / 2, q0 / 2): S[a, b] = sum of the 2 x 2 group of
    // lambda_p lambda_q T[p][q]; a diagonal tile (I == J) takes a <= b and mirrors it (the
    // quarter its skipped wave left holds a > b only).  Two passes, each with consecutive threads
    // on consecutive rows of what they store: S[a, b] (thread -> a) and S[b, a] (thread -> b)
    const int D = d.K >> 1, a0 = p0 >> 1, b0 = q0 >> 1;
    auto gsum = [&](int al, int bl) {
      const int p = 2 * al, q = 2 * bl;
      return (lamS[p] * lamS[64 + q] * Tt[p * TP + q] + lamS[p] * lamS[64 + q + 1] * Tt[p * TP + q + 1]) +
             (lamS[p + 1] * lamS[64 + q] * Tt[(p + 1) * TP + q] +
              lamS[p + 1] * lamS[64 + q + 1] * Tt[(p + 1) * TP + q + 1]);
    };
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int al = tid & 31, bl = (tid >> 5) + 8 * c;
      const int a = a0 + al, bb = b0 + bl;
      if (a < D && bb < D && (I < J || al <= bl)) d.G[a + (size_t)bb * d.ldG] = gsum(al, bl);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int bl = tid & 31, al = (tid >> 5) + 8 * c;
      const int a = a0 + al, bb = b0 + bl;
      if (a < D && bb < D && (I < J || al < bl)) d.G[bb + (size_t)a * d.ldG] = gsum(al, bl);
    }
    if (stamp) {
      __syncthreads();
      if (threadIdx.x == 0) atomicMax(stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    return;
  }
  // G[p, q] for p <= q: lane -> p, wave -> 16 columns q;  mirror G[q, p] for p < q: lane -> q
  {
    const int pl = lane, p = p0 + pl;
#ifndef CLRSDP_PAIRS_NO_STORE
    if (p < K) {
#else
    if (p == -7) {
#endif
      const double lp = lamS[pl];
#pragma unroll 4
      for (int c = 0; c < 16; ++c) {
        const int ql = w * 16 + c, q = q0 + ql;
        if (q < K && (I < J || p <= q)) d.G[p + (size_t)q * d.ldG] = lp * lamS[64 + ql] * Tt[pl * TP + ql];
      }
    }
  }
  {
    const int ql = lane, q = q0 + ql;
#ifndef CLRSDP_PAIRS_NO_STORE
    if (q < K) {
#else
    if (q == -7) {
#endif
      const double lq = lamS[64 + ql];
#pragma unroll 4
      for (int c = 0; c < 16; ++c) {
        const int pl = w * 16 + c, p = p0 + pl;
        if (p < K && (I < J || p < q)) d.G[q + (size_t)p * d.ldG] = lamS[pl] * lq * Tt[pl * TP + ql];
      }
    }
  }
  if (stamp) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

// ------------------------------------------------------------------------------------------
// schur_fused_f64: the Schur pairing of one block (m = 1, delta <= 128) with V^T X^-1 formed on
// chip, one 512-thread workgroup per 64-row block `a` of the K x K result.  It replaces the
// V^T X^-1 GEMM and schur_pairs_f64: the K x delta product never goes to HBM.
//   phase 1: C' = X^-1 V_a (delta x 64, LDS-staged MFMA GEMM).  Wave w = (nt = w & 3, h = w >> 2)
//            keeps the 16x16 tiles (mt, nt), mt = 4h..4h+3, in its accumulators; register r of
//            lane l of tile (mt, nt) is TXt[a-row 16nt + (l & 15)][k = 16mt + 4r + (l >> 4)],
//            i.e. exactly the A-operand fragment of k-chunk 4mt + r of TXt_a V_b.  The two
//            K halves are swapped once through LDS, so every wave holds all 32 chunks of its row
//            tile in registers.
//   phase 2: for each column block b of this workgroup's share of the upper triangle (b = a,
//            a+1, .., a + floor(T/2) mod T, the pair {a, a+T/2} once when T is even: 2-3 tiles
//            for T = 4), P_X = TXt_a V_b and P_Y = TYt_a V_b.  TYt_a (V^T Y, computed ahead on
//            the side stream) and V_b sit in LDS in MFMA-fragment order (one 64-lane row per
//            fragment: conflict-free, and few enough registers that the fragment reads run
//            ahead of the MFMAs); the next V_b is loaded into registers before the MFMAs of the
//            current one.  G[p, q] = lambda_p lambda_q P_X P_Y is staged in LDS (XOR-swizzled
//            64 x 64) and written to (p, q) and to its mirror (q, p) as whole 64-row column
//            segments; a diagonal tile takes its p <= q half for both, and writes AY[p] =
//            P_Y[p, p].  With full = false (G is S itself and every reader of it takes the lower
//            triangle: the fp64 Cholesky path) only the tile below the diagonal and the lower
//            half of a diagonal tile are written, K(K+1)/2-ish instead of K^2 stores.
// MPMP.jl:1291-1330 + 1373-1398 at m = 1, as schur_pairs_f64.
// ------------------------------------------------------------------------------------------
struct FusedPairDesc {
  const double* Vt;    // K x delta, ld K
  const double* Xinv;  // delta x delta, ld ldx
  const double* TYt;   // K x delta, ld K (YV = false)
  const double* Y;     // delta x delta, ld ldy (YV = true: TYt_a = V_a^T Y formed on chip)
  const double* lam;   // K
  double* G;           // K x K, ld ldG
  double* AY;          // K
  int K, del, ldG, ldx, ldy;
  int grp, pad;        // grp = 2: S itself, the 2 x 2 rank groups summed (PairTileDesc::grp)
};
namespace schur_fused {
constexpr int BK = 32;                  // phase-1 k-slab
constexpr int LA = 144, LBV = 80;       // phase-1 slab pitches (doubles): 32 banks apart per k-row
constexpr int FR = 32 * 4 * 64;         // fragment-ordered 128 x 64 operand (TYt_a or V_b)
constexpr int YR = 0, VR = FR, SR = 2 * FR, END = 2 * FR + 64 * 64;
static_assert(BK * LA + BK * LBV <= FR && BK * LA + BK * LBV <= END - VR,
              "phase-1 images fit in the TYt_a region and in the V_b + staging regions");
constexpr int P1Y = 2 * BK * LA + BK * LBV;  // YV: one image of the X^-1, Y and V_a slabs
static_assert(P1Y <= END, "YV phase-1 image fits");
constexpr size_t LDS = sizeof(double) * END;  // 160 KB
__device__ __forceinline__ int st_idx(int row, int col) { return row * 64 + (col ^ (row & 31)); }
}  // namespace schur_fused

// DBG (timing experiments only): 1 = no phase-2 MFMAs, 2 = no phase-1 MFMAs.
// YV: phase 1 also forms TYt_a^T = Y V_a (sharing the V_a slab; one single-buffered image of
// the three slabs), whose accumulators are written straight into the fragment-ordered TYt_a
// region -- no V^T Y GEMM and no K x delta round trip through HBM for it either.
// GRP2 (every descriptor grp = 2): the rank-2 group-sum epilogue.  A template parameter, not a
// branch on d.grp: the branch made the rank-1 (C3) instance spill 92 B/lane at 256 VGPRs
// (63.7 against 57.3 us per launch, round 6).
// ONE (round 6, small batches): each workgroup forms TXt_a (and TYt_a) and then ONE column tile
// s of row block a's share (tile ref t = a + 64 s) instead of all nb of them, so a batch with
// few row blocks (C2: 16 clusters x 4 = 64 workgroups, the 8-cluster shard: 32) spreads over
// 2.5x the workgroups at the price of recomputing phase 1 per tile.
// D64 (every block delta <= 64: C2): rows 64..127 of C' and k-chunks 16..31 of phase 2 are zero,
// so the waves of the upper half (h = 1) issue no phase-1 MFMAs (they share their SIMDs with the
// h = 0 waves of the same nt) and phase 2 runs 16 chunks instead of 32: half the MFMAs of both
// phases, the same sums over the nonzero terms in the same order.
template <int DBG = 0, bool YV = false, bool GRP2 = false, bool ONE = false, bool D64 = false>
__global__ __launch_bounds__(512) void schur_fused_f64(const FusedPairDesc* __restrict__ descs,
                                                       const TileRef* __restrict__ t2d,
                                                       unsigned long long* stamp = nullptr,
                                                       bool full = true) {
  using namespace schur_fused;
  if (stamp && threadIdx.x == 0) atomicMin(stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  extern __shared__ __attribute__((aligned(16))) double sm_fused[];
  double* Yf = sm_fused + YR;  // TYt_a fragments: (row tile t, chunk c, lane l) at (t*32 + c)*64 + l
  double* Vf = sm_fused + VR;  // V_b fragments: (chunk c, column tile bt, lane l) at (c*4 + bt)*64 + l
  double* St = sm_fused + SR;  // output staging, st_idx
  // phase-1 slabs, double-buffered: image 0 over the TYt_a region, image 1 over V_b + staging
  auto P1 = [&](int img) { return sm_fused + (img ? VR : YR); };
  const TileRef tr = t2d[blockIdx.x];
  const FusedPairDesc d = descs[tr.p];
  const int a = ONE ? tr.t % 64 : tr.t, K = d.K, D = d.del;
  const int T = (K + 63) / 64, a0 = 64 * a;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nt = w & 3, h = w >> 2, lr = lane & 15, lk = lane >> 4;
  const int nb = (T % 2 == 0 && a >= T / 2) ? T / 2 : T / 2 + 1;  // tiles of this row block
  const int s_lo = ONE ? tr.t / 64 : 0, s_hi = ONE ? s_lo + 1 : nb;  // the ones of this workgroup
  // ---------------- phase 1: C' = X^-1 V_a (and Y V_a)
  d4 c1[4], c1y[YV ? 4 : 1];
#pragma unroll
  for (int q = 0; q < 4; ++q) c1[q] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < (YV ? 4 : 1); ++q) c1y[q] = d4{0.0, 0.0, 0.0, 0.0};
  double ra[8], rb[4], ryy[YV ? 8 : 1];
  auto load1 = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {  // X^-1 (i, k'): i = e % 128 contiguous
      const int e = tid + 512 * q, i = e & 127, k = k0 + (e >> 7);
      ra[q] = gload(d.Xinv + min(i, D - 1) + (size_t)min(k, D - 1) * d.ldx);
      if constexpr (YV) ryy[q] = gload(d.Y + min(i, D - 1) + (size_t)min(k, D - 1) * d.ldy);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // V_a (k', j) = Vt[a0 + j + k' K]
      const int e = tid + 512 * q, j = e & 63, k = k0 + (e >> 6);
      rb[q] = gload(d.Vt + min(a0 + j, K - 1) + (size_t)min(k, D - 1) * K);
    }
  };
  // image layout: X^-1 slab [k][LA], (YV: Y slab [k][LA]), V_a slab [k][LBV]
  constexpr int VOFF = (YV ? 2 : 1) * BK * LA;
  auto store1 = [&](double* S, int k0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 512 * q, i = e & 127, k = e >> 7;
      S[k * LA + i] = (i < D && k0 + k < D) ? ra[q] : 0.0;
      if constexpr (YV) S[BK * LA + k * LA + i] = (i < D && k0 + k < D) ? ryy[q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 512 * q, j = e & 63, k = e >> 6;
      S[VOFF + k * LBV + j] = k0 + k < D ? rb[q] : 0.0;
    }
  };
  // V_b element (k, j) = Vt[b0 + j + k K]: thread element e = tid + 512 q is (k = e >> 6,
  // j = e & 63), kept at Vf[((k >> 2) * 4 + (j >> 4)) * 64 + (k & 3) * 16 + (j & 15)]
  double rv[16];
  auto loadv = [&](int b) {
    const int b0 = 64 * b;
    const double* src = d.Vt + min(b0 + lane, K - 1);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = w + 8 * q;
      rv[q] = gload(src + (size_t)min(k, D - 1) * K);
    }
  };
  auto storev = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = w + 8 * q;
      Vf[((k >> 2) * 4 + (lane >> 4)) * 64 + (k & 3) * 16 + (lane & 15)] = k < D ? rv[q] : 0.0;
    }
  };
  // TYt_a element (row i = 16t + (l & 15), k = 4c + (l >> 4)) for (t, c, l) = (e >> 11,
  // (e >> 6) & 31, e & 63), kept at Yf[e]
  double ry[16];
  auto loady = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = tid + 512 * q, l = e & 63, c = (e >> 6) & 31, t = e >> 11;
      const int p = min(a0 + 16 * t + (l & 15), K - 1), k = 4 * c + (l >> 4);
      ry[q] = gload(d.TYt + p + (size_t)min(k, D - 1) * K);
    }
  };
  auto storey = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = tid + 512 * q, l = e & 63, c = (e >> 6) & 31;
      Yf[e] = 4 * c + (l >> 4) < D ? ry[q] : 0.0;
    }
  };
  load1(0);
  store1(P1(0), 0);
  __syncthreads();
  int img = 0;
  for (int k0 = 0; k0 < D; k0 += BK) {
    const bool more = k0 + BK < D;
    if (more) load1(k0 + BK);
    const double* S = P1(img);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      if (DBG == 2 || (D64 && h == 1)) break;
      const double bf = S[VOFF + (kk + lk) * LBV + 16 * nt + lr];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double af = S[(kk + lk) * LA + 16 * (4 * h + q) + lr];
        c1[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf, c1[q], 0, 0, 0);
        if constexpr (YV) {
          const double ay = S[BK * LA + (kk + lk) * LA + 16 * (4 * h + q) + lr];
          c1y[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(ay, bf, c1y[q], 0, 0, 0);
        }
      }
    }
    if (!more) break;
    if constexpr (YV) {  // one image: wait for every wave before overwriting it
      __syncthreads();
      store1(P1(0), k0 + BK);
    } else {
      img ^= 1;
      store1(P1(img), k0 + BK);  // (the other image was last read before the previous barrier)
    }
    __syncthreads();
  }
  // phase 2's first operands load during the swap of the K halves (through the V_b region)
  if constexpr (!YV) loady();
  loadv((a + s_lo) % T);
  __syncthreads();  // every wave is done with the last phase-1 image
  if constexpr (YV) {  // TYt_a fragments straight from the accumulators (tile (mt, nt), mt = 4h + q)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) Yf[(nt * 32 + 4 * (4 * h + q) + r) * 64 + lane] = c1y[q][r];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) Vf[((w * 4 + q) * 4 + r) * 64 + lane] = c1[q][r];
  double lp[4];  // lambda of this lane's four rows
#pragma unroll
  for (int r = 0; r < 4; ++r) lp[r] = d.lam[min(a0 + 16 * nt + 4 * r + lk, K - 1)];
  __syncthreads();
  double tf[32];  // TXt_a fragment of k-chunk c = 4 mt + r
  const int wp = w ^ 4;  // the wave with the other K half of this row tile
#pragma unroll
  for (int mt = 0; mt < 8; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      tf[4 * mt + r] = (mt >> 2) == h ? c1[mt & 3][r] : Vf[((wp * 4 + (mt & 3)) * 4 + r) * 64 + lane];
  __syncthreads();
  if constexpr (!YV) storey();
  storev();
  __syncthreads();
  const double* yrow = Yf + nt * 32 * 64 + lane;     // chunk c at yrow[64 c]
  const double* vrow = Vf + 2 * h * 64 + lane;       // chunk c, tile 2h + u at vrow[256 c + 64 u]
  for (int s = s_lo; s < s_hi; ++s) {
    const int b = (a + s) % T, b0 = 64 * b;
    const bool diag = s == 0;
    if (s + 1 < s_hi) loadv((a + s + 1) % T);
    // ---------------- phase 2: P_X, P_Y for the column tiles bt = 2h, 2h+1
    d4 px[2], py[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) px[u] = py[u] = d4{0.0, 0.0, 0.0, 0.0};
    // fragment reads two chunks ahead of their MFMAs (a read an MFMA waits on exposes its
    // latency; the scheduling barriers keep the compiler from regrouping them)
    constexpr int PD = 2, NCH = D64 ? 16 : 32;
    double fy[PD + 1], f0[PD + 1], f1[PD + 1];
#pragma unroll
    for (int c = 0; c < PD; ++c) {
      fy[c] = yrow[64 * c];
      f0[c] = vrow[256 * c];
      f1[c] = vrow[256 * c + 64];
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (DBG == 1) break;
      if (c + PD < NCH) {
        fy[(c + PD) % (PD + 1)] = yrow[64 * (c + PD)];
        f0[(c + PD) % (PD + 1)] = vrow[256 * (c + PD)];
        f1[(c + PD) % (PD + 1)] = vrow[256 * (c + PD) + 64];
      }
      const int q = c % (PD + 1);
      px[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(tf[c], f0[q], px[0], 0, 0, 0);
      py[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fy[q], f0[q], py[0], 0, 0, 0);
      px[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(tf[c], f1[q], px[1], 0, 0, 0);
      py[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fy[q], f1[q], py[1], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // element (p, q) of register r: p = a0 + 16 nt + 4r + lk, q = b0 + 16 bt + lr
    double g[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ql = 16 * (2 * h + u) + lr, q = b0 + ql;
      const double lq = d.lam[min(q, K - 1)];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pl = 16 * nt + 4 * r + lk, p = a0 + pl;
        const double yv = py[u][r];
        g[u][r] = lp[r] * lq * (px[u][r] * yv);
        if (diag && pl == ql && p < K) d.AY[p] = yv;
      }
    }
    __syncthreads();  // every wave is done with this V_b and with the previous staging tile
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) St[st_idx(16 * nt + 4 * r + lk, 16 * (2 * h + u) + lr)] = g[u][r];
    if (s + 1 < s_hi) storev();
    __syncthreads();
    // (p, q) and its mirror (q, p) from the staging tile as 64-row column segments (lower
    // triangle only unless full: the tile whose row block is the larger one, and p >= q of a
    // diagonal tile)
    if constexpr (GRP2) {
      // rank 2: the 32 x 32 tile of S at (a0 / 2, b0 / 2), each entry the sum of its 2 x 2 group
      // of the staged tile; the same triangle rules as below, in S's coordinates
      const int D = K >> 1, sa0 = a0 >> 1, sb0 = b0 >> 1;
      const bool w_pq = full || a > b, w_qp = full || b > a;
      auto gs = [&](int al, int bl) {
        const int p = 2 * al, q = 2 * bl;
        return (St[st_idx(p, q)] + St[st_idx(p, q + 1)]) + (St[st_idx(p + 1, q)] + St[st_idx(p + 1, q + 1)]);
      };
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int al = tid & 31, bl = (tid >> 5) + 16 * c;
        if (sa0 + al < D && sb0 + bl < D && (diag ? full && al <= bl : w_pq))
          d.G[(sa0 + al) + (size_t)(sb0 + bl) * d.ldG] = gs(al, bl);
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int bl = tid & 31, al = (tid >> 5) + 16 * c;
        if (sb0 + bl < D && sa0 + al < D && (diag ? bl > al || (!full && bl == al) : w_qp))
          d.G[(sb0 + bl) + (size_t)(sa0 + al) * d.ldG] = gs(al, bl);
      }
    } else {
      const int il = tid & 63;
      const bool w_pq = full || a > b, w_qp = full || b > a;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int jl = (tid >> 6) + 8 * c;
        if (a0 + il < K && b0 + jl < K && (diag ? full && il <= jl : w_pq))  // G[a0 + il][b0 + jl]
          d.G[(a0 + il) + (size_t)(b0 + jl) * d.ldG] = St[st_idx(il, jl)];
        if (b0 + il < K && a0 + jl < K && (diag ? jl < il || (!full && jl == il) : w_qp))
          d.G[(b0 + il) + (size_t)(a0 + jl) * d.ldG] = St[st_idx(jl, il)];  // G[b0 + il][a0 + jl]
      }
    }
  }
  if (stamp) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

// S_c[k1, k2] = sum over blocks l of cluster c, sum over p1 in sample k1, p2 in sample k2 of
// G_l[p1, p2]  (the rank / block sums of MPMP.jl:1373-1399 when m = 1 and the pairings were
// formed by schur_pairs_f64).  grid = (chunks, clusters).
template <class T>
__global__ __launch_bounds__(256) void schur_gsum(const SchurClusterDesc* __restrict__ cd,
                                                  const SchurBlockDesc* __restrict__ bd,
                                                  const int* __restrict__ rank_sums,
                                                  const T* __restrict__ G, T* __restrict__ S) {
  const SchurClusterDesc c = cd[blockIdx.y];
  const long long n = (long long)c.D * c.D;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const int k1 = (int)(e % c.D), k2 = (int)(e / c.D);
    T tot = T(0.0);
    for (int b = c.blk0; b < c.blk0 + c.nblk; ++b) {
      const SchurBlockDesc B = bd[b];
      const int* rs = rank_sums + B.rs_off;
      const T* g = G + B.bx_off;
      for (int p2 = rs[k2]; p2 < rs[k2 + 1]; ++p2)
        for (int p1 = rs[k1]; p1 < rs[k1 + 1]; ++p1) tot += g[p1 + (size_t)p2 * B.K];
    }
    S[c.S_off + e] = tot;
  }
}

// ------------------------------------------------------------------------------------------
// small batched elementwise kernels over block matrices (one workgroup per block)
// ------------------------------------------------------------------------------------------
struct BlkDesc {
  long long off;  // offset in the block arena
  int n;
  int pad;
};

// out = a*X + b*Y (+ s*I with s = *sc if sc != nullptr)
template <class T>
__global__ void blk_axpby(const BlkDesc* __restrict__ bd, T* out, const T* X, const T* Y, double a,
                          double b, const T* sc, double sc_mult) {
  const BlkDesc B = bd[blockIdx.x];
  const int nn = B.n * B.n;
  T s = T(0.0);
  if (sc) s = (*sc) * T(sc_mult);
  for (int e = threadIdx.x; e < nn; e += blockDim.x) {
    T v = T(0.0);
    if (a != 0.0) v += X[B.off + e] * T(a);
    if (b != 0.0) v += Y[B.off + e] * T(b);
    if (sc && (e % B.n) == (e / B.n)) v += s;
    out[B.off + e] = v;
  }
}

// *flag = OR of info[0..n): a failed factorisation anywhere in this iteration
__global__ void status_reduce(const int* info, int n, int* flag) {
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    if (info[i]) atomicOr(&any, 1);
  __syncthreads();
  if (threadIdx.x == 0) *flag = any;
}

// R_b += s I with s = (*sc) * mult; one workgroup per block
template <class T>
__global__ void diag_add(const BlkDesc* __restrict__ bd, T* R, const T* sc, double mult) {
  const BlkDesc B = bd[blockIdx.x];
  const T s = (*sc) * T(mult);
  for (int i = threadIdx.x; i < B.n; i += blockDim.x) {
    T* p = R + B.off + (size_t)i * (B.n + 1);
    *p = *p + s;
  }
}

// per-block symmetrise / mirror / transpose with a 2-D grid (block, column class):
//   mode 0: out = (Z + Z^T)/2   mode 1: out = upper triangle mirrored   mode 2: out = Z^T
template <class T>
__global__ void blk_sym2(const BlkDesc* __restrict__ bd, T* out, const T* Z, int mode) {
  const BlkDesc B = bd[blockIdx.x];
  const int n = B.n;
  const T* z = Z + B.off;
  T* o = out + B.off;
  for (int j = blockIdx.y; j < n; j += gridDim.y) {
    if (mode == 2) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) o[i + (size_t)j * n] = z[j + (size_t)i * n];
    } else {
      for (int i = threadIdx.x; i < j; i += blockDim.x) {
        T v;
        if (mode == 0) v = (z[i + (size_t)j * n] + z[j + (size_t)i * n]) * T(0.5);
        else v = z[i + (size_t)j * n];
        o[i + (size_t)j * n] = v;
        o[j + (size_t)i * n] = v;
      }
      if (threadIdx.x == 0) o[j + (size_t)j * n] = z[j + (size_t)j * n];
    }
  }
}

// fp64 out = (Z + Z^T)/2 per block (blk_sym2 mode 0) by 32x32 tile pairs staged in LDS, so
// both the reads and the writes of the transposed tile are coalesced column segments (blk_sym2
// reads and writes one of the two orientations with a stride of n doubles per lane).
// grid = (blocks, pairs of a 32-tile grid of the largest block); pair q = (I, J), I >= J, in
// row-major order over the lower tiles.  The diagonal is copied (as blk_sym2).
__global__ __launch_bounds__(256) void blk_sym_tiles(const BlkDesc* __restrict__ bd, double* out,
                                                     const double* Z) {
  __shared__ double ta[32][33], tb[32][33];
  const BlkDesc B = bd[blockIdx.x];
  const int n = B.n, nt = (n + 31) / 32;
  int I = 0;
  const int q = blockIdx.y;
  while ((I + 1) * (I + 2) / 2 <= q) ++I;
  const int J = q - I * (I + 1) / 2;
  if (I >= nt) return;
  const double* z = Z + B.off;
  double* o = out + B.off;
  const int r = threadIdx.x & 31, c0 = threadIdx.x >> 5;
  const int i0 = 32 * I, j0 = 32 * J;
  // ta = tile (I, J), tb = tile (J, I), each as column segments
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = c0 + 8 * u;
    const bool a_ok = i0 + r < n && j0 + c < n, b_ok = j0 + r < n && i0 + c < n;
    ta[c][r] = a_ok ? z[(i0 + r) + (size_t)(j0 + c) * n] : 0.0;
    tb[c][r] = b_ok ? z[(j0 + r) + (size_t)(i0 + c) * n] : 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = c0 + 8 * u;
    // (i0 + r, j0 + c) = (A(i0+r, j0+c) + A(j0+c, i0+r)) / 2; tile (J, I) gets its transpose
    if (i0 + r < n && j0 + c < n) {
      const bool dg = i0 + r == j0 + c;
      o[(i0 + r) + (size_t)(j0 + c) * n] = dg ? ta[c][r] : (ta[c][r] + tb[r][c]) * 0.5;
    }
    if (I != J && j0 + r < n && i0 + c < n)
      o[(j0 + r) + (size_t)(i0 + c) * n] = (ta[r][c] + tb[c][r]) * 0.5;
  }
}

// X += alpha * dX with alpha = *sc  (skipped when *flag != 0: the state survives a failed step)
template <class T>
__global__ void blk_axpy_dev(const BlkDesc* __restrict__ bd, T* X, const T* dX, const T* sc,
                             const int* flag) {
  if (*flag) return;
  const BlkDesc B = bd[blockIdx.x];
  const int nn = B.n * B.n;
  const T a = *sc;
  for (int e = threadIdx.x; e < nn; e += blockDim.x) X[B.off + e] = X[B.off + e] + a * dX[B.off + e];
}

// identity
template <class T>
__global__ void blk_identity(const BlkDesc* __restrict__ bd, T* out) {
  const BlkDesc B = bd[blockIdx.x];
  const int nn = B.n * B.n;
  for (int e = threadIdx.x; e < nn; e += blockDim.x)
    out[B.off + e] = T(((e % B.n) == (e / B.n)) ? 1.0 : 0.0);
}

// out = (Z + Z^T)/2   (mode 0);  out = upper triangle mirrored (mode 1, Symmetric(.)) ;
// out = Z^T (mode 2)
template <class T>
__global__ void blk_sym(const BlkDesc* __restrict__ bd, T* out, const T* Z, int mode) {
  const BlkDesc B = bd[blockIdx.x];
  const int n = B.n;
  const T* z = Z + B.off;
  T* o = out + B.off;
  if (mode == 2) {
    for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
      const int i = e % n, j = e / n;
      o[i + (size_t)j * n] = z[j + (size_t)i * n];
    }
    return;
  }
  // in-place safe: each unordered pair handled by one thread
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    const int i = e % n, j = e / n;
    if (i > j) {
      T v;
      if (mode == 0) v = (z[i + (size_t)j * n] + z[j + (size_t)i * n]) * T(0.5);
      else v = z[j + (size_t)i * n];
      o[i + (size_t)j * n] = v;
      o[j + (size_t)i * n] = v;
    } else if (i == j) {
      o[i + (size_t)j * n] = z[i + (size_t)j * n];
    }
  }
}

// per-block reductions: op 0 = sum X.*Y, op 1 = sum (X+dX).*(Y+dY), op 2 = max |X|
template <class T>
__global__ __launch_bounds__(256) void blk_reduce(const BlkDesc* __restrict__ bd, const T* X,
                                                  const T* Y, const T* dX, const T* dY, int op,
                                                  T* __restrict__ partial) {
  __shared__ T red[256];
  const BlkDesc B = bd[blockIdx.x];
  const int nn = B.n * B.n;
  T acc = T(0.0);
  for (int e = threadIdx.x; e < nn; e += blockDim.x) {
    const size_t o = B.off + e;
    if (op == 0) acc += X[o] * Y[o];
    else if (op == 1) acc += (X[o] + dX[o]) * (Y[o] + dY[o]);
    else {
      const T a = Num<T>::abs_(X[o]);
      if (a > acc) acc = a;
    }
  }
  T r = (op == 2) ? block_max(acc, red) : block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = r;
}

// vector reductions over [0, n): op 0 = sum a.*b, op 2 = max |a|; single workgroup of
// vec_reduce_threads<T>() threads.  Thread t owns elements t + NT (U u + q), combined q = 0..U-1
// in order.  fp64: 1024 threads, U = 4.  Multi-word: 256 threads and U = 2 (dd) / 1 (qd), so a
// lane has the registers of its multi-word products (at 1024 threads, 128 VGPRs per lane, the
// accumulators and loads spilled to scratch: 160 B/lane at dd, 304 at qd); the remainder walks
// the accumulators with compile-time indices
template <class T>
__host__ __device__ constexpr int vec_reduce_threads() { return sizeof(T) == 8 ? 1024 : 256; }
template <class T>
__global__ __launch_bounds__(vec_reduce_threads<T>()) void vec_reduce(const T* a, const T* b, long long n, int op,
                                                                      T* __restrict__ out) {
  constexpr int U = sizeof(T) == 8 ? 4 : (sizeof(T) == 16 ? 2 : 1);
  constexpr int NT = vec_reduce_threads<T>();
  __shared__ T red[NT];
  // (if/else throughout: a ternary on the struct types is lowered to a select of addresses,
  // which keeps the operands in scratch; the accumulators are named variables, not an array)
  auto elem = [&](long long f) {
    T v;
    if (op == 0) v = a[f] * b[f];
    else if (op == 3) v = a[f];
    else v = Num<T>::abs_(a[f]);
    return v;
  };
  auto comb = [&](T& acc, const T& v) {
    if (op == 2) {
      if (v > acc) acc = v;
    } else {
      acc += v;
    }
  };
  T a0(0.0), a1(0.0), a2(0.0), a3(0.0);
  long long e = threadIdx.x;
  for (; e + (U - 1) * NT < n; e += U * NT) {
    if constexpr (U == 4) {
      const T v0 = elem(e), v1 = elem(e + NT), v2 = elem(e + 2 * NT), v3 = elem(e + 3 * NT);
      comb(a0, v0);
      comb(a1, v1);
      comb(a2, v2);
      comb(a3, v3);
    } else if constexpr (U == 2) {
      const T v0 = elem(e), v1 = elem(e + NT);
      comb(a0, v0);
      comb(a1, v1);
    } else {
      comb(a0, elem(e));
    }
  }
  // remainder: at most U - 1 more elements, in accumulator order
  if (U > 1 && e < n) { comb(a0, elem(e)); e += NT; }
  if (U > 2 && e < n) { comb(a1, elem(e)); e += NT; }
  if (U > 3 && e < n) { comb(a2, elem(e)); e += NT; }
  T t = a0;
  if constexpr (U == 4) {
    if (op == 2) {
      if (a1 > t) t = a1;
      if (a2 > t) t = a2;
      if (a3 > t) t = a3;
    } else {
      t = (a0 + a1) + (a2 + a3);   // the pairwise order of the round-3 kernel
    }
  } else if constexpr (U == 2) {
    comb(t, a1);
  }
  red[threadIdx.x] = t;
  __syncthreads();
  for (int s2 = blockDim.x / 2; s2 > 0; s2 >>= 1) {
    if ((int)threadIdx.x < s2) {
      const T o = red[threadIdx.x + s2];
      T m = red[threadIdx.x];
      comb(m, o);
      red[threadIdx.x] = m;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

// sum or max of `cnt` values spaced `stride` apart (fixed order), single thread -> *out
template <class T>
__global__ void ordered_reduce(const T* in, int cnt, long long stride, int op, T* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  T acc = in[0];
  for (int i = 1; i < cnt; ++i) {
    const T v = in[(size_t)i * stride];
    if (op == 0) acc += v;
    else if (op == 2) { if (v > acc) acc = v; }
    else { if (v < acc) acc = v; }  // op 3: min
  }
  *out = acc;
}

// out[e] = sum_{i<cnt} in[i*stride + e]  (fixed order), e < n
// (optionally out[e] = cbase*base[e] + csum*sum, the two vector updates that follow a slab sum)
template <class T>
__global__ void slab_sum(const T* in, int cnt, long long stride, long long n, T* out,
                         const T* base = nullptr, double cbase = 0.0, double csum = 1.0) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  T acc = in[e];
  int i = 1;
  for (; i + 7 < cnt; i += 8) {  // 8 loads in flight, summed in slab order
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = in[(size_t)(i + u) * stride + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; i < cnt; ++i) acc += in[(size_t)i * stride + e];
  if (base) acc = base[e] * T(cbase) + acc * T(csum);
  out[e] = acc;
}

// slab_sum with the slabs split into 4 contiguous chunks (fixed order inside each, then
// ((c0 + c1) + (c2 + c3))): 256 threads = 64 elements x 4 chunks, each chunk's loads 8 in flight,
// so a sum over 64 slabs takes two memory latencies instead of eight.  grid = cdiv(n, 64).
template <class T>
__device__ __forceinline__ T slab_chunk_sum(const T* in, int i0, int i1, long long stride, long long e) {
  T acc = T(0.0);
  int i = i0;
  for (; i + 7 < i1; i += 8) {
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = in[(size_t)(i + u) * stride + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; i < i1; ++i) acc += in[(size_t)i * stride + e];
  return acc;
}
template <class T>
__global__ __launch_bounds__(256) void slab_sum4(const T* in, int cnt, long long stride, long long n,
                                                 T* out, const T* base = nullptr, double cbase = 0.0,
                                                 double csum = 1.0, T* out2 = nullptr) {
  __shared__ T part[4][64];
  const int el = threadIdx.x & 63, ch = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + el;
  const int i0 = (int)((long long)cnt * ch / 4), i1 = (int)((long long)cnt * (ch + 1) / 4);
  part[ch][el] = e < n ? slab_chunk_sum(in, i0, i1, stride, e) : T(0.0);
  __syncthreads();
  if (ch != 0 || e >= n) return;
  T acc = (part[0][el] + part[1][el]) + (part[2][el] + part[3][el]);
  if (base) acc = base[e] * T(cbase) + acc * T(csum);
  out[e] = acc;
  if (out2) out2[e] = acc;
}

// dy = Q^-1 r with r = cbase*base + csum*sum_{i<cnt} in[i*stride + .] (slab_sum's order): the
// slab sum and the Q^-1 GEMV of the block solve (MPMP.jl:1758-1764) in one launch.  Every
// workgroup forms all of r in LDS (n values, a few KB), then 64 rows of the product: 4 column
// chunks per row (coalesced reads of the column-major Q^-1), summed in a fixed order.
__global__ __launch_bounds__(256) void slab_qsolve(const double* __restrict__ in, int cnt,
                                                   long long stride, int n,
                                                   const double* __restrict__ base, double cbase,
                                                   double csum, const double* __restrict__ Q,
                                                   int ldq, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_sq[];
  double* r = reinterpret_cast<double*>(smem_sq);  // n
  double* part = r + n;                            // 4 x 64
  {  // r in slab_sum4's order: 64 elements x 4 slab chunks at a time
    const int el = threadIdx.x & 63, sc = threadIdx.x >> 6;
    const int i0 = (int)((long long)cnt * sc / 4), i1 = (int)((long long)cnt * (sc + 1) / 4);
    for (int e0 = 0; e0 < n; e0 += 64) {
      const int e = e0 + el;
      part[sc * 64 + el] = e < n ? slab_chunk_sum(in, i0, i1, stride, e) : 0.0;
      __syncthreads();
      if (sc == 0 && e < n) {
        double acc = (part[el] + part[64 + el]) + (part[128 + el] + part[192 + el]);
        if (base) acc = base[e] * cbase + acc * csum;
        r[e] = acc;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, ch = threadIdx.x >> 6;
  const int row = blockIdx.x * 64 + lane;
  const int j0 = (int)((long long)n * ch / 4), j1 = (int)((long long)n * (ch + 1) / 4);
  double s0 = 0.0, s1 = 0.0;
  if (row < n) {
    int j = j0;
    for (; j + 1 < j1; j += 2) {
      s0 = fma(Q[row + (size_t)j * ldq], r[j], s0);
      s1 = fma(Q[row + (size_t)(j + 1) * ldq], r[j + 1], s1);
    }
    if (j < j1) s0 = fma(Q[row + (size_t)j * ldq], r[j], s0);
  }
  part[ch * 64 + lane] = s0 + s1;
  __syncthreads();
  if (ch == 0 && row < n) out[row] = (part[lane] + part[64 + lane]) + (part[128 + lane] + part[192 + lane]);
}

// vector: out = a*x + b*y (+ c*z) over n
template <class T>
__global__ void vec_lin(T* out, const T* x, double a, const T* y, double b, const T* z, double c,
                        long long n) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    T v = x[e] * T(a);
    if (y) v += y[e] * T(b);
    if (z) v += z[e] * T(c);
    out[e] = v;
  }
}

// fill rectangles (rows x cols, column-major with ld) with v; blockIdx.y = rectangle
struct RectDesc {
  void* p;
  int rows, cols, ld;
};
template <class T>
__global__ void rect_fill(const RectDesc* __restrict__ rd, double v) {
  const RectDesc R = rd[blockIdx.y];
  T* p = reinterpret_cast<T*>(R.p);
  for (int c = blockIdx.x; c < R.cols; c += gridDim.x)
    for (int r = threadIdx.x; r < R.rows; r += blockDim.x) p[r + (size_t)c * R.ld] = T(v);
}

// out[0..n) = v
// dst = src unless *halt (the loop body was skipped by device-side termination): keeps P, p, d
// of the last loop body that ran for the pipelined loop
template <class T>
__global__ void vec_copy_guard(T* __restrict__ dst, const T* __restrict__ src, long long n,
                               const int* __restrict__ halt) {
  if (*halt) return;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x)
    dst[e] = src[e];
}

// dst_q = src_q for the (up to two) segments q unless *halt: 16-byte moves over the segments'
// bytes (the buffers are 256-byte aligned device allocations; an 8-byte tail when a segment's
// byte count is odd in 8-byte words), one launch for the keep-residuals copies of a pipelined
// loop body (P and d; the 8 MB P of C3 took 16.7 us as 8-byte element copies)
__global__ void copy_guard2(void* __restrict__ d0, const void* __restrict__ s0, long long b0,
                            void* __restrict__ d1, const void* __restrict__ s1, long long b1,
                            const int* __restrict__ halt) {
  if (*halt) return;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  auto seg = [&](void* dv, const void* sv, long long bytes) {
    const long long n16 = bytes >> 4;
    uint4* dq = reinterpret_cast<uint4*>(dv);
    const uint4* sq = reinterpret_cast<const uint4*>(sv);
    for (long long e = tid; e < n16; e += stride) dq[e] = sq[e];
    if ((bytes & 15) && tid == 0)
      reinterpret_cast<double*>(dv)[(bytes >> 3) - 1] = reinterpret_cast<const double*>(sv)[(bytes >> 3) - 1];
  };
  seg(d0, s0, b0);
  if (d1) seg(d1, s1, b1);
}

template <class T>
__global__ void vec_fill(T* out, double v, long long n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) out[e] = T(v);
}

// x += (*sc) * dx
// x_q += alpha_q dx_q for up to 4 vectors (blockIdx.y = q), unless *flag (failed factorisation)
template <class T> struct AxpyItem {
  T* x;
  const T* dx;
  const T* alpha;
  long long n;
};
template <class T> struct AxpyList { AxpyItem<T> it[4]; };
// guard: skip when any status word info[0..ninfo) is set (a factorisation failed)
template <class T>
__global__ void vec_axpy_list(AxpyList<T> L, const int* info, int ninfo) {
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < ninfo; i += blockDim.x)
    if (info[i]) any = 1;
  __syncthreads();
  if (any) return;
  const AxpyItem<T> I = L.it[blockIdx.y];
  const T a = *I.alpha;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < I.n;
       e += (long long)gridDim.x * blockDim.x)
    I.x[e] = I.x[e] + a * I.dx[e];
}
template <class T>
__global__ void vec_axpy_dev(T* x, const T* dx, const T* sc, long long n, const int* flag) {
  if (*flag) return;
  const T a = *sc;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x)
    x[e] = x[e] + a * dx[e];
}

// ------------------------------------------------------------------------------------------
// Low-rank operators
// ------------------------------------------------------------------------------------------
// Per (block, r>=s) pair: column dots val[p] = sum_i V[i,p] U[i,p]  (U = Z[r,s] V), one wave
// per column (trace_A, MPMP.jl:1558-1560)
struct PairDesc {
  long long u_off;    // U_{b,rs} (delta x K, ld delta)
  long long v_off;    // V_b
  long long val_off;  // val_{b,rs} (K)
  int delta, K;
  int lam_off;        // lambda_b (K)
  int x_off;          // tuple of column 0 when the cluster's tuples map 1:1 to columns (m = L =
                      // rank = 1), else -1
};

template <class T>
__device__ __forceinline__ T wave_sum_t(T v) {
  if constexpr (sizeof(T) == 8) {
    return wave_sum_dpp(v);
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += shfl_xor_t(v, o);
    return v;
  }
}

// trace_A + tuple aggregation in one launch for clusters with m = L = rank = 1 (tuple k <->
// column k): out[x_off + col] = c_agg lambda_col (U[:,col] . V[:,col]) + c_in in[.] + c_in2 in2[.]
template <class T>
__global__ __launch_bounds__(256) void colsum_rhs(const PairDesc* __restrict__ pd, const T* U,
                                                  const T* V, const T* lam, const T* in,
                                                  double c_in, const T* in2, double c_in2,
                                                  double c_agg, T* out) {
  const PairDesc P = pd[blockIdx.y];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = blockIdx.x * 4 + wave;
  if (col >= P.K) return;
  const T* u = U + P.u_off + (size_t)col * P.delta;
  const T* v = V + P.v_off + (size_t)col * P.delta;
  T acc = T(0.0);
  for (int i = lane; i < P.delta; i += 64) acc += u[i] * v[i];
  acc = wave_sum_t(acc);
  if (lane == 0) {
    const long long g = (long long)P.x_off + col;
    T o = lam[P.lam_off + col] * acc * T(c_agg);
    if (in) o += in[g] * T(c_in);
    if (in2) o += in2[g] * T(c_in2);
    out[g] = o;
  }
}
template <class T>
__global__ __launch_bounds__(256) void colsum_dot(const PairDesc* __restrict__ pd, const T* U,
                                                  const T* V, T* val) {
  const PairDesc P = pd[blockIdx.y];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = blockIdx.x * 4 + wave;
  if (col >= P.K) return;
  const T* u = U + P.u_off + (size_t)col * P.delta;
  const T* v = V + P.v_off + (size_t)col * P.delta;
  T acc = T(0.0);
  for (int i = lane; i < P.delta; i += 64) acc += u[i] * v[i];
  // fixed butterfly over the wave
  for (int s = 32; s > 0; s >>= 1) {
    if constexpr (sizeof(T) == 8) {
      acc += __shfl_xor(acc, s);
    } else {
      T o;
      double* od = reinterpret_cast<double*>(&o);
      const double* ad = reinterpret_cast<const double*>(&acc);
#pragma unroll
      for (int q = 0; q < (int)(sizeof(T) / 8); ++q) od[q] = __shfl_xor(ad[q], s);
      acc += o;
    }
  }
  if (lane == 0) val[P.val_off + col] = acc;
}

// Per (block, r>=s): Vs[:,p] = V[:,p] * w_p with w_p = a[xoff + tuple(r,s,k(p))] * lambda_p * scale
// (compute_weighted_A!, MPMP.jl:1654)
struct ScaleDesc {
  long long v_off, vs_off;
  int delta, K;
  int ks_off;     // sample index of each column
  int lam_off;
  int a_off;      // local x offset of the cluster + (s + r(r+1)/2) N
  int pad;
  double scale;   // 1/2 on off-diagonal (r != s) blocks, MPMP.jl:1661-1663
};
template <class T>
__global__ void scale_cols(const ScaleDesc* __restrict__ sd, const T* V, const T* lam,
                           const int* ksamp, const T* a, T* Vs) {
  const ScaleDesc S = sd[blockIdx.y];
  const long long tot = (long long)S.delta * S.K;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int p = (int)(e / S.delta);
    const T w = a[S.a_off + ksamp[S.ks_off + p]] * lam[S.lam_off + p] * T(S.scale);
    Vs[S.vs_off + e] = V[S.v_off + e] * w;
  }
}

// Tuple aggregation (trace_A's sample sum, MPMP.jl:1563-1578 / 1592-1615):
//   out[t] = c_in * in[t] + c_in2 * in2[t] + c_agg * sum_{l} sum_{p in k} lambda_p val_{b,rs}[p]
// one thread per local tuple t = xoff_c + (s + r(r+1)/2) N + k
struct TupleDesc {
  int x_off;      // local x offset of this cluster
  int N, m;
  int blk0, nblk; // local blocks
  int t0;         // first local tuple index (== x_off)
};
struct TupleBlock {
  long long val_off;   // val of (b, rs=0); rs stride = K
  int K;
  int rs_off;          // rank_sums offset (N+1 entries)
  int lam_off;
  int pad;
};
template <class T>
__global__ void tuple_aggregate(const TupleDesc* __restrict__ td, int ncl,
                                const TupleBlock* __restrict__ tb, const int* rank_sums,
                                const T* lam, const T* val, const T* in, double c_in,
                                const T* in2, double c_in2, double c_agg, T* out, long long ntup) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ntup) return;
  int lo = 0, hi = ncl - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (td[mid].t0 <= g) lo = mid; else hi = mid - 1;
  }
  const TupleDesc C = td[lo];
  const int loc = (int)(g - C.t0);
  const int k = loc % C.N, rs = loc / C.N;
  T agg = T(0.0);
  for (int b = C.blk0; b < C.blk0 + C.nblk; ++b) {
    const TupleBlock B = tb[b];
    const int* rsum = rank_sums + B.rs_off;
    const T* vv = val + B.val_off + (size_t)rs * B.K;
    for (int p = rsum[k]; p < rsum[k + 1]; ++p) agg += lam[B.lam_off + p] * vv[p];
  }
  T o = agg * T(c_agg);
  if (in) o += in[g] * T(c_in);
  if (in2) o += in2[g] * T(c_in2);
  out[g] = o;
}

// A_Y extraction: val_{b,rs}[p] = BY_b[r K + p, s K + p]   (MPMP.jl:1320-1330)
struct AYDesc {
  long long by_off, ay_off;
  int K, m;
};
template <class T>
__global__ void extract_AY(const AYDesc* __restrict__ ad, const T* BY, T* AY) {
  const AYDesc A = ad[blockIdx.x];
  const int nrs = A.m * (A.m + 1) / 2;
  const int ld = A.m * A.K;
  for (int e = threadIdx.x; e < nrs * A.K; e += blockDim.x) {
    const int p = e % A.K, rs = e / A.K;
    int r = 0;
    while ((r + 1) * (r + 2) / 2 <= rs) ++r;
    const int s = rs - r * (r + 1) / 2;
    AY[A.ay_off + e] = BY[A.by_off + (r * A.K + p) + (size_t)(s * A.K + p) * ld];
  }
}

// ------------------------------------------------------------------------------------------
// scalar logic of the driver loop, on the device (MPMP.jl:755-756, 832-837, 871-874, 1893-1897)
// ------------------------------------------------------------------------------------------
enum { SC_MU = 0, SC_MU_P, SC_R, SC_BETA, SC_BETA_C, SC_MU_C, SC_ALPHA_P, SC_ALPHA_D, SC_MINEIG_X,
       SC_MINEIG_Y, SC_POBJ, SC_DOBJ, SC_ERR_PMAT, SC_ERR_PVEC, SC_ERR_DVEC, SC_DOT_XY, SC_DOT_XDY,
       SC_DOT_CX, SC_DOT_BY, SC_DOT_CY, SC_TMP0, SC_TMP1, SC_TMP2,
       SC_DMU,  // mu_c - mu_p (the corrector's R from the predictor's, fp64)
       // loop control decided on the device (pipelined iterate): check_pd_feasibility and
       // terminate of the state after the last update (MPMP.jl:942-945, 1147-1185)
       SC_PDFEAS, SC_HALT, SC_GAP, SC_COUNT };

// A fixed-order reduction folded into scalar_kernel: sc[dst] = op over cnt values spaced
// `stride` apart (op 0 sum, 2 max, 3 min, 4 max |.|).  Used for the rank-ordered reductions of
// the exchanged partials and other short vectors, so they cost no launch of their own.
template <class T> struct FoldRed {
  const T* src;
  long long stride;
  int cnt, op, dst, pad;
};
template <class T> struct ScalarParams {
  T beta_inf, beta_feas, gamma, b0;
  T gap_thr, p_thr, d_thr;  // terminate / check_pd_feasibility thresholds (device loop control)
  double dim;
  int pd_feas;  // 0/1 from the host; -1: read sc[SC_PDFEAS] (decided at the end of the last update)
  int need_p, need_d;
  int nred;
  int zero_cy;  // which == 3 without C: <C,Y> = 0
  int fold_all;  // fp64: fold_all_f64 (all loads of all folds in flight; CLRSDP_FOLD_ALL=0: off)
  int zero_n;   // zero the status words zero_ptr[0..zero_n) (start of an iteration)
  int* zero_ptr;
  int* halt_ptr;  // which == 0: status word "skip this loop body" (device-decided termination)
  unsigned long long* stamps;  // which == 0: reset the SCHUR-stage clock pair (min start, max end)
  // which == 3: the loop control (gap, pd_feas, halt) is left as the last body that ran decided
  // it when a status word guard[0..nguard) is set: the body failed and applied nothing (the LU
  // fallback re-runs it with the control of the body before)
  const int* guard;
  int nguard;
  FoldRed<T> red[6];
};

// This rank's failure bits (1 S_j, 2 Q, 4 X, 8 X^-1 by LU, 16 Y; the layout of the Solver's
// status words) as a value of T for STEP's all-gather, and their OR over the gathered ranks
// into one status word (so every rank skips its update and reports alike).
template <class T>
__global__ __launch_bounds__(256) void status_bits(const int* __restrict__ info, int nb, int nS,
                                                   int s0, int q0, int l0, T* out) {
  __shared__ int bits;
  if (threadIdx.x == 0) bits = 0;
  __syncthreads();
  int v = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    if (info[i]) v |= 4;
    if (info[nb + i]) v |= 16;
    if (info[l0 + i]) v |= 8;
  }
  for (int i = threadIdx.x; i < nS; i += 256)
    if (info[s0 + i]) v |= 1;
  if (threadIdx.x == 0 && info[q0]) v |= 2;
  if (v) atomicOr(&bits, v);
  __syncthreads();
  if (threadIdx.x == 0) *out = T((double)bits);
}
template <class T>
__global__ void status_gather(const T* __restrict__ recv, int world, long long stride, int slot,
                              int* dst) {
  if (threadIdx.x != 0) return;
  int b = 0;
  for (int r = 0; r < world; ++r) b |= (int)Num<T>::hi(recv[(size_t)r * stride + slot]);
  *dst = b;
}

template <class T>
__device__ inline bool pd_feasible(const T* sc, const ScalarParams<T>& p) {
  return p.pd_feas < 0 ? sc[SC_PDFEAS] > T(0.5) : p.pd_feas != 0;
}

// gap, pd_feas and terminate() of the current objectives and errors (MPMP.jl:942-945 and
// 1067-1078, 1147-1185); excl_b0: the initial gap of MPMP.jl:725 (compute_duality_gap has no b0)
template <class T>
__device__ __forceinline__ void control_update(T* sc, const ScalarParams<T>& p, bool excl_b0) {
  T po = sc[SC_POBJ], dob = sc[SC_DOBJ];
  if (excl_b0) {
    po = po - p.b0;
    dob = dob - p.b0;
  }
  T den = Num<T>::abs_(po + dob);
  if (!(den > T(1.0))) den = T(1.0);
  const T gap = Num<T>::abs_(po - dob) / den;
  T perr = sc[SC_ERR_PVEC];
  if (sc[SC_ERR_PMAT] > perr) perr = sc[SC_ERR_PMAT];
  const T derr = sc[SC_ERR_DVEC];
  const bool pf = perr < p.p_thr, df = derr < p.d_thr, go = gap < p.gap_thr;
  // sticky once set (a skipped body must not un-terminate the loop); reset by excl_b0 (initial)
  const bool halt = (p.need_p && pf) || (p.need_d && df) || (pf && df && go) ||
                    (!excl_b0 && sc[SC_HALT] > T(0.5));
  sc[SC_GAP] = gap;
  sc[SC_PDFEAS] = T((pf && df) ? 1.0 : 0.0);
  sc[SC_HALT] = T(halt ? 1.0 : 0.0);
}

// one wave: lane l folds elements l, l+64, ... in order, then a fixed xor butterfly
template <class T>
__device__ __forceinline__ T fold_wave(const FoldRed<T>& r, int lane) {
  const bool sum = r.op == 0;
  const bool mn = r.op == 3;
  T acc;
  bool have = false;
  for (int i = lane; i < r.cnt; i += 64) {
    T v = r.src[(size_t)i * r.stride];
    if (r.op == 4) v = Num<T>::abs_(v);
    if (!have) { acc = v; have = true; }
    else if (sum) acc += v;
    else if (mn) { if (v < acc) acc = v; }
    else { if (v > acc) acc = v; }
  }
  // lanes without elements hold the first element (neutral for min/max) or 0 (sum)
  if (!have) {
    if (sum) acc = T(0.0);
    else if (r.op == 4) acc = Num<T>::abs_(r.src[0]);
    else acc = r.src[0];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const T v = shfl_xor_t(acc, o);
    if (sum) acc += v;
    else if (mn) { if (v < acc) acc = v; }
    else { if (v > acc) acc = v; }
  }
  return acc;
}

// fp64: all folds of a launch at once -- every lane issues its loads of every fold before the
// first combine (one memory latency instead of one per fold and per 64 elements), then the six
// butterflies interleaved.  Bitwise fold_wave's result: lane l combines elements l, l+64, ... in
// order, then the same xor butterfly.
__device__ __forceinline__ double fold_op(int op, double acc, double v) {
  if (op == 0) return acc + v;
  if (op == 3) return v < acc ? v : acc;
  return v > acc ? v : acc;
}
__device__ __forceinline__ void fold_all_f64(const ScalarParams<double>& p, double* sc, int lane) {
  double acc[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) acc[q] = 0.0;
  const int nred = p.nred;
  int maxcnt = 0;
#pragma unroll
  for (int q = 0; q < 6; ++q)
    if (q < nred) maxcnt = max(maxcnt, p.red[q].cnt);
  for (int i0 = 0; i0 < maxcnt; i0 += 256) {
    double v[6][4];
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + lane + 64 * u;
        v[q][u] = (q < nred && i < p.red[q].cnt) ? p.red[q].src[(size_t)i * p.red[q].stride] : 0.0;
      }
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      if (q >= nred) continue;
      const int op = p.red[q].op, cnt = p.red[q].cnt;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + lane + 64 * u;
        if (i >= cnt) continue;
        double x = op == 4 ? fabs(v[q][u]) : v[q][u];
        acc[q] = (i < 64) ? x : fold_op(op, acc[q], x);  // the lane's first element starts it
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) {  // lanes without elements: neutral (sum 0, else element 0)
    if (q >= nred) continue;
    if (lane >= p.red[q].cnt && p.red[q].op != 0) {
      const double x0 = p.red[q].src[0];
      acc[q] = p.red[q].op == 4 ? fabs(x0) : x0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (q < nred) acc[q] = fold_op(p.red[q].op, acc[q], __shfl_xor(acc[q], o));
#pragma unroll
  for (int q = 0; q < 6; ++q)
    if (q < nred && lane == 0) sc[p.red[q].dst] = acc[q];
}

// the scalar control logic of one launch, lane 0 (sc: the slots, in LDS or global)
template <class T>
__device__ __forceinline__ void scalar_logic(T* sc, const ScalarParams<T>& p, int which, bool failed) {
  const T dim = T(p.dim);
  if (which == 0) {  // mu, mu_p
    const bool pdf = pd_feasible(sc, p);
    if (p.halt_ptr) *p.halt_ptr = (p.pd_feas < 0 && sc[SC_HALT] > T(0.5)) ? 1 : 0;
    if (p.stamps) {
      p.stamps[0] = p.stamps[2] = p.stamps[4] = ~0ull;
      p.stamps[1] = p.stamps[3] = p.stamps[5] = 0ull;
    }
    sc[SC_MU] = sc[SC_DOT_XY] / dim;
    sc[SC_MU_P] = sel(pdf, T(0.0), p.beta_inf * sc[SC_MU]);
  } else if (which == 1) {  // r, beta, beta_c, mu_c
    const T r = sc[SC_DOT_XDY] / (sc[SC_MU] * dim);
    const T beta = sel(r < T(1.0), r * r, r);
    T bc;
    if (pd_feasible(sc, p)) {
      bc = sel(p.beta_feas > beta, p.beta_feas, beta);
      if (bc > T(1.0)) bc = T(1.0);
    } else {
      bc = sel(p.beta_inf > beta, p.beta_inf, beta);
    }
    sc[SC_R] = r;
    sc[SC_BETA] = beta;
    sc[SC_BETA_C] = bc;
    sc[SC_MU_C] = bc * sc[SC_MU];
    sc[SC_DMU] = sc[SC_MU_C] - sc[SC_MU_P];
  } else if (which == 2) {  // step lengths
    const T g = p.gamma;
    T ap = T(1.0), ad = T(1.0);
    if (!(sc[SC_MINEIG_X] > -g)) ap = -g / sc[SC_MINEIG_X];
    if (!(sc[SC_MINEIG_Y] > -g)) ad = -g / sc[SC_MINEIG_Y];
    if (pd_feasible(sc, p)) {
      if (ad < ap) ap = ad;
      else ad = ap;
    }
    sc[SC_ALPHA_P] = ap;
    sc[SC_ALPHA_D] = ad;
  } else if (which == 3) {  // objectives
    if (p.zero_cy) sc[SC_DOT_CY] = T(0.0);
    sc[SC_POBJ] = sc[SC_DOT_CX] + p.b0;
    sc[SC_DOBJ] = sc[SC_DOT_CY] + sc[SC_DOT_BY] + p.b0;
    if (!failed) control_update(sc, p, false);
  } else if (which == 4) {  // objectives + control of the initial point (MPMP.jl:723-736)
    if (p.zero_cy) sc[SC_DOT_CY] = T(0.0);
    sc[SC_POBJ] = sc[SC_DOT_CX] + p.b0;
    sc[SC_DOBJ] = sc[SC_DOT_CY] + sc[SC_DOT_BY] + p.b0;
    control_update(sc, p, true);
  }
}

// (the opt-in LDS mirror of the slots, CLRSDP_SC_LDS=1, measured within noise in round 5 and is
// gone, round 6)
template <class T>
__global__ __launch_bounds__(64) void scalar_kernel(T* scg, ScalarParams<T> p, int which) {
  const int lane = threadIdx.x;
  T* sc = scg;
  bool fl = false;  // any status word set (which == 3): the wave reads them strided, one ballot
  for (int e = lane; e < p.zero_n; e += 64) p.zero_ptr[e] = 0;
  if (sizeof(T) == 8 && p.fold_all) {
    if constexpr (sizeof(T) == 8) fold_all_f64(p, sc, lane);
  } else {
    // compile-time indices into the by-value parameter block (a runtime index makes the
    // compiler copy the whole block to scratch: 104 B/lane at quad-double)
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      if (q < p.nred) {
        const T v = fold_wave(p.red[q], lane);
        if (lane == 0) sc[p.red[q].dst] = v;
      }
    }
  }
  if (which == 3)
    for (int e = lane; e < p.nguard; e += 64) fl = fl || p.guard[e] != 0;
  const bool failed = __any(fl);
  if (lane == 0) scalar_logic(sc, p, which, failed);
}

// x += alpha_p dx, y += alpha_d dy (guarded), then <c,x>, <b,y> and the objectives
// (MPMP.jl:877-878, 940-941; one rank, C = 0).  One 1024-thread workgroup.
template <class T>
__global__ __launch_bounds__(1024) void update_small(T* __restrict__ x, const T* __restrict__ dx,
                                                     long long nx, T* __restrict__ y,
                                                     const T* __restrict__ dy, long long ny,
                                                     const T* __restrict__ c,
                                                     const T* __restrict__ b, T* sc,
                                                     const int* info, int ninfo,
                                                     ScalarParams<T> p) {
  const T b0 = p.b0;
  __shared__ T red[1024];
  __shared__ int any;
  const int tid = threadIdx.x;
  if (tid == 0) any = 0;
  __syncthreads();
  for (int i = tid; i < ninfo; i += 1024)
    if (info[i]) any = 1;
  __syncthreads();
  const bool upd = !any;
  const T ap = sc[SC_ALPHA_P], ad = sc[SC_ALPHA_D];
  T acc = T(0.0);
  // (restrict + unroll: the loads of several elements are in flight together; the per-thread
  // accumulation order is unchanged)
#pragma unroll 8
  for (long long e = tid; e < nx; e += 1024) {
    T v = x[e];
    if (upd) { v = v + ap * dx[e]; x[e] = v; }
    acc += c[e] * v;
  }
  red[tid] = acc;
  __syncthreads();
  for (int s2 = 512; s2 > 0; s2 >>= 1) {
    if (tid < s2) red[tid] = red[tid] + red[tid + s2];
    __syncthreads();
  }
  const T cx = red[0];
  __syncthreads();
  acc = T(0.0);
  for (long long e = tid; e < ny; e += 1024) {
    T v = y[e];
    if (upd) { v = v + ad * dy[e]; y[e] = v; }
    acc += b[e] * v;
  }
  red[tid] = acc;
  __syncthreads();
  for (int s2 = 512; s2 > 0; s2 >>= 1) {
    if (tid < s2) red[tid] = red[tid] + red[tid + s2];
    __syncthreads();
  }
  if (tid == 0) {
    sc[SC_DOT_CX] = cx;
    sc[SC_DOT_CY] = T(0.0);
    sc[SC_DOT_BY] = red[0];
    sc[SC_POBJ] = cx + b0;
    sc[SC_DOBJ] = red[0] + b0;
    control_update(sc, p, false);
  }
}

}  // namespace clrsdp
