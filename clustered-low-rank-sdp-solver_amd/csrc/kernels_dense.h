// kernels_dense.h -- small dense factorisations kept on chip (registers / LDS).
//
//   chol_inv_reg   A = L L^T and L^-1 in one pass, the matrix held in registers (a TRxTC tile per
//                  thread), columns broadcast through LDS.  Replaces spd_inv! (MPMP.jl:766),
//                  cho! (1846) and the LU solves of S_j / Q (1436-1463, 1501, 1752-1772): every
//                  later solve becomes an MFMA GEMM with L^-1.
//   eigmin_lds     lambda_min of a symmetric n <= 128 matrix held in LDS: Householder
//                  tridiagonalisation + Sturm multisection (approx_eig_qr!, MPMP.jl:1857-1870).
#pragma once
#include "kernels.h"

namespace clrsdp {

// Deterministic block reduction for 512 threads: wave butterfly, then 8 wave sums in order.
template <class T>
__device__ __forceinline__ T wave_sum(T v) {
  for (int s = 32; s > 0; s >>= 1) {
    if constexpr (sizeof(T) == 8) {
      v += __shfl_xor(v, s);
    } else {
      T o;
      double* od = reinterpret_cast<double*>(&o);
      const double* vd = reinterpret_cast<const double*>(&v);
#pragma unroll
      for (int q = 0; q < (int)(sizeof(T) / 8); ++q) od[q] = __shfl_xor(vd[q], s);
      v += o;
    }
  }
  return v;
}
template <class T, int NW>
__device__ __forceinline__ T block_sum_w(T v, T* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  T s = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) s += red[i];
  __syncthreads();
  return s;
}

// ------------------------------------------------------------------------------------------
// chol_inv_reg: for each matrix b of the batch, read A_b (n x n, SPD, lower triangle used),
// write Linv_b = L^-1 (lower triangular, exact zeros above the diagonal) and optionally L_b.
// Thread t owns rows [tr*TR, tr*TR+TR) x cols [tc*TC, tc*TC+TC) with tr = t % GR, tc = t / GR.
// Right-looking: step j broadcasts column j of L and row j of L^-1 through LDS (2 barriers); the
// column is scaled by the reciprocal of the pivot, formed once by the pivot's owner.
// In-place safe (out == A): every thread reads its own tile before anything is written.
// ------------------------------------------------------------------------------------------
// INV = false: the Cholesky factor only (out_l, in place allowed; out_inv unused)
template <class T, int TR, int TC, int GR, int GC, bool INV = true>
__global__ __launch_bounds__(GR * GC) void chol_inv_reg(const MatDesc<T>* __restrict__ in,
                                                        const MatDesc<T>* __restrict__ out_inv,
                                                        const MatDesc<T>* __restrict__ out_l,
                                                        int* __restrict__ info) {
  constexpr int NMAX = TR * GR;
  static_assert(TR * GR == TC * GC, "square tile grid");
  __shared__ T col[NMAX];
  __shared__ T row[NMAX];
  __shared__ T sd, rsd;  // pivot and its reciprocal (one division per column, by its owner)
  __shared__ int fail;
  const MatDesc<T> d = in[blockIdx.x];
  const int n = d.n;
  const int t = threadIdx.x, tr = t % GR, tc = t / GR;
  const int r0 = tr * TR, c0 = tc * TC;
  T a[TR][TC], x[TR][TC];
#pragma unroll
  for (int i = 0; i < TR; ++i)
#pragma unroll
    for (int c = 0; c < TC; ++c) {
      const int gi = r0 + i, gc = c0 + c;
      a[i][c] = T(0.0);
      if (gi < n && gc < n && gc <= gi) a[i][c] = d.A[gi + (size_t)gc * d.lda];
      x[i][c] = T(gi == gc ? 1.0 : 0.0);
    }
  if (t == 0) {
    fail = 0;
    const T d0 = d.A[0];
    if (!(d0 > T(0.0))) fail = 1;
    pivot_sqrt(d0, sd, rsd);
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    if (fail) break;
    const T s = sd, rs = rsd;
    // phase B: column j of L -> col[], row j of L^-1 -> row[]  (static register indices only)
    const int jc = j % TC, jr = j % TR;
    if (tc == j / TC) {
#pragma unroll
      for (int c = 0; c < TC; ++c) {
        if (c == jc) {
#pragma unroll
          for (int i = 0; i < TR; ++i) {
            const int gi = r0 + i;
            if (gi >= j && gi < n) {
              const T l = (gi == j) ? s : a[i][c] * rs;
              a[i][c] = l;
              col[gi] = l;
            }
          }
        }
      }
    }
    if (INV && tr == j / TR) {
#pragma unroll
      for (int i = 0; i < TR; ++i) {
        if (i == jr) {
#pragma unroll
          for (int c = 0; c < TC; ++c) {
            x[i][c] = x[i][c] * rs;
            row[c0 + c] = x[i][c];
          }
        }
      }
    }
    __syncthreads();
    // phase C: trailing update of A and of L^-1
    if (r0 + TR - 1 > j) {
      T ci[TR];
#pragma unroll
      for (int i = 0; i < TR; ++i) {
        ci[i] = T(0.0);
        if (r0 + i > j && r0 + i < n) ci[i] = col[r0 + i];
      }
      if (c0 + TC - 1 > j && c0 <= r0 + TR - 1) {
#pragma unroll
        for (int c = 0; c < TC; ++c) {
          const int gc = c0 + c;
          if (gc > j && gc < n) {
            const T cc = col[gc];
#pragma unroll
            for (int i = 0; i < TR; ++i)
              if (gc <= r0 + i) a[i][c] = a[i][c] - ci[i] * cc;
          }
        }
      }
      if (INV && c0 <= j) {
#pragma unroll
        for (int c = 0; c < TC; ++c) {
          const T rc = row[c0 + c];
#pragma unroll
          for (int i = 0; i < TR; ++i) x[i][c] = x[i][c] - ci[i] * rc;
        }
      }
    }
    // next pivot, by the owner of (j+1, j+1)
    const int jn = j + 1;
    if (jn < n && tr == jn / TR && tc == jn / TC) {
      T dn = T(0.0);
#pragma unroll
      for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int c = 0; c < TC; ++c)
          if (i == jn % TR && c == jn % TC) dn = a[i][c];
      if (!(dn > T(0.0))) fail = jn + 1;
      pivot_sqrt(dn, sd, rsd);
    }
    __syncthreads();
  }
  if (t == 0 && info) info[blockIdx.x] = fail;
  if (INV) {
    const MatDesc<T> o = out_inv[blockIdx.x];
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int c = 0; c < TC; ++c) {
        const int gi = r0 + i, gc = c0 + c;
        if (gi < n && gc < n) o.A[gi + (size_t)gc * o.lda] = x[i][c];
      }
  }
  if (out_l) {
    const MatDesc<T> ol = out_l[blockIdx.x];
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int c = 0; c < TC; ++c) {
        const int gi = r0 + i, gc = c0 + c;
        if (gi < n && gc < n) ol.A[gi + (size_t)gc * ol.lda] = sel(gc <= gi, a[i][c], T(0.0));
      }
  }
}

// ------------------------------------------------------------------------------------------
// chol_packed: the column steps of chol_inv_reg for multi-word blocks n <= 64, with the elements
// placed by the steps at which they are live instead of on a fixed tile grid.  The lower
// triangle of A is numbered column-major (element (r, c) is updated at the steps j < c) and cut
// into 64-element slots; L^-1 (element (r, c) updated at the steps c <= j < r) is cut into 8 x 8
// tiles on and below the diagonal.  Slot s is register s / NW of wave s % NW, and a wave skips a
// slot (uniform branch) outside its live steps.  The waves then issue about n^3/384 multi-word
// FMAs for A instead of the grid's ~n^2/2 (a grid wave stays busy while any of its 64 rows is
// live) -- at quad-double one FMA is ~225 fp64 instructions.  With LDL = false every element goes
// through the same operations in the same order as in chol_inv_reg, so L and L^-1 are bitwise
// the same.
// LDL = true (quad-double): the square-root-free form A = U D U^T (U unit lower), so that the
// serial chain per column carries one reciprocal 1/d_j (two quad-double products) instead of a
// square root and its reciprocal (five); L = U D^1/2 and L^-1 = D^-1/2 U^-1 follow at the end
// with all n square roots side by side.  The factors then differ from chol_inv_reg's in the
// last bits only.
// ------------------------------------------------------------------------------------------
// NMAX = 128 (round 3, late): the multi-word potrf of blocks up to 128 (the double-double S_j
// of config 4), 129 slots of A, nine registers per thread at 1024 threads.
template <class T, int NT, bool INV, bool LDL = false, int NMAX = 64>
__global__ __launch_bounds__(NT) void chol_packed(const MatDesc<T>* __restrict__ in,
                                                  const MatDesc<T>* __restrict__ out_inv,
                                                  const MatDesc<T>* __restrict__ out_l,
                                                  int* __restrict__ info) {
  constexpr int NW = NT / 64;
  constexpr int SA = (NMAX * (NMAX + 1) / 2 + 63) / 64;  // 33 slots of A at n = 64
  constexpr int SX = (NMAX / 8) * (NMAX / 8 + 1) / 2;     // 36 tiles of L^-1
  constexpr int KA = (SA + NW - 1) / NW, KX = INV ? (SX + NW - 1) / NW : 1;
  __shared__ T col[NMAX];   // column j of L (LDL: of U)
  __shared__ T row[NMAX];   // row j of L^-1 (LDL: of U^-1)
  __shared__ T colu[LDL ? NMAX : 1];  // LDL: column j of the trailing matrix, unscaled
  __shared__ T dgl[LDL ? NMAX : 1];   // LDL: the pivots d_j
  __shared__ T sd, rsd;
  __shared__ int fail;
  const MatDesc<T> d = in[blockIdx.x];
  const int n = d.n, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  auto wave_max = [](int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return __builtin_amdgcn_readfirstlane(v);
  };
  // A: slot w + NW k, element e = 64 slot + lane of the column-major lower triangle
  T a[KA];
  int ar[KA], ac[KA], alo[KA], ahi[KA];  // (ar, ac) = -1: no element; [alo, ahi] slot columns
  const int ne = n * (n + 1) / 2;
#pragma unroll
  for (int k = 0; k < KA; ++k) {
    const int e = 64 * (w + NW * k) + lane;
    int r = -1, c = -1;
    if (e < ne) {
      int rem = e;
      c = 0;
      while (rem >= n - c) {
        rem -= n - c;
        ++c;
      }
      r = c + rem;
    }
    ar[k] = r;
    ac[k] = c;
    a[k] = T(0.0);
    if (c >= 0) a[k] = d.A[r + (size_t)c * d.lda];
    ahi[k] = wave_max(c);
    alo[k] = -wave_max(c >= 0 ? -c : -NMAX);
  }
  // L^-1: tile w + NW k of the column-major 8 x 8 tiles (R >= C); lane (r, c) = (8R + l%8, 8C + l/8)
  T x[KX];
  int xr[KX], xc[KX], xR[KX], xC[KX];  // xR = -1: no tile
  if constexpr (INV) {
    const int nt8 = (n + 7) / 8;
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      int t = w + NW * k, C = 0;
      while (C < nt8 && t >= nt8 - C) {
        t -= nt8 - C;
        ++C;
      }
      const bool tv = C < nt8;
      const int R = C + t;
      xR[k] = tv ? R : -1;
      xC[k] = tv ? C : 0;
      const int r = 8 * R + (lane & 7), c = 8 * C + (lane >> 3);
      const bool v = tv && r < n && c < n;
      xr[k] = v ? r : -1;
      xc[k] = v ? c : NMAX;
      x[k] = T((v && r == c) ? 1.0 : 0.0);
    }
  }
  // the pivot of column jp from its (updated) diagonal entry dn: sd = sqrt, rsd = 1/sqrt (LDL:
  // dgl[jp] = dn, rsd = 1/dn)
  auto pivot = [&](int jp, const T& dn) {
    if (!(dn > T(0.0))) fail = jp + 1;
    if constexpr (LDL) {
      dgl[jp] = dn;
      rsd = recip_fast(dn);
    } else {
      pivot_sqrt(dn, sd, rsd);
    }
  };
  if (tid == 0) {
    fail = 0;
    pivot(0, d.A[0]);
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    if (fail) break;
    const T s = sd, rs = rsd;
    // column j of L -> col[] (LDL: of U, and the unscaled column -> colu[]), row j of L^-1 -> row[]
#pragma unroll
    for (int k = 0; k < KA; ++k)
      if (alo[k] <= j && j <= ahi[k] && ac[k] == j) {
        if constexpr (LDL) {
          if (ar[k] > j) {  // (the diagonal keeps d_j; dgl holds it)
            const T u = a[k];
            a[k] = u * rs;
            col[ar[k]] = a[k];
            colu[ar[k]] = u;
          }
        } else {
          const T l = (ar[k] == j) ? s : a[k] * rs;
          a[k] = l;
          col[ar[k]] = l;
        }
      }
    if constexpr (INV) {
#pragma unroll
      for (int k = 0; k < KX; ++k)
        if (xR[k] == (j >> 3) && xr[k] == j && xc[k] <= j) {
          if constexpr (!LDL) x[k] = x[k] * rs;  // (U^-1 has a unit diagonal)
          row[xc[k]] = x[k];
        }
    }
    __syncthreads();
    // trailing update of A and of L^-1
#pragma unroll
    for (int k = 0; k < KA; ++k)
      if (ahi[k] > j && ac[k] > j) a[k] = a[k] - col[ar[k]] * (LDL ? colu : col)[ac[k]];
    if constexpr (INV) {
#pragma unroll
      for (int k = 0; k < KX; ++k)
        if (xR[k] >= 0 && 8 * xC[k] <= j && j < 8 * xR[k] + 7 && xr[k] > j && xc[k] <= j)
          x[k] = x[k] - col[xr[k]] * row[xc[k]];
    }
    // next pivot, by the owner of (j+1, j+1)
    const int jn = j + 1;
    if (jn < n) {
#pragma unroll
      for (int k = 0; k < KA; ++k)
        if (alo[k] <= jn && jn <= ahi[k] && ar[k] == jn && ac[k] == jn) pivot(jn, a[k]);
    }
    __syncthreads();
  }
  if (tid == 0 && info) info[blockIdx.x] = fail;
  if constexpr (LDL) {
    // L = U D^1/2 (column c times sqrt d_c, the diagonal sqrt d_c), L^-1 = D^-1/2 U^-1 (row r
    // times 1/sqrt d_r): the n square roots side by side, into col (sqrt) and row (1/sqrt)
    if (!fail) {
      for (int c = tid; c < n; c += NT) pivot_sqrt(dgl[c], col[c], row[c]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KA; ++k)
      if (ac[k] >= 0) a[k] = (ar[k] == ac[k]) ? col[ac[k]] : a[k] * col[ac[k]];
    if constexpr (INV) {
#pragma unroll
      for (int k = 0; k < KX; ++k)
        if (xr[k] >= 0) x[k] = x[k] * row[xr[k]];
    }
  }
  if constexpr (INV) {
    const MatDesc<T> o = out_inv[blockIdx.x];
#pragma unroll
    for (int k = 0; k < KX; ++k)
      if (xr[k] >= 0) o.A[xr[k] + (size_t)xc[k] * o.lda] = x[k];
    for (int e = tid; e < n * n; e += NT) {  // zeros above the diagonal tiles
      const int r = e % n, c = e / n;
      if ((c >> 3) > (r >> 3)) o.A[r + (size_t)c * o.lda] = T(0.0);
    }
  }
  if (out_l) {
    const MatDesc<T> ol = out_l[blockIdx.x];
#pragma unroll
    for (int k = 0; k < KA; ++k)
      if (ac[k] >= 0) ol.A[ar[k] + (size_t)ac[k] * ol.lda] = a[k];
    for (int e = tid; e < n * n; e += NT) {
      const int r = e % n, c = e / n;
      if (c > r) ol.A[r + (size_t)c * ol.lda] = T(0.0);
    }
  }
}

// chol_lookahead's per-column timestamps (tools/micro/potrf_blk_bench.hip; compiled out in the
// library): [block][wave][column][point]
#ifdef CLRSDP_LA_TRACE
__device__ unsigned long long g_la_trace[64 * 16 * 128 * 4];
#define LA_STAMP(q) do { if (lane == 0 && w < 16 && j < 128 && blockIdx.x < 64 && blockIdx.y == 0) \
  g_la_trace[((blockIdx.x * 16 + w) * 128 + j) * 4 + (q)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define LA_STAMP(q)
#endif
// a - b c in the factorisations' trailing updates: mw::fms_fast at double-double (its bound and
// the reason it suffices there are in mwfloat.h), the plain expression otherwise.
// CLRSDP_FMS_EXACT (compile time) keeps the accurate form everywhere.
template <class T>
__device__ __forceinline__ T fms_upd(const T& a, const T& b, const T& c) { return a - b * c; }
#ifndef CLRSDP_FMS_EXACT
template <>
__device__ __forceinline__ mw::dd fms_upd<mw::dd>(const mw::dd& a, const mw::dd& b, const mw::dd& c) {
  return mw::fms_fast(a, b, c);
}
#endif

// A workgroup barrier that orders LDS only: the waves' outstanding global stores (final L / L^-1
// entries, read by no wave of the launch before a full barrier) are not waited for, as
// __syncthreads' release fence would (s_waitcnt vmcnt(0) on every column's or panel's critical
// path)
__device__ __forceinline__ void lds_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// ------------------------------------------------------------------------------------------
// chol_lookahead: the multi-word potrf (A = L L^T in place, INV = false) of chol_packed with a
// one-column look-ahead, so the serial pivot chain no longer waits for the trailing update.
// 1024 threads: wave 0 is the CHAIN, waves 1..15 the BULK.  Phase j (one barrier each):
//   chain: column j+1 as the bulk published it (updated by columns 0..j-1) minus column j's
//          contribution, its pivot (LDL: d and 1/d by recip_fast; LL^T: sqrt and 1/sqrt by
//          pivot_sqrt), the scaled column j+1 -> LDS (buffer (j+1) & 1) and to the output;
//   bulk:  every element of columns >= j+2 minus column j's contribution (chol_packed's
//          liveness-packed slots, 15 waves), then the owners of column j+2 publish it.
// The chain's step (one multi-word FMA per lane, the pivot, one product per lane) and the bulk's
// update run side by side: a phase costs max(chain, bulk) + one barrier, where chol_packed's
// step costs chain + bulk + two barriers.  Every element sees its terms in the same order as in
// chol_packed (column j's term at step j); the factors agree with chol_packed's to the multi-word
// rounding, not bitwise: at double-double every update is fms_upd's one-two-sum form (round 6),
// and at quad-double with opts bit 1 (the default) the LDL pivot reciprocal takes one Newton
// step from the double-double one (~2^-208 relative instead of chol_packed's ~2^-212)
// (tests/test_gpu_parity.py::test_chol_lookahead_qd_one_newton_step).
// LDL (quad-double): A = U D U^T, then L = U D^1/2 with all n square roots side by side.
// MPMP.jl:1433-1442 / 1499-1505 (the factorisations of S_j and Q; the reference's approx_lu!).
// ------------------------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ T readlane0(const T& v) {
  T o;
  const double* s = reinterpret_cast<const double*>(&v);
  double* d = reinterpret_cast<double*>(&o);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(T) / 8); ++q) d[q] = readlane_d(s[q], 0);
  return o;
}
// The body on one matrix d (in place when ol.A == d.A), callable from other kernels of
// 64 (NW + 1) threads (potrf_blk_update, round 6); returns the failure column + 1 or 0 to
// every thread.
template <class T, bool INV, bool LDL, int NMAX, int NW, bool SKIP0 = false>
__device__ __forceinline__ int chol_lookahead_body(const MatDesc<T>& d, const MatDesc<T>& oi,
                                                   const MatDesc<T>& ol, int opts) {
  // opts (A/B switches): bit 0 = the chain wave at raised issue priority (its SIMD also runs
  // three bulk waves); bit 1 = one Newton step for the pivot's reciprocal (from the
  // double-double one: ~2^-208 relative instead of ~2^-212)
  constexpr int NTH = 64 * (NW + 1);
  constexpr int SA = (NMAX * (NMAX + 1) / 2 + 63) / 64;  // 64-element slots of the triangle
  // SKIP0: the bulk waves on the chain's SIMD (w % 4 == 0) stay idle, the others take their
  // slots -- the chain then issues alone on its SIMD (quad-double: its pivot is thousands of
  // cycles of dependent work, and the three bulk waves beside it finished last)
  constexpr int NWB = SKIP0 ? NW - NW / 4 : NW;  // bulk waves with slots
  constexpr int KA = (SA + NWB - 1) / NWB;
  constexpr int SX = (NMAX / 8) * (NMAX / 8 + 1) / 2;    // 8 x 8 tiles of L^-1
  constexpr int KX = INV ? (SX + NWB - 1) / NWB : 1;
  constexpr int RC = (NMAX + 63) / 64;                   // chain rows per lane
  static_assert(!INV || NMAX <= 64, "the chain holds one row of L^-1 per lane");
  __shared__ T colb[2][NMAX];    // scaled column j (LDL: of U), by parity
  __shared__ T colub[LDL ? 2 : 1][LDL ? NMAX : 1];  // LDL: the unscaled column j
  __shared__ T nextc[2][NMAX];   // column j+1 as the bulk leaves it, by parity
  __shared__ T rowb[INV ? 2 : 1][INV ? NMAX : 1];   // row j of L^-1 (LDL: of U^-1), by parity
  __shared__ T nextr[INV ? 2 : 1][INV ? NMAX : 1];  // row j+1 of L^-1 as the bulk leaves it
  __shared__ T dgl[LDL ? NMAX : 1];
  __shared__ int fail;
  const int n = d.n, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const bool chain = w == 0;
  const bool idle = chain || (SKIP0 && (w & 3) == 0);
  const int wb = SKIP0 ? w - 1 - (w >> 2) : w - 1;  // rank among the bulk waves with slots
  auto wave_max = [](int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return __builtin_amdgcn_readfirstlane(v);
  };
  // ---- bulk slots of A: slot wb + NW k, element e = 64 slot + lane of the column-major triangle
  T a[KA];
  int ar[KA], ac[KA], alo[KA], ahi[KA];
  const int ne = n * (n + 1) / 2;
#pragma unroll
  for (int k = 0; k < KA; ++k) {
    const int e = 64 * (wb + NWB * k) + lane;
    int r = -1, c = -1;
    if (!idle && e < ne) {
      int rem = e;
      c = 0;
      while (rem >= n - c) {
        rem -= n - c;
        ++c;
      }
      r = c + rem;
    }
    ar[k] = r;
    ac[k] = c;
    a[k] = T(0.0);
    if (c >= 0) a[k] = d.A[r + (size_t)c * d.lda];
    ahi[k] = idle ? -1 : wave_max(c);
    alo[k] = idle ? NMAX : -wave_max(c >= 0 ? -c : -NMAX);
  }
  // ---- bulk tiles of L^-1 (chol_packed's 8 x 8 tiles, R >= C), identity to start
  T x[KX];
  int xr[KX], xc[KX], xR[KX], xC[KX];
  if constexpr (INV) {
    const int nt8 = (n + 7) / 8;
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      int t = wb + NWB * k, C = 0;
      bool tv = !idle;
      if (tv) {
        while (C < nt8 && t >= nt8 - C) {
          t -= nt8 - C;
          ++C;
        }
        tv = C < nt8;
      }
      const int R = C + t;
      xR[k] = tv ? R : -1;
      xC[k] = tv ? C : 0;
      const int r = 8 * R + (lane & 7), c = 8 * C + (lane >> 3);
      const bool v = tv && r < n && c < n;
      xr[k] = v ? r : -1;
      xc[k] = v ? c : NMAX;
      x[k] = T((v && r == c) ? 1.0 : 0.0);
    }
  }
  // chain: the pivot of column c from the updated column cv (row c in lane 0), the scaled
  // column to colb / colub (buffer q) and to L
  T cv[RC];
  auto chain_column = [&](int c, int q) {
    const T dn = readlane0(cv[0]);
    T s, rs;
    if constexpr (LDL) {
      if constexpr (std::is_same<T, mw::qd>::value) {
        if (opts & 2) {
          rs = recip_qd_newton1(dn);
        } else {
          rs = recip_fast(dn);
        }
      } else {
        rs = recip_fast(dn);
      }
    } else {
      pivot_sqrt(dn, s, rs);
    }
#pragma unroll
    for (int u = 0; u < RC; ++u) {
      const int r = c + lane + 64 * u;
      if (r < n) {
        T o;
        if constexpr (LDL) {
          o = r == c ? dn : cv[u] * rs;
          colub[q][r] = cv[u];
        } else {
          o = r == c ? s : cv[u] * rs;
        }
        colb[q][r] = o;
        if (ol.A) ol.A[r + (size_t)c * ol.lda] = o;
      }
    }
    if (lane == 0) {
      if constexpr (LDL) dgl[c] = dn;
      if (!(dn > T(0.0))) fail = c + 1;
    }
    return rs;
  };
  // chain: row c of L^-1 (lane = column index <= c) scaled by the pivot's 1/sqrt (LL^T; U^-1 has
  // a unit diagonal) -> rowb (buffer q) and the output
  auto chain_row = [&](int c, int q, T xv, const T& rs) {
    if constexpr (INV) {
      if (lane <= c) {
        if constexpr (!LDL) xv = xv * rs;
        rowb[q][lane] = xv;
        oi.A[c + (size_t)lane * oi.lda] = xv;
      }
    }
  };
  // ---- phase -1: the chain factors column 0 (and row 0 of L^-1), the bulk publishes column 1
  // and row 1
  if (chain) {
    if (opts & 1) __builtin_amdgcn_s_setprio(3);
    if (lane == 0) fail = 0;
#pragma unroll
    for (int u = 0; u < RC; ++u) {
      const int r = lane + 64 * u;
      cv[u] = r < n ? d.A[r] : T(0.0);
    }
    const T rs = chain_column(0, 0);
    chain_row(0, 0, T(1.0), rs);
  } else {
#pragma unroll
    for (int k = 0; k < KA; ++k)
      if (alo[k] <= 1 && 1 <= ahi[k] && ac[k] == 1) nextc[1][ar[k]] = a[k];
    if constexpr (INV) {
#pragma unroll
      for (int k = 0; k < KX; ++k)
        if (xR[k] == 0 && xr[k] == 1) nextr[1][xc[k]] = x[k];
    }
  }
  lds_barrier();  // (the chain's L / L^-1 stores are read back only after the loop's full barrier)
  for (int j = 0; j + 1 < n; ++j) {
    LA_STAMP(0);
    if (fail) break;
    const int p = j & 1, p1 = (j + 1) & 1;
    if (chain) {
      // column j+1 (and row j+1 of L^-1): the published values minus step j's term, the pivot
      const int c = j + 1;
      const T cuj = LDL ? colub[p][c] : colb[p][c];
#pragma unroll
      for (int u = 0; u < RC; ++u) {
        const int r = c + lane + 64 * u;
        cv[u] = r < n ? fms_upd(nextc[p1][r], colb[p][r], cuj) : T(0.0);
      }
      T xv = T(0.0);
      if constexpr (INV) {
        if (lane <= c) xv = lane <= j ? fms_upd(nextr[p1][lane], colb[p][c], rowb[p][lane]) : T(1.0);
      }
      LA_STAMP(1);
      const T rs = chain_column(c, p1);
      LA_STAMP(2);
      chain_row(c, p1, xv, rs);
      LA_STAMP(3);
    } else {
      // columns >= j+2 (and rows >= j+2 of L^-1) minus step j's term; then the owners of
      // column j+2 (and of row j+2) publish it
#pragma unroll
      for (int k = 0; k < KA; ++k)
        if (ahi[k] >= j + 2 && ac[k] >= j + 2)
          a[k] = fms_upd(a[k], colb[p][ar[k]], (LDL ? colub[p] : colb[p])[ac[k]]);
      if constexpr (INV) {
#pragma unroll
        for (int k = 0; k < KX; ++k)
          if (xR[k] >= 0 && 8 * xC[k] <= j && j + 2 <= 8 * xR[k] + 7 && xr[k] >= j + 2 && xc[k] <= j)
            x[k] = fms_upd(x[k], colb[p][xr[k]], rowb[p][xc[k]]);
      }
      const int c2 = j + 2;
      if (c2 < n) {
#pragma unroll
        for (int k = 0; k < KA; ++k)
          if (alo[k] <= c2 && c2 <= ahi[k] && ac[k] == c2) nextc[p][ar[k]] = a[k];
        if constexpr (INV) {
#pragma unroll
          for (int k = 0; k < KX; ++k)
            if (xR[k] == (c2 >> 3) && xr[k] == c2) nextr[p][xc[k]] = x[k];
        }
      }
      LA_STAMP(3);
    }
    lds_barrier();
  }
  __syncthreads();
  const int failed = fail;
  if constexpr (LDL) {
    // L = U D^1/2 (column c times sqrt d_c, the diagonal sqrt d_c); L^-1 = D^-1/2 U^-1 (row r
    // times 1/sqrt d_r): the n square roots side by side
    if (!failed) {
      for (int c = tid; c < n; c += NTH) {
        T sq, rq;
        pivot_sqrt(dgl[c], sq, rq);
        colb[0][c] = sq;
        colb[1][c] = rq;
      }
    }
    __syncthreads();
    if (!failed)
      for (int e = tid; e < n * n; e += NTH) {
        const int r = e % n, c = e / n;
        if (ol.A) {
          if (r > c) ol.A[r + (size_t)c * ol.lda] = ol.A[r + (size_t)c * ol.lda] * colb[0][c];
          else if (r == c) ol.A[r + (size_t)c * ol.lda] = colb[0][c];
        }
        if constexpr (INV) {
          if (r >= c) oi.A[r + (size_t)c * oi.lda] = oi.A[r + (size_t)c * oi.lda] * colb[1][r];
        }
      }
  }
  for (int e = tid; e < n * n; e += NTH) {  // zeros above the diagonal
    const int r = e % n, c = e / n;
    if (c > r) {
      if (ol.A) ol.A[r + (size_t)c * ol.lda] = T(0.0);
      if constexpr (INV) oi.A[r + (size_t)c * oi.lda] = T(0.0);
    }
  }
  return failed;
}
template <class T, bool INV, bool LDL, int NMAX, int NW = 15, bool SKIP0 = false>  // NW bulk waves
__global__ __launch_bounds__(64 * (NW + 1)) void chol_lookahead(const MatDesc<T>* __restrict__ in,
                                                       const MatDesc<T>* __restrict__ out_inv,
                                                       const MatDesc<T>* __restrict__ out_l,
                                                       int* __restrict__ info, int opts = 0) {
  const MatDesc<T> d = in[blockIdx.x];
  const MatDesc<T> ol = out_l ? out_l[blockIdx.x] : MatDesc<T>{nullptr, 0, 0};
  const MatDesc<T> oi = INV ? out_inv[blockIdx.x] : MatDesc<T>{nullptr, 0, 0};
  const int f = chol_lookahead_body<T, INV, LDL, NMAX, NW, SKIP0>(d, oi, ol, opts);
  if (threadIdx.x == 0 && info) info[blockIdx.x] = f;
}

// ------------------------------------------------------------------------------------------
// Blocked multi-word potrf across workgroups (round 6).  chol_lookahead keeps a whole block on
// one CU: at C4 (16 Schur blocks of 127, double-double) 16 of 256 CUs run the ~n^3/6 trailing
// update and a column costs ~1.8 us (the bulk's multi-word FMAs, not the pivot chain).  Here
// the block is cut into NB-column panels k (k0 = NB k) and each panel costs three steps, the
// last two spread over many workgroups:
//   diag  (1 WG / matrix): L_kk and L_kk^-1 of the (updated) NB x NB diagonal block
//         (chol_lookahead_body, 256 threads);
//   trsm  (rows / 16 WGs): the panel below it, L_ik = A_ik L_kk^-T (a product with L_kk^-1 in
//         LDS, no serial chain), and zeros in the block row above the diagonal;
//   update(lower 16 x 16 tiles of the trailing matrix): A_ij -= L_ik L_jk^T; the workgroup 0 of
//         each matrix updates the next diagonal block itself and goes straight on to its diag
//         step, so one launch does both (update k + diag k+1).
// Launches for n = 127, NB = 32: diag, trsm, {update, diag} x 3 with trsm between = 7.  The
// factor is LL^T with every element's panel contributions summed panel by panel (a different
// order from chol_lookahead's column by column: agreement to the multi-word rounding, not bitwise).
// MPMP.jl:1433-1442 (the factorisation of S_j).
// ------------------------------------------------------------------------------------------
template <class T>
struct BlkPotrfDesc {
  T* A;      // the matrix (column-major, lower triangle in, L out, zeros above)
  T* Linv;   // NB x NB scratch: L_kk^-1 of the current panel (ld NB)
  int n, lda;
};

// the diagonal step of panel k (k0 = NB k) on matrix m: L_kk, L_kk^-1; failure -> info[m]
template <class T, bool LDL, int NB>
__device__ __forceinline__ void potrf_blk_diag(const BlkPotrfDesc<T>& b, int k0, int* info, int m,
                                               int opts) {
  const int nb = min(NB, b.n - k0);
  const MatDesc<T> dk{b.A + k0 + (size_t)k0 * b.lda, nb, b.lda};
  const MatDesc<T> oi{b.Linv, nb, NB};
  const int f = chol_lookahead_body<T, true, LDL, NB, 3>(dk, oi, dk, opts);
  if (threadIdx.x == 0 && info && f) info[m] = k0 + f;
}

template <class T, bool LDL, int NB>
__global__ __launch_bounds__(256) void potrf_blk_first(const BlkPotrfDesc<T>* __restrict__ bd,
                                                       int* __restrict__ info, int opts) {
  const BlkPotrfDesc<T> b = bd[blockIdx.x];
  if (threadIdx.x == 0 && info) info[blockIdx.x] = 0;
  __syncthreads();
  potrf_blk_diag<T, LDL, NB>(b, 0, info, blockIdx.x, opts);
}

// trsm of panel k: blockIdx.y = matrix, blockIdx.x = 16-row chunk of rows k0 + NB .. n-1
// (chunk 0 also zeros the NB rows k0.. above the diagonal in the columns right of the panel)
template <class T, int NB>
__global__ __launch_bounds__(256) void potrf_blk_trsm(const BlkPotrfDesc<T>* __restrict__ bd, int k0) {
  const BlkPotrfDesc<T> b = bd[blockIdx.y];
  const int r0 = k0 + NB + 16 * blockIdx.x, tid = threadIdx.x;
  if (blockIdx.x == 0)
    for (int e = tid; e < NB * max(0, b.n - k0 - NB); e += 256) {
      const int r = k0 + e % NB, c = k0 + NB + e / NB;
      if (r < b.n) b.A[r + (size_t)c * b.lda] = T(0.0);
    }
  if (r0 >= b.n) return;
  __shared__ T li[NB][NB + 1];  // L_kk^-1, [c][t]
  __shared__ T ar[NB][17];      // the 16 rows of A_ik, [t][row]
  for (int e = tid; e < NB * NB; e += 256) {
    const int c = e % NB, t = e / NB;
    li[c][t] = b.Linv[c + (size_t)t * NB];
  }
  for (int e = tid; e < NB * 16; e += 256) {
    const int rr = e % 16, t = e / 16;
    ar[t][rr] = r0 + rr < b.n ? b.A[r0 + rr + (size_t)(k0 + t) * b.lda] : T(0.0);
  }
  __syncthreads();
  const int rr = tid % 16;
  for (int c = tid / 16; c < NB; c += 16) {  // L_ik[r, c] = sum_{t <= c} A_ik[r, t] L_kk^-1[c, t]
    T acc = T(0.0);
    for (int t = 0; t <= c; ++t) acc = fms_upd(acc, -ar[t][rr], li[c][t]);
    if (r0 + rr < b.n && k0 + c < b.n) b.A[r0 + rr + (size_t)(k0 + c) * b.lda] = acc;
  }
}

// update of panel k (A_ij -= L_ik L_jk^T over the lower 16 x 16 tiles of rows / columns
// k1 = k0 + NB .. n-1) fused with the diagonal step of panel k+1: blockIdx.y = matrix,
// blockIdx.x = 0 updates the diagonal block k+1 and factors it, blockIdx.x >= 1 the other tiles
// (lower tiles (I, J), I >= J, of the trailing matrix, the ones inside the diagonal block skipped)
template <class T, bool LDL, int NB>
__global__ __launch_bounds__(256) void potrf_blk_update(const BlkPotrfDesc<T>* __restrict__ bd,
                                                        int k0, int* __restrict__ info, int opts) {
  const BlkPotrfDesc<T> b = bd[blockIdx.y];
  const int k1 = k0 + NB, tid = threadIdx.x;
  if (k1 >= b.n) return;
  __shared__ T lr[NB][17], lc[NB][17];  // rows of L_ik, L_jk: [t][row]
  const int ntr = (b.n - k1 + 15) / 16;  // 16-tiles of the trailing matrix
  constexpr int DT = NB / 16;            // 16-tiles per diagonal block
  auto upd_tile = [&](int I, int J) {    // tile (I, J) of the trailing matrix, I >= J
    const int ri = k1 + 16 * I, cj = k1 + 16 * J;
    for (int e = tid; e < NB * 16; e += 256) {
      const int rr = e % 16, t = e / 16;
      lr[t][rr] = ri + rr < b.n ? b.A[ri + rr + (size_t)(k0 + t) * b.lda] : T(0.0);
      lc[t][rr] = cj + rr < b.n ? b.A[cj + rr + (size_t)(k0 + t) * b.lda] : T(0.0);
    }
    __syncthreads();
    const int rr = tid % 16, cc = tid / 16, r = ri + rr, c = cj + cc;
    if (r < b.n && c < b.n && r >= c) {
      T acc = b.A[r + (size_t)c * b.lda];
#pragma unroll 8
      for (int t = 0; t < NB; ++t) acc = fms_upd(acc, lr[t][rr], lc[t][cc]);
      b.A[r + (size_t)c * b.lda] = acc;
    }
    __syncthreads();
  };
  if (blockIdx.x == 0) {
    for (int I = 0; I < DT && I < ntr; ++I)
      for (int J = 0; J <= I; ++J) upd_tile(I, J);
    potrf_blk_diag<T, LDL, NB>(b, k1, info, blockIdx.y, opts);
    return;
  }
  // tile index q = blockIdx.x - 1 over the lower tiles outside the diagonal block, row by row
  int q = blockIdx.x - 1, I = DT, J = 0;
  int before = DT * (DT + 1) / 2;  // tiles of rows < DT (all inside the diagonal block)
  // rows I >= DT hold I + 1 tiles each
  int rem = q;
  I = DT;
  while (I < ntr && rem >= I + 1) {
    rem -= I + 1;
    ++I;
  }
  (void)before;
  if (I >= ntr) return;
  J = rem;
  upd_tile(I, J);
}

// ------------------------------------------------------------------------------------------
// Double-double GEMM on the int8 matrix cores (Ozaki scheme; round 6, the Schur products of
// multi-word m = 1 blocks).  Every row of op(A) is scaled by 2^-E (|a| 2^-E < 1/2) and written as
// OZ_S base-2^7 digits d_p in [-64, 64], each the rounded leading part of the exact double-double
// remainder:  a = 2^E sum_{p < OZ_S} d_p 2^-7(p+1)  (every column of op(B) likewise, 2^F).  Then
//     (op(A) op(B))_ij = 2^(E_i + F_j) sum_L 2^-7(L+2) sum_{p+q=L} (D_p G_q)_ij ,
// every level-L sum of int8 products accumulates exactly in int32 (|.| <= 16 Kpad 64^2 < 2^31 for
// Kpad < 2^15) on v_mfma_i32_16x16x64_i8 and converts exactly to fp64; the OZ_S levels are summed
// in double-double, smallest first.  Levels L >= OZ_S are dropped: ~2^-7 OZ_S = 2^-112 relative
// to 2^(E_i + F_j) K -- a row / column-normwise bound, where the VALU GEMM's is componentwise.
// 136 int8 MFMAs per 16 x 16 tile and 64-k chunk against 64 double-double FMAs per output and k
// on the VALU: 9.1 against 15.0 us for 16 products 64 x 64 @ 64 x 128, 15.1 against 43.0 us for
// 64 (tools/micro/ozaki_dd_bench.hip, same accuracy against a host double-double reference).
// Digit planes: D[(p * Rpad + v) * Kpad + k] (int8, zero-padded: the buffers are zeroed once and
// the split writes only v < nv, k < K).
// (Ozaki, Ogita, Oishi & Rump, Numer. Algorithms 59 (2012); integer slices as in Ootomo, Ozaki &
// Yokota, IJHPCA 38 (2024).)
// ------------------------------------------------------------------------------------------
constexpr int OZ_S = 16;
typedef int oz_v4i __attribute__((ext_vector_type(4)));
struct OzSplitDesc {
  const mw::dd* X;     // vector v, element k at X[v * sv + k * sk]
  long long sv, sk;
  signed char* D;      // digit planes, [OZ_S][Rpad][Kpad]
  int* E;              // per-vector exponent
  int nv, K, Rpad, Kpad;
};
// one wave per vector (4 per workgroup); t2d: TileRef{desc, group of 4 vectors}
__global__ __launch_bounds__(256) void oz_split(const OzSplitDesc* __restrict__ descs,
                                                const TileRef* __restrict__ t2d) {
  const TileRef tr = t2d[blockIdx.x];
  const OzSplitDesc d = descs[tr.p];
  const int v = 4 * tr.t + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (v >= d.nv) return;
  const mw::dd* x = d.X + (size_t)v * d.sv;
  int ex = -1100;
  for (int k = lane; k < d.K; k += 64) {
    const double h = x[(size_t)k * d.sk].hi;
    if (h != 0.0) ex = max(ex, ilogb(h));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ex = max(ex, __shfl_xor(ex, o));
  const int E = ex + 2;  // |x| < 2^(ex+1) = 2^E / 2
  for (int k = lane; k < d.K; k += 64) {
    const mw::dd a = x[(size_t)k * d.sk];
    double h = ldexp(a.hi, -E), l = ldexp(a.lo, -E);
    signed char* out = d.D + (size_t)v * d.Kpad + k;
#pragma unroll
    for (int p = 0; p < OZ_S; ++p) {
      h *= 128.0;
      l *= 128.0;
      const double dg = rint(h);
      double e;
      h = mw::two_sum(h - dg, l, e);  // (h - dg is exact: |h - dg| <= 1/2 on h's grid)
      l = e;
      out[(size_t)p * d.Rpad * d.Kpad] = (signed char)(int)dg;
    }
  }
  if (lane == 0) d.E[v] = E;
}
struct OzGemmDesc {
  const signed char* DA;  // rows of op(A): [OZ_S][RpadA][Kpad]
  const int* EA;
  const signed char* DB;  // columns of op(B): [OZ_S][RpadB][Kpad]
  const int* EB;
  mw::dd* C;              // M x N, ld ldc:  C = op(A) op(B)
  int RpadA, RpadB, Kpad, ldc, M, N, tn, pad;
};
// one wave per 16 x 16 output tile (tile t: rows 16 (t / tn), columns 16 (t % tn)), 4 per
// workgroup; t2d: TileRef{desc, tile} by groups of 4 consecutive entries per workgroup
__global__ __launch_bounds__(256) void oz_gemm(const OzGemmDesc* __restrict__ descs,
                                               const TileRef* __restrict__ t2d, int ntiles) {
  const int wi = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (wi >= ntiles) return;
  const TileRef tr = t2d[wi];
  const OzGemmDesc d = descs[tr.p];
  const int r0 = 16 * (tr.t / d.tn), c0 = 16 * (tr.t % d.tn);
  const size_t pa = (size_t)d.RpadA * d.Kpad, pb = (size_t)d.RpadB * d.Kpad;
  const signed char* ra = d.DA + (size_t)(r0 + (l & 15)) * d.Kpad + 16 * (l >> 4);
  const signed char* rb = d.DB + (size_t)(c0 + (l & 15)) * d.Kpad + 16 * (l >> 4);
  oz_v4i acc[OZ_S];
#pragma unroll
  for (int L = 0; L < OZ_S; ++L) acc[L] = oz_v4i{0, 0, 0, 0};
  for (int k0 = 0; k0 < d.Kpad; k0 += 64) {
    oz_v4i a[OZ_S], b[OZ_S];
#pragma unroll
    for (int p = 0; p < OZ_S; ++p) {
      a[p] = *reinterpret_cast<const oz_v4i*>(ra + p * pa + k0);
      b[p] = *reinterpret_cast<const oz_v4i*>(rb + p * pb + k0);
    }
#pragma unroll
    for (int L = 0; L < OZ_S; ++L)
#pragma unroll
      for (int p = 0; p <= L; ++p) acc[L] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[p], b[L - p], acc[L], 0, 0, 0);
  }
  // C/D layout: column l & 15, row 4 (l >> 4) + r
  const int col = c0 + (l & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double hi = 0.0, lo = 0.0;
#pragma unroll
    for (int L = OZ_S - 1; L >= 0; --L) {  // smallest level first; every term exact in fp64
      double e;
      hi = mw::two_sum(hi, ldexp((double)acc[L][r], -7 * (L + 2)), e);
      lo += e;
    }
    const int row = r0 + 4 * (l >> 4) + r;
    if (row < d.M && col < d.N) {
      double e;
      const double h = mw::quick_two_sum(hi, lo, e);
      const int sc = d.EA[row] + d.EB[col];
      d.C[row + (size_t)col * d.ldc] = mw::dd(ldexp(h, sc), ldexp(e, sc));
    }
  }
}

// ------------------------------------------------------------------------------------------
// eigmin_lds: smallest eigenvalue of a symmetric matrix (n <= NMAX), 512 threads.  The matrix
// is symmetrised into LDS (ld = n), tridiagonalised by Householder reflections (full storage),
// then one wave runs a 64-point Sturm multisection.
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// eigmin_reg: lambda_min of a symmetric n <= 128 fp64 block with the matrix held in REGISTERS
// (replaces approx_eig_qr! in compute_step_length, MPMP.jl:1857-1860).  The input must be exactly
// symmetric (every caller's block comes from the symmetric GEMM epilogue).  512 threads; wave w
// owns row block rb(w) (rows 16 rb..16 rb+15, lane r = l & 15), lane class c = l >> 4 owns the column pairs
// j = 2c + 8s + {0,1}, s = 0..15 (fixed slots): 32 entries per thread.  Householder
// tridiagonalisation with ONE barrier per column k:
//   p_i = sum_j A_ij v_j in registers (+ 2 swaps across the column classes), per-wave v^T p to
//   LDS                                                                             -- barrier
//   w = beta p - K v; A -= v w^T + w v^T in registers; meanwhile every wave recomputes row k+1
//   of the updated matrix from the copy its owners published a step earlier (the owners' own
//   operations, so bitwise their registers) and builds the next reflector from it redundantly
//   (wave reduction, no barrier); the owners of row k+2 publish it for the step after next.
// The 16 lanes of a DPP row share a column class and so need the same 32 values of v and of p:
// lane t of the row reads only slot t and every FMA takes slot s from lane s by row_newbcast
// (v_fmac_f64_dpp).  Slots whose 8 columns are all <= k are skipped in groups of 4 by a uniform
// branch; the slots never move, so the loop carries no register copies.
// Then 512-way multisection with Sturm counts on the tridiagonal matrix.
// ------------------------------------------------------------------------------------------
// Compile-time loop (the DPP lane selector of row_newbcast is an instruction immediate).
template <int K, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (K < E) {
    f(std::integral_constant<int, K>{});
    static_for<K + 1, E>(f);
  }
}
// acc += src[lane J of this lane's 16-lane DPP row] * mul: one v_fmac_f64_dpp with
// row_newbcast (the f64 DPP form of CDNA3/4; the builtin route costs a copy + v_mov_b64_dpp +
// v_fma_f64 and serialises on the copy register).  A DPP source needs 2 wait states after a
// VALU write, which the compiler does not see inside inline asm: NOP = true puts an s_nop 1
// in front.  The statements are volatile, so they keep their program order among themselves.
template <int J, bool NOP>
__device__ __forceinline__ void fmac_bcast(double& acc, double src, double mul) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "n"(J));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "n"(J));
}

#ifdef CLRSDP_EIGREG_STAMPS
__device__ unsigned long long g_eigreg_stamps[8];
#endif
// Sturm count of the symmetric tridiagonal (dg, e2 = squared off-diagonals) below sigma, with a
// Newton-refined hardware reciprocal instead of the IEEE division (only signs are used) and
// the coefficients read two at a time.
__device__ inline int sturm_count_fast(const double* dg, const double* e2, int n, double sigma) {
  int cnt = 0;
  double q = dg[0] - sigma;
  cnt += q < 0.0;
  int i = 1;
  for (; i + 1 < n; i += 2) {
    const double d0 = dg[i], d1 = dg[i + 1], f0 = e2[i - 1], f1 = e2[i];
    q = q == 0.0 ? 1e-300 : q;
    double r = __builtin_amdgcn_rcp(q);
    r = fma(fma(-q, r, 1.0), r, r);
    r = fma(fma(-q, r, 1.0), r, r);
    q = (d0 - sigma) - f0 * r;
    cnt += q < 0.0;
    q = q == 0.0 ? 1e-300 : q;
    r = __builtin_amdgcn_rcp(q);
    r = fma(fma(-q, r, 1.0), r, r);
    r = fma(fma(-q, r, 1.0), r, r);
    q = (d1 - sigma) - f1 * r;
    cnt += q < 0.0;
  }
  for (; i < n; ++i) {
    q = q == 0.0 ? 1e-300 : q;
    double r = __builtin_amdgcn_rcp(q);
    r = fma(fma(-q, r, 1.0), r, r);
    r = fma(fma(-q, r, 1.0), r, r);
    q = (dg[i] - sigma) - e2[i - 1] * r;
    cnt += q < 0.0;
  }
  return cnt;
}

// Is lambda_min < sigma?  The multisection only needs "count >= 1", and with p_0 = 1 > 0 the
// Sturm sequence of leading principal minors has a sign change iff some minor is negative, so
// the count becomes an OR of sign bits: per row one FMA on the chain (e_{i-1} p_{i-2} is formed a
// row ahead), one subtraction, one multiplication and one integer OR; no compares, selects or
// branches.  sd/se are the padded arrays of eigmin_reg (nr a multiple of 8, se[i] = e2_{i-1} > 0
// inside the matrix, so a zero minor is followed by a nonzero one of the opposite sign of its
// predecessor and the sign test stays exact); (p_{i-1}, p_i) is rescaled by a power of two every
// 8 rows.
__device__ inline bool sturm_any_below(const double* __restrict__ sd, const double* __restrict__ se,
                                       int nr, double sigma) {
  double pm = 0.0, pc = 1.0;
  int acc = 0;
  for (int i0 = 0; i0 < nr; i0 += 8) {
    double dv[8], ev[8];
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      const double2 a = *reinterpret_cast<const double2*>(sd + i0 + u);
      const double2 b = *reinterpret_cast<const double2*>(se + i0 + u);
      dv[u] = a.x; dv[u + 1] = a.y;
      ev[u] = b.x; ev[u + 1] = b.y;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double pn = fma(dv[u] - sigma, pc, -(ev[u] * pm));
      acc |= __double2hiint(pn);
      pm = pc;
      pc = pn;
    }
    const int ex = __builtin_amdgcn_frexp_exp(pc);
    pc = __builtin_ldexp(pc, -ex);
    pm = __builtin_ldexp(pm, -ex);
  }
  return acc < 0;
}

// The same test with the chain split in two (round 4): leading principal minors p_i of rows
// [0, h) top-down and trailing minors q_i of rows [h, nr) bottom-up, two independent recurrences
// (the count is latency-bound: each row is one dependent FMA chain link), joined by
// det(T - sigma I) = p_{h-1} q_h - e2_{h-1} p_{h-2} q_{h+1}.  With the twisted factorisation
// N D N^T of T - sigma I at row h (Sylvester), lambda_min < sigma iff some p_i < 0 (i < h), some
// q_i < 0 (i >= h) or det < 0 (the twist pivot has the sign of det when p_{h-1}, q_h > 0).  Both
// chains rescale by powers of two every 8 rows; det's three terms carry one p and one q factor
// each, so the scales agree.
__device__ inline bool sturm_any_below2(const double* __restrict__ sd, const double* __restrict__ se,
                                        int nr, double sigma) {
  const int h = 8 * ((nr >> 3) >> 1);
  double pm = 0.0, pc = 1.0;  // p_{i-2}, p_{i-1}
  double qm = 0.0, qc = 1.0;  // q_{i+2}, q_{i+1}
  int acc = 0;
  const int nb = nr - h, nt = h;
  const int nmax = nb > nt ? nb : nt;
  for (int g = 0; g < nmax; g += 8) {
    double dt[8], et[8], db[8], eb[8];
    const bool top = g < nt;
    const int ib = nr - 8 - g;  // rows ib..ib+7 of the bottom chain, walked downwards
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      if (top) {
        const double2 a = *reinterpret_cast<const double2*>(sd + g + u);
        const double2 b = *reinterpret_cast<const double2*>(se + g + u);
        dt[u] = a.x; dt[u + 1] = a.y;
        et[u] = b.x; et[u + 1] = b.y;
      }
      const double2 c = *reinterpret_cast<const double2*>(sd + ib + u);
      // q_i couples to row i+1 through e2_i = se[i+1]
      const double2 e = *reinterpret_cast<const double2*>(se + ib + u);
      db[u] = c.x; db[u + 1] = c.y;
      eb[u] = e.y;
      eb[u + 1] = (u + 2 < 8) ? se[ib + u + 2] : (ib + 8 < nr + 0 ? se[ib + 8] : 0.0);
    }
    if (top) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double pn = fma(dt[u] - sigma, pc, -(et[u] * pm));
        acc |= __double2hiint(pn);
        pm = pc;
        pc = pn;
      }
      const int ex = __builtin_amdgcn_frexp_exp(pc);
      pc = __builtin_ldexp(pc, -ex);
      pm = __builtin_ldexp(pm, -ex);
    }
    if (g < nb) {
#pragma unroll
      for (int u = 7; u >= 0; --u) {
        const double qn = fma(db[u] - sigma, qc, -(eb[u] * qm));
        acc |= __double2hiint(qn);
        qm = qc;
        qc = qn;
      }
      const int ex = __builtin_amdgcn_frexp_exp(qc);
      qc = __builtin_ldexp(qc, -ex);
      qm = __builtin_ldexp(qm, -ex);
    }
  }
  // p_{h-1} = pc, p_{h-2} = pm; q_h = qc, q_{h+1} = qm; e2_{h-1} = se[h]
  const double det = fma(pc, qc, -(se[h] * pm * qm));
  acc |= __double2hiint(det);
  return acc < 0;
}

// NWV waves (8: one row block per wave, two waves per SIMD; 4: two row blocks per lane, one wave
// per SIMD, so the redundant per-column reflector chain costs each SIMD half the issue slots).
template <int DBG = 0, int NWV = 8>  // DBG (timing experiments only): 1 = no update FMAs, 2 = no matvec FMAs
__global__ __launch_bounds__(64 * NWV) void eigmin_reg(const MatDesc<double>* __restrict__ descs,
                                                        double* __restrict__ out) {
  constexpr int NS = 16, RPL = 8 / NWV;
#ifdef CLRSDP_EIGREG_STAMPS
  unsigned long long t_prev = __builtin_amdgcn_s_memtime();
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define ER_STAMP(slot) { unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[slot] += t_ - t_prev; t_prev = t_; }
#else
#define ER_STAMP(slot)
#endif
  // rowb[r&1] = row r of the matrix before the step that reflects column r-1 (published by the
  // lanes that own it); pb[k&1] = p = A'v of step k (inactive rows zero); vb[k&1] = v of step k;
  // redw[k&1] = the per-wave parts of v^T p.  Every buffer alternates between two copies, so one
  // barrier per column separates each write from the reads of the copy it replaces.
  __shared__ __attribute__((aligned(16))) double rowb[2][128];
  __shared__ __attribute__((aligned(16))) double pb[2][128];
  __shared__ __attribute__((aligned(16))) double vb[2][128];
  __shared__ __attribute__((aligned(16))) double redw[2][8];
  __shared__ double dg[128], e2[128];
  __shared__ __attribute__((aligned(16))) double sd[128], se[128];
  __shared__ double bnd[2];
  __shared__ unsigned long long masks[8];
  const MatDesc<double> d = descs[blockIdx.x];
  const int n = d.n, lda = d.lda, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  // row blocks of the lanes of wave w, paired so that every SIMD carries blocks that go idle
  // early and late (0/7, 1/6, 2/5, 3/4): NWV = 8, waves w and w+4 share a SIMD; NWV = 4, one
  // wave holds both blocks
  int blk[RPL];
  if constexpr (RPL == 1) {
    blk[0] = w < 4 ? w : 11 - w;
  } else {
    blk[0] = w;
    blk[1] = 7 - w;
  }
  const int c = lane >> 4, t16 = lane & 15;
  // the wave that holds the block of row n-1 (live to the last column) writes v, the diagonal
  // and the off-diagonal of every step; a wave with no row in (k+1, n) skips the reflector and
  // the update of step k (its rows are never read again, or are padding)
  bool writer = false;
#pragma unroll
  for (int h = 0; h < RPL; ++h) writer = writer || blk[h] == ((n - 1) >> 4);
  int i[RPL];
#pragma unroll
  for (int h = 0; h < RPL; ++h) i[h] = blk[h] * 16 + t16;
  // a[h][s][e] = A(i_h, 2c + 8s + e).  The input is exactly symmetric (the step-length product
  // is written by the symmetric GEMM epilogue), so only coalesced A(i, j) loads are needed.
  double a[RPL][NS][2];
#pragma unroll
  for (int h = 0; h < RPL; ++h)
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * c + 8 * s + e;
        const int ic = min(i[h], n - 1), jc = min(j, n - 1);  // unconditional loads, masked after
        const double v = gload(d.A + ic + (size_t)jc * lda);
        a[h][s][e] = (i[h] < n && j < n) ? v : 0.0;
      }
  // scale the block by 2^-ex0 so that its largest entry lies in [0.5, 1): the column norms of the
  // Householder reduction neither overflow nor underflow for any block norm in fp64 range (exact,
  // undone on the result)
  int ex0 = 0;
  {
    double amax = 0.0;
#pragma unroll
    for (int h = 0; h < RPL; ++h)
#pragma unroll
      for (int s = 0; s < NS; ++s) amax = fmax(amax, fmax(fabs(a[h][s][0]), fabs(a[h][s][1])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
    if (lane == 0) redw[0][w] = amax;
    __syncthreads();
    amax = redw[0][0];
#pragma unroll
    for (int r = 1; r < NWV; ++r) amax = fmax(amax, redw[0][r]);
    ex0 = (amax > 0.0 && amax < INFINITY) ? __builtin_amdgcn_frexp_exp(amax) : 0;
#pragma unroll
    for (int h = 0; h < RPL; ++h)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        a[h][s][0] = __builtin_ldexp(a[h][s][0], -ex0);
        a[h][s][1] = __builtin_ldexp(a[h][s][1], -ex0);
      }
  }
  // the owners of row r (lane r & 15 of every class, in the wave holding block r >> 4) write all
  // 32 entries
  auto publish_row = [&](int r, double* dst) {
#pragma unroll
    for (int h = 0; h < RPL; ++h)
      if (blk[h] == (r >> 4) && t16 == (r & 15)) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
          *reinterpret_cast<double2*>(dst + 2 * c + 8 * s) = make_double2(a[h][s][0], a[h][s][1]);
      }
  };
  const int j0 = 2 * c + 8 * t16;  // this lane's column pair (its slot of the v/p broadcasts)
  double cx = 0.0, cy = 0.0, beta = 0.0, v0 = 0.0, vi[RPL];
#pragma unroll
  for (int h = 0; h < RPL; ++h) vi[h] = 0.0;
  // the update of one group of 4 slots of row set h: a_ij += g_i v_j - h_i p_j (mhi = -h_i)
  // (the p terms of the 8 entries first, then the v terms: a dependent pair is 8 issues apart)
  auto upd_group = [&](auto G, auto H, double px, double py, double gi, double mhi) {
    constexpr int g = decltype(G)::value, h = decltype(H)::value;
    static_for<4 * g, 4 * g + 4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      fmac_bcast<s, s == 4 * g>(a[h][s][0], px, mhi);
      fmac_bcast<s, false>(a[h][s][1], py, mhi);
    });
    static_for<4 * g, 4 * g + 4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      fmac_bcast<s, false>(a[h][s][0], cx, gi);
      fmac_bcast<s, false>(a[h][s][1], cy, gi);
    });
  };
  // Reflector of column r from x = row r of the current matrix (at j0, j0+1, the lane's rows,
  // r and r+1), every wave redundantly: v_j = 0 (j <= r), v0 (j = r+1), x_j (j > r+1);
  // H = I - beta v v^T.  The sum of squares is a wave reduction whose six steps are interleaved
  // (sched_barrier) with the slot groups of the pending update `upd(g)` (in-order issue: the
  // update's FMAs fill the reduction's latency).
  auto reflector = [&](int r, double xj0, double xj1, const double* xi, double xr, double x0,
                       auto&& upd) {
    double tl = (j0 >= r + 2 ? xj0 * xj0 : 0.0);
    tl = fma(j0 + 1 >= r + 2 ? xj1 : 0.0, xj1, tl);
    tl += dpp_d<0xB1>(tl);
    __builtin_amdgcn_sched_barrier(0);
    upd(std::integral_constant<int, 0>{});
    __builtin_amdgcn_sched_barrier(0);
    tl += dpp_d<0x4E>(tl);
    __builtin_amdgcn_sched_barrier(0);
    upd(std::integral_constant<int, 1>{});
    __builtin_amdgcn_sched_barrier(0);
    tl += dpp_d<0x141>(tl);
    __builtin_amdgcn_sched_barrier(0);
    upd(std::integral_constant<int, 2>{});
    __builtin_amdgcn_sched_barrier(0);
    tl += dpp_d<0x140>(tl);
    __builtin_amdgcn_sched_barrier(0);
    upd(std::integral_constant<int, 3>{});
    __builtin_amdgcn_sched_barrier(0);
    tl = xsum32(xsum16(tl));  // sum_{j >= r+2} x_j^2 over the wave
    beta = 0.0;
    v0 = x0;
    double e2r = x0 * x0;
    if (tl > 0.0) {
      const double ss = fma(x0, x0, tl);
      double nrm;
      if (ss > 0x1p-900) {  // Newton-refined hardware rsq / rcp (~1 ulp), no IEEE sqrt/div chain
        double rs = __builtin_amdgcn_rsq(ss);
        rs = rs * fma(-0.5 * ss, rs * rs, 1.5);
        nrm = ss * rs;
        nrm = fma(fma(-nrm, nrm, ss), 0.5 * rs, nrm);
      } else {
        nrm = sqrt(ss);
      }
      const double alpha = x0 > 0.0 ? -nrm : nrm;
      v0 = x0 - alpha;
      const double q = fma(v0, v0, tl);
      double rc = __builtin_amdgcn_rcp(q);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      beta = 2.0 * rc;
      e2r = alpha * alpha;
    }
    if (writer && lane == 0) {
      dg[r] = xr;
      e2[r] = e2r;
    }
    cx = j0 <= r ? 0.0 : (j0 == r + 1 ? v0 : xj0);
    cy = j0 + 1 <= r ? 0.0 : (j0 + 1 == r + 1 ? v0 : xj1);
#pragma unroll
    for (int h = 0; h < RPL; ++h) vi[h] = i[h] > r ? (i[h] == r + 1 ? v0 : xi[h]) : 0.0;
    if (writer) *reinterpret_cast<double2*>(&vb[r & 1][j0]) = make_double2(cx, cy);
  };
  publish_row(0, rowb[0]);
  if (n >= 2) publish_row(1, rowb[1]);
  __syncthreads();
  if (n >= 2) {
    const double2 xr = *reinterpret_cast<const double2*>(&rowb[0][j0]);
    double xi0[RPL];
#pragma unroll
    for (int h = 0; h < RPL; ++h) xi0[h] = rowb[0][i[h]];
    reflector(0, xr.x, xr.y, xi0, rowb[0][0], rowb[0][1], [](auto) {});
  } else if (tid == 0) {
    dg[0] = rowb[0][0];
  }
  ER_STAMP(0)
  for (int k = 0; k + 2 < n; ++k) {
    const int lo = (k + 1) >> 3;  // slots s < lo hold columns <= k only
    bool live[RPL];               // wave-uniform: some row of row set h is active
#pragma unroll
    for (int h = 0; h < RPL; ++h) live[h] = blk[h] * 16 + 15 > k && blk[h] * 16 < n;
    // ---- p = A' v (registers) and this wave's part of v^T p; two FMA chains per row set
    double pp[RPL];
    double t = 0.0;
    static_for<0, RPL>([&](auto H) {
      constexpr int h = decltype(H)::value;
      double pa[4] = {0.0, 0.0, 0.0, 0.0};
      // slots in groups of 4 behind one uniform branch each (a per-slot condition gets
      // if-converted into computing everything plus selects)
      if (live[h] && !(DBG & 2)) {
        static_for<0, NS / 4>([&](auto G) {
          constexpr int g = decltype(G)::value;
          if (4 * g + 3 >= lo) {
            static_for<4 * g, 4 * g + 4>([&](auto S) {
              constexpr int s = decltype(S)::value;
              // cx/cy were written by VALU selects: wait states before the first DPP read
              fmac_bcast<s, s == 4 * g>(pa[2 * (s & 1)], cx, a[h][s][0]);
              fmac_bcast<s, false>(pa[2 * (s & 1) + 1], cy, a[h][s][1]);
            });
          }
        });
      }
      pp[h] = (pa[0] + pa[1]) + (pa[2] + pa[3]);
    });
    ER_STAMP(1)
#pragma unroll
    for (int h = 0; h < RPL; ++h) {
      pp[h] = xsum32(xsum16(pp[h]));
      if (c == 0) {
        pb[k & 1][i[h]] = i[h] > k ? pp[h] : 0.0;
        t = fma(vi[h], pp[h], t);
      }
    }
    t = row16_sum(t);  // only lanes 0..15 (class 0) carry the rows' v_i p_i
    if (lane == 0) redw[k & 1][w] = t;
    ER_STAMP(2)
    __syncthreads();
    ER_STAMP(3)
    bool need = false;  // wave-uniform: some row of this wave lies beyond k+1
#pragma unroll
    for (int h = 0; h < RPL; ++h) need = need || (blk[h] * 16 + 15 > k + 1 && blk[h] * 16 < n);
    if (!need) continue;  // (the barrier of the next step is at its top, after the matvec)
    // ---- every LDS read of the step at once
    const int r = k + 1;
    const double* old = rowb[r & 1];
    double rw[NWV];
#pragma unroll
    for (int q = 0; q < NWV; q += 2) {
      const double2 v2 = *reinterpret_cast<const double2*>(&redw[k & 1][q]);
      rw[q] = v2.x;
      rw[q + 1] = v2.y;
    }
    const double2 pvr = *reinterpret_cast<const double2*>(&pb[k & 1][j0]);
    const double2 o = *reinterpret_cast<const double2*>(old + j0);
    double oi[RPL];
#pragma unroll
    for (int h = 0; h < RPL; ++h) oi[h] = old[i[h]];
    const double orr = old[r], or1 = old[r + 1];
    const double vr = vb[k & 1][r], vr1 = vb[k & 1][r + 1];
    const double pr = pb[k & 1][r], pr1 = pb[k & 1][r + 1];
    // ---- w = beta p - K v;  A' -= v w^T + w v^T, i.e. a_ij += g_i v_j - h_i p_j with
    // g_i = K v_i - w_i, h_i = beta v_i
    double tot;
    if constexpr (NWV == 8)
      tot = ((rw[0] + rw[1]) + (rw[2] + rw[3])) + ((rw[4] + rw[5]) + (rw[6] + rw[7]));
    else
      tot = (rw[0] + rw[1]) + (rw[2] + rw[3]);
    const double Kc = beta * beta * tot * 0.5;
    double gi[RPL], mhi[RPL];
#pragma unroll
    for (int h = 0; h < RPL; ++h) {
      const double wi = beta * pp[h] - Kc * vi[h];
      gi[h] = Kc * vi[h] - wi;
      mhi[h] = -(beta * vi[h]);
    }
    // row r = k+1 after this update, recomputed by every lane from the published row with the
    // owners' own operations (bitwise their registers): x_j = a_rj + g_r v_j - h_r p_j
    const double wr = beta * pr - Kc * vr;
    const double gr = Kc * vr - wr, mhr = -(beta * vr);
    const double xj0 = fma(cx, gr, fma(pvr.x, mhr, o.x));
    const double xj1 = fma(cy, gr, fma(pvr.y, mhr, o.y));
    double xi[RPL];
#pragma unroll
    for (int h = 0; h < RPL; ++h) xi[h] = fma(vi[h], gr, fma(pp[h], mhr, oi[h]));
    const double xr = fma(vr, gr, fma(pr, mhr, orr));
    const double x0 = fma(vr1, gr, fma(pr1, mhr, or1));
    ER_STAMP(4)
    // the pending update (old v in cx/cy) runs inside the reflector's reduction
    const double pxu = pvr.x, pyu = pvr.y;
    reflector(r, xj0, xj1, xi, xr, x0, [&](auto G) {
      constexpr int g = decltype(G)::value;
      static_for<0, RPL>([&](auto H) {
        constexpr int h = decltype(H)::value;
        if (blk[h] * 16 + 15 > k + 1 && blk[h] * 16 < n && !(DBG & 1) && 4 * g + 3 >= lo)
          upd_group(G, H, pxu, pyu, gi[h], mhi[h]);
      });
    });
    ER_STAMP(5)
    // the owners of row k+2 publish it (after their update) for the step after next; rowb[k&1]
    // was last read before this step's barrier
    publish_row(k + 2, rowb[k & 1]);
    ER_STAMP(6)
  }
  // the last diagonal entry: row n-1 as its owners published it at the last step (or at the start)
  __syncthreads();
  if (tid == 0 && n >= 2) dg[n - 1] = rowb[(n - 1) & 1][n - 1];
  __syncthreads();
  // Gershgorin interval of the tridiagonal: row r in thread r (waves 0-1), wave min/max, then
  // the two wave results through LDS (the masks words are free until the multisection)
  int bnd_ex = 0;
  {
    double lo = INFINITY, hi = -INFINITY;
    if (tid < n) {
      double rr = 0.0;
      if (tid > 0) rr += sqrt(e2[tid - 1]);
      if (tid + 1 < n) rr += sqrt(e2[tid]);
      lo = dg[tid] - rr;
      hi = dg[tid] + rr;
    }
    if (w < 2) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o));
        hi = fmax(hi, __shfl_xor(hi, o));
      }
      if (lane == 0) {
        reinterpret_cast<double*>(masks)[2 * w] = lo;
        reinterpret_cast<double*>(masks)[2 * w + 1] = hi;
      }
    }
    __syncthreads();
    // every thread forms the interval; the tridiagonal is then scaled by 2^-ex so that the
    // interval lies in [-1, 1]: every |d_i - sigma| <= 2 and e_i <= 1, so 8 rows of minors grow
    // by at most 3^8 and sturm_any_below cannot overflow whatever the norm of the block (a
    // power-of-two scaling is exact and leaves every Sturm count unchanged)
    const double* m = reinterpret_cast<const double*>(masks);
    const double l = fmin(m[0], m[2]), h = fmax(m[1], m[3]);
    const double mag = fmax(fabs(l), fabs(h));
    const int ex = (mag > 0.0 && mag < INFINITY) ? __builtin_amdgcn_frexp_exp(mag) : 0;
    bnd_ex = ex;
    // the scaled, padded copy the counts read: rows n..127 get d = 4 (above every sigma, which
    // lies in [-1.002, 1.002]) and no coupling, so they add no negative minor; se[i] = e2_{i-1}
    // (se[0] = 0) floored at 2^-900, so that a zero minor is always followed by a nonzero one
    // (p_{i+1} = -e2_i p_{i-1}) and the recurrence never stalls at zero
    if (tid < 128) {
      sd[tid] = tid < n ? __builtin_ldexp(dg[tid], -ex) : 4.0;
      se[tid] = (tid >= 1 && tid < n) ? fmax(__builtin_ldexp(e2[tid - 1], -2 * ex), 0x1p-900) : 0.0;
    }
    if (tid == 0) {
      const double ls = __builtin_ldexp(l, -ex), hs = __builtin_ldexp(h, -ex);
      const double span = hs - ls;
      bnd[0] = ls - span * 1e-3 - 1e-300;
      bnd[1] = hs + span * 1e-3 + 1e-300;
    }
  }
  __syncthreads();
  // ---- 256-way multisection on waves 0-3 (one per SIMD: a count is a 128-row chain of ~5 VALU
  // instructions per row, so a second wave per SIMD would double the round's issue time for one
  // more bit): 7 rounds of 8 bits bracket lambda_min to 2^-56 of the Gershgorin span, below the
  // Sturm count's own backward error (~n eps ||T||)
  double lo = bnd[0], hi = bnd[1];
  const int nr = (n + 7) & ~7;
  for (int it = 0; it < 7; ++it) {
    const double width = hi - lo;
    if (w < 4) {
      const double sigma = lo + width * ((double)(tid + 1) / 257.0);
      const unsigned long long mk = __ballot(sturm_any_below(sd, se, nr, sigma));
      if (lane == 0) masks[w] = mk;
    }
    __syncthreads();
    int f = -1;
    for (int q = 0; q < 4 && f < 0; ++q)
      if (masks[q]) f = q * 64 + __ffsll((long long)masks[q]) - 1;
    __syncthreads();
    if (f < 0) {
      lo = lo + width * (256.0 / 257.0);
    } else {
      hi = lo + width * ((double)(f + 1) / 257.0);
      if (f > 0) lo = lo + width * ((double)f / 257.0);
    }
  }
  ER_STAMP(7)
#ifdef CLRSDP_EIGREG_STAMPS
  if (tid == 0)
    for (int q = 0; q < 8; ++q) atomicAdd(&g_eigreg_stamps[q], st_acc[q]);
#endif
  if (tid == 0) out[blockIdx.x] = __builtin_ldexp((lo + hi) * 0.5, bnd_ex + ex0);
#undef ER_STAMP
}

// ------------------------------------------------------------------------------------------
// eigmin_split (round 4): lambda_min of a symmetric fp64 block (n <= 128), the same Householder
// tridiagonalisation as eigmin_reg with the matrix in the registers of 8 "bulk" waves (same
// layout), but the reflector of each column is built ONCE, by a ninth "chain" wave at raised
// issue priority, instead of redundantly by every live wave: that redundancy made eigmin_reg
// VALU-issue bound (~300 instructions per column and wave against 96 useful FMAs, two waves per
// SIMD).  Two barriers per column k:
//   bulk:  p = A_k v_k in registers, per-wave v^T p, the rows of p to LDS          -- barrier 1
//   bulk:  w = beta p - K v; A_{k+1} = A_k - v w^T - w v^T in registers; the owners of row k+2
//          publish it (for step k+1)
//   chain: row k+1 of A_{k+1} from the copy its owners published a step earlier (their own
//          operations), the reflector v_{k+1} and beta_{k+1}, the tridiagonal entries -> LDS
//                                                                                   -- barrier 2
// The rank-2 update (two of the three FMAs per entry) runs under the chain's latency; per column
// only the matvec, two LDS round trips and the chain's ~40 dependent operations are serial.
// The chain lane (c, t16) holds the same column pair j0 = 2c + 8 t16 as a bulk lane, so its sums
// run in eigmin_reg's order.  Same scaling, Gershgorin bracket and multisection as eigmin_reg.
// ------------------------------------------------------------------------------------------
#ifdef CLRSDP_EIGSPLIT_STAMPS
__device__ unsigned long long g_eigsplit_stamps[8];
#endif
// DBG (timing experiments only): 1 = no update FMAs, 2 = no matvec FMAs, 4 = the chain wave
// skips the reflector (v_{k+1} = the published row), 8 = the old one-chain 256-way multisection,
// 128 / 256 = the column loop stops 32 / 64 columns early (what the tail columns cost)
// TAIL (round 5): the last TAIL columns (TAIL <= 32, n >= TAIL + 8) run on the chain wave alone:
// the trailing TAIL x TAIL matrix goes through LDS into its registers (row lane & 31 per lane,
// both half-waves alike) and every step is wave-local -- no barrier, no cross-wave exchange.
// The two-barrier skeleton costs ~0.8 us per column however small the trailing matrix is
// (the last 32 columns of a 128 block: 26 us of 145, tools/micro/eig_split_bench.hip).
template <int DBG = 0, int TAIL = 0>
__global__ __launch_bounds__(576) void eigmin_split(const MatDesc<double>* __restrict__ descs,
                                                     double* __restrict__ out) {
  static_assert(TAIL == 0 || (TAIL >= 8 && TAIL <= 32), "tail size");
  constexpr int NS = 16, NWB = 8, GS = (DBG & 16) ? 2 : 4;
#ifdef CLRSDP_EIGSPLIT_STAMPS
  // per column: chain lane 0 (slots 0-2: wait at barrier 1, reflector, wait at barrier 2) and
  // bulk wave 4 lane 0 (row block 7, live to the end; slots 3-6: matvec phase, wait at barrier
  // 1, update phase, wait at barrier 2); slot 7: multisection
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#define ES_STAMP(slot)                                            \
  {                                                               \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    st_acc[slot] += t_ - t_prev;                                  \
    t_prev = t_;                                                  \
  }
#else
#define ES_STAMP(slot)
#endif
  __shared__ __attribute__((aligned(16))) double rowb[2][128];
  __shared__ __attribute__((aligned(16))) double pb[2][128];
  __shared__ __attribute__((aligned(16))) double vb[2][128];
  __shared__ __attribute__((aligned(16))) double redw[2][NWB];
  __shared__ double betab[2];
  __shared__ double dg[128], e2[128];
  __shared__ __attribute__((aligned(16))) double sd[128], se[128];
  __shared__ double bnd[2];
  __shared__ unsigned long long masks[8];
  __shared__ double amaxw[NWB];
  const MatDesc<double> d = descs[blockIdx.x];
  const int n = d.n, lda = d.lda, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const bool chain = w == NWB;
  const int blk = w < 4 ? w : 11 - w;  // bulk row block (pairs 0/7, 1/6, 2/5, 3/4 per SIMD)
  const int c = lane >> 4, t16 = lane & 15;
  const int i = blk * 16 + t16;       // bulk: this lane's row
  const int j0 = 2 * c + 8 * t16;     // this lane's column pair (bulk: broadcast slot; chain: x_j)
  double a[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s) a[s][0] = a[s][1] = 0.0;
  if (!chain) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * c + 8 * s + e;
        const int ic = min(i, n - 1), jc = min(j, n - 1);
        const double v = gload(d.A + ic + (size_t)jc * lda);
        a[s][e] = (i < n && j < n) ? v : 0.0;
      }
    double amax = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) amax = fmax(amax, fmax(fabs(a[s][0]), fabs(a[s][1])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
    if (lane == 0) amaxw[w] = amax;
  }
  __syncthreads();
  int ex0;
  {
    double amax = amaxw[0];
#pragma unroll
    for (int r = 1; r < NWB; ++r) amax = fmax(amax, amaxw[r]);
    ex0 = (amax > 0.0 && amax < INFINITY) ? __builtin_amdgcn_frexp_exp(amax) : 0;
  }
  if (!chain) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      a[s][0] = __builtin_ldexp(a[s][0], -ex0);
      a[s][1] = __builtin_ldexp(a[s][1], -ex0);
    }
  }
  auto publish_row = [&](int r, double* dst) {  // the owners of row r write its 128 entries
    if (!chain && blk == (r >> 4) && t16 == (r & 15)) {
#pragma unroll
      for (int s = 0; s < NS; ++s)
        *reinterpret_cast<double2*>(dst + 2 * c + 8 * s) = make_double2(a[s][0], a[s][1]);
    }
  };
  // chain state: v of the current step at the lane's column pair, and beta
  double cx = 0.0, cy = 0.0, beta = 0.0, vi = 0.0;
  // the reflector of column r from x = row r of the current matrix (chain wave only):
  // v_j = 0 (j <= r), v0 (j = r+1), x_j (j > r+1), H = I - beta v v^T
  auto reflector = [&](int r, double xj0, double xj1, double xr, double x0) {
    double tl = (j0 >= r + 2 ? xj0 * xj0 : 0.0);
    tl = fma(j0 + 1 >= r + 2 ? xj1 : 0.0, xj1, tl);
    tl = xsum32(xsum16(row16_sum(tl)));  // sum_{j >= r+2} x_j^2
    double bt = 0.0, v0 = x0, e2r = x0 * x0;
    if (tl > 0.0) {
      const double ss = fma(x0, x0, tl);
      double nrm;
      if (ss > 0x1p-900) {  // Newton-refined hardware rsq / rcp (~1 ulp)
        double rs = __builtin_amdgcn_rsq(ss);
        rs = rs * fma(-0.5 * ss, rs * rs, 1.5);
        nrm = ss * rs;
        nrm = fma(fma(-nrm, nrm, ss), 0.5 * rs, nrm);
      } else {
        nrm = sqrt(ss);
      }
      const double alpha = x0 > 0.0 ? -nrm : nrm;
      v0 = x0 - alpha;
      const double q = fma(v0, v0, tl);
      double rc = __builtin_amdgcn_rcp(q);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      bt = 2.0 * rc;
      e2r = alpha * alpha;
    }
    cx = j0 <= r ? 0.0 : (j0 == r + 1 ? v0 : xj0);
    cy = j0 + 1 <= r ? 0.0 : (j0 + 1 == r + 1 ? v0 : xj1);
    beta = bt;
    *reinterpret_cast<double2*>(&vb[r & 1][j0]) = make_double2(cx, cy);
    if (lane == 0) {
      dg[r] = xr;
      e2[r] = e2r;
      betab[r & 1] = bt;
    }
  };
  publish_row(0, rowb[0]);
  if (n >= 2) publish_row(1, rowb[1]);
  __syncthreads();
  if (chain) {
    __builtin_amdgcn_s_setprio(3);
    if (n >= 2) {
      const double2 xr = *reinterpret_cast<const double2*>(&rowb[0][j0]);
      reflector(0, xr.x, xr.y, rowb[0][0], rowb[0][1]);
    } else if (lane == 0) {
      dg[0] = rowb[0][0];
    }
  }
  __syncthreads();
  if (!chain && n >= 2) {
    const double2 v2 = *reinterpret_cast<const double2*>(&vb[0][j0]);
    cx = v2.x;
    cy = v2.y;
    vi = vb[0][i];
    beta = betab[0];
  }
  constexpr int KSKIP = (DBG & 128) ? 32 : (DBG & 256) ? 64 : 0;
  // with the tail: the loop stops at iteration k0 = n - TAIL - 1 (A_{k0} in the registers, the
  // reflector v_{k0} in vb / betab), the chain wave does iterations k0 .. n - 3
  const bool tail = TAIL > 0 && n >= TAIL + 8;
  const int kend = tail ? n - TAIL - 1 + 2 : n;  // loop while k + 2 < kend
  for (int k = 0; k + 2 + KSKIP < kend; ++k) {
    const int lo = (k + 1) >> 3;  // slots s < lo hold columns <= k only
    const int r = k + 1;
    double pp = 0.0;
    if (!chain) {
      // ---- p = A_k v_k and this wave's part of v^T p (two FMA chains per column parity)
      const bool live = blk * 16 + 15 > k && blk * 16 < n;
      double pa[4] = {0.0, 0.0, 0.0, 0.0};
      if (live && !(DBG & 2)) {
        // slots in groups of GS behind one uniform branch each (pairs measured slower: a
        // branch and the DPP wait state per group)
        static_for<0, NS / GS>([&](auto G) {
          constexpr int g = decltype(G)::value;
          if (GS * g + GS - 1 >= lo) {
            static_for<GS * g, GS * g + GS>([&](auto S) {
              constexpr int s = decltype(S)::value;
              fmac_bcast<s, s == GS * g>(pa[2 * (s & 1)], cx, a[s][0]);
              fmac_bcast<s, false>(pa[2 * (s & 1) + 1], cy, a[s][1]);
            });
          }
        });
      }
      pp = xsum32(xsum16((pa[0] + pa[1]) + (pa[2] + pa[3])));
      double t = 0.0;
      if (c == 0) {
        pb[k & 1][i] = i > k ? pp : 0.0;
        t = vi * pp;
      }
      t = row16_sum(t);  // class-0 lanes carry the rows' v_i p_i
      if (lane == 0) redw[k & 1][w] = t;
      ES_STAMP(3)
    }
    __syncthreads();
    ES_STAMP(chain ? 0 : 4)
    if (chain) {
      // ---- row r of A_{k+1} and the reflector v_{k+1}
      double rw[NWB];
#pragma unroll
      for (int q = 0; q < NWB; q += 2) {
        const double2 v2 = *reinterpret_cast<const double2*>(&redw[k & 1][q]);
        rw[q] = v2.x;
        rw[q + 1] = v2.y;
      }
      const double* old = rowb[r & 1];
      const double2 pj = *reinterpret_cast<const double2*>(&pb[k & 1][j0]);
      const double2 o = *reinterpret_cast<const double2*>(old + j0);
      const double orr = old[r], or1 = old[r + 1];
      const double vr = vb[k & 1][r], vr1 = vb[k & 1][r + 1];
      const double pr = pb[k & 1][r], pr1 = pb[k & 1][r + 1];
      const double tot = ((rw[0] + rw[1]) + (rw[2] + rw[3])) + ((rw[4] + rw[5]) + (rw[6] + rw[7]));
      const double Kc = beta * beta * tot * 0.5;
      const double wr = fma(beta, pr, -(Kc * vr));
      const double gr = fma(Kc, vr, -wr), mhr = -(beta * vr);
      const double xj0 = fma(cx, gr, fma(pj.x, mhr, o.x));
      const double xj1 = fma(cy, gr, fma(pj.y, mhr, o.y));
      const double xr = fma(vr, gr, fma(pr, mhr, orr));
      const double x0 = fma(vr1, gr, fma(pr1, mhr, or1));
      if constexpr (DBG & 4) {
        cx = o.x;
        cy = o.y;
        *reinterpret_cast<double2*>(&vb[r & 1][j0]) = make_double2(cx, cy);
        if (lane == 0) { dg[r] = xr + xj0 + x0; e2[r] = 1.0; betab[r & 1] = 0.0; }
      } else {
        reflector(r, xj0, xj1, xr, x0);
      }
      ES_STAMP(1)
    } else if (blk * 16 + 15 > k + 1 && blk * 16 < n) {
      // ---- w = beta p - K v;  A -= v w^T + w v^T, i.e. a_ij += g_i v_j - h_i p_j
      double rw[NWB];
#pragma unroll
      for (int q = 0; q < NWB; q += 2) {
        const double2 v2 = *reinterpret_cast<const double2*>(&redw[k & 1][q]);
        rw[q] = v2.x;
        rw[q + 1] = v2.y;
      }
      const double2 pv = *reinterpret_cast<const double2*>(&pb[k & 1][j0]);
      const double tot = ((rw[0] + rw[1]) + (rw[2] + rw[3])) + ((rw[4] + rw[5]) + (rw[6] + rw[7]));
      const double Kc = beta * beta * tot * 0.5;
      const double wi = fma(beta, pp, -(Kc * vi));
      const double gi = fma(Kc, vi, -wi), mhi = -(beta * vi);
      // per group the p terms, then the v terms (a dependent pair is 8 issues apart); all p
      // terms ahead of all v terms measured slower
      if (!(DBG & 1)) static_for<0, NS / GS>([&](auto G) {
        constexpr int g = decltype(G)::value;
        if (GS * g + GS - 1 >= lo) {
          static_for<GS * g, GS * g + GS>([&](auto S) {
            constexpr int s = decltype(S)::value;
            fmac_bcast<s, s == GS * g>(a[s][0], pv.x, mhi);
            fmac_bcast<s, false>(a[s][1], pv.y, mhi);
          });
          static_for<GS * g, GS * g + GS>([&](auto S) {
            constexpr int s = decltype(S)::value;
            fmac_bcast<s, false>(a[s][0], cx, gi);
            fmac_bcast<s, false>(a[s][1], cy, gi);
          });
        }
      });
      publish_row(k + 2, rowb[k & 1]);
      ES_STAMP(5)
    }
    __syncthreads();
    ES_STAMP(chain ? 2 : 6)
    if (!chain) {
      const double2 v2 = *reinterpret_cast<const double2*>(&vb[r & 1][j0]);
      cx = v2.x;
      cy = v2.y;
      vi = vb[r & 1][i];
      beta = betab[r & 1];
    }
  }
  if (chain) __builtin_amdgcn_s_setprio(0);
  if constexpr (TAIL > 0) {
    if (tail) {
      constexpr int TT = TAIL;
      __shared__ double Mt[TT][TT + 1];
      __shared__ double ub[TT], pt[TT];
      const int k0 = n - TT - 1;
      // A_{k0}'s trailing block (rows and columns > k0) from the bulk registers, v_{k0} there
      if (!chain) {
#pragma unroll
        for (int sl = 0; sl < NS; ++sl)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int j = 2 * c + 8 * sl + e;
            if (i > k0 && j > k0 && i < n && j < n) Mt[i - k0 - 1][j - k0 - 1] = a[sl][e];
          }
      }
      if (tid < TT) ub[tid] = vb[k0 & 1][k0 + 1 + tid];
      __syncthreads();
      if (chain) {
        // lanes 0..TT-1 hold rows 0..TT-1; the others a dummy copy of row 0, masked out of
        // every sum and every LDS write
        const bool lo32 = lane < TT;
        const int t = lo32 ? lane : 0;
        double ar[TT];
#pragma unroll
        for (int j = 0; j < TT; ++j) ar[j] = Mt[t][j];
        double bt = betab[k0 & 1], ut = lo32 ? ub[t] : 0.0;
        static_for<0, TT - 1>([&](auto S) {
          constexpr int st = decltype(S)::value;  // global iteration k0 + st: apply v, then v'
          // p = A v over the live rows / columns (>= st), v^T p over the 32 lanes
          double p0 = 0.0, p1 = 0.0;
#pragma unroll
          for (int j = st; j < TT; ++j) {
            if ((j - st) & 1) p1 = fma(ar[j], ub[j], p1);
            else p0 = fma(ar[j], ub[j], p0);
          }
          const double p = (t >= st && lo32) ? p0 + p1 : 0.0;
          const double tot = xsum16(row16_sum(ut * p));
          const double Kc = bt * bt * tot * 0.5;
          const double wv = fma(bt, p, -(Kc * ut));
          const double g = fma(Kc, ut, -wv), mh = -(bt * ut);
          if (lo32) pt[t] = p;
          // A -= v w^T + w v^T: a_tj += mh p_j + g v_j (the p terms, then the v terms; the
          // broadcast reads phase by phase, not all hoisted: register pressure)
          asm volatile("" ::: "memory");
#pragma unroll
          for (int j = st; j < TT; ++j) ar[j] = fma(pt[j], mh, ar[j]);
          asm volatile("" ::: "memory");
#pragma unroll
          for (int j = st; j < TT; ++j) ar[j] = fma(ub[j], g, ar[j]);
          asm volatile("" ::: "memory");
          // the next reflector from column st of the updated matrix (global row r = k0 + 1 + st)
          const double xr = readlane_d(ar[st], st), x0 = readlane_d(ar[st], st + 1);
          const double tl = xsum16(row16_sum((t >= st + 2 && lo32) ? ar[st] * ar[st] : 0.0));
          double b2 = 0.0, v0 = x0, e2r = x0 * x0;
          if (tl > 0.0) {
            const double ss = fma(x0, x0, tl);
            double nrm;
            if (ss > 0x1p-900) {
              double rs = __builtin_amdgcn_rsq(ss);
              rs = rs * fma(-0.5 * ss, rs * rs, 1.5);
              nrm = ss * rs;
              nrm = fma(fma(-nrm, nrm, ss), 0.5 * rs, nrm);
            } else {
              nrm = sqrt(ss);
            }
            const double alpha = x0 > 0.0 ? -nrm : nrm;
            v0 = x0 - alpha;
            const double q = fma(v0, v0, tl);
            double rc = __builtin_amdgcn_rcp(q);
            rc = fma(fma(-q, rc, 1.0), rc, rc);
            rc = fma(fma(-q, rc, 1.0), rc, rc);
            b2 = 2.0 * rc;
            e2r = alpha * alpha;
          }
          ut = (t <= st || !lo32) ? 0.0 : (t == st + 1 ? v0 : ar[st]);
          bt = b2;
          if (lo32) ub[t] = ut;
          if (lane == 0) {
            dg[k0 + 1 + st] = xr;
            e2[k0 + 1 + st] = e2r;
          }
        });
        if (lane == TT - 1) dg[n - 1] = ar[TT - 1];  // (the last reflector only flips its sign)
      }
    } else if (tid == 0 && n >= 2) {
      dg[n - 1] = rowb[(n - 1) & 1][n - 1];
    }
  } else {
    // the last diagonal entry: row n-1 as its owners published it at the last step (or at the start)
    if (tid == 0 && n >= 2) dg[n - 1] = rowb[(n - 1) & 1][n - 1];
  }
  __syncthreads();
  // Gershgorin interval, scaling and 256-way multisection: as eigmin_reg
  int bnd_ex = 0;
  {
    double lo = INFINITY, hi = -INFINITY;
    if (tid < n) {
      double rr = 0.0;
      if (tid > 0) rr += sqrt(e2[tid - 1]);
      if (tid + 1 < n) rr += sqrt(e2[tid]);
      lo = dg[tid] - rr;
      hi = dg[tid] + rr;
    }
    if (w < 2) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o));
        hi = fmax(hi, __shfl_xor(hi, o));
      }
      if (lane == 0) {
        reinterpret_cast<double*>(masks)[2 * w] = lo;
        reinterpret_cast<double*>(masks)[2 * w + 1] = hi;
      }
    }
    __syncthreads();
    const double* m = reinterpret_cast<const double*>(masks);
    const double l = fmin(m[0], m[2]), h = fmax(m[1], m[3]);
    const double mag = fmax(fabs(l), fabs(h));
    const int ex = (mag > 0.0 && mag < INFINITY) ? __builtin_amdgcn_frexp_exp(mag) : 0;
    bnd_ex = ex;
    if (tid < 128) {
      sd[tid] = tid < n ? __builtin_ldexp(dg[tid], -ex) : 4.0;
      se[tid] = (tid >= 1 && tid < n) ? fmax(__builtin_ldexp(e2[tid - 1], -2 * ex), 0x1p-900) : 0.0;
    }
    if (tid == 0) {
      const double ls = __builtin_ldexp(l, -ex), hs = __builtin_ldexp(h, -ex);
      const double span = hs - ls;
      bnd[0] = ls - span * 1e-3 - 1e-300;
      bnd[1] = hs + span * 1e-3 + 1e-300;
    }
  }
  __syncthreads();
  double lo = bnd[0], hi = bnd[1];
  const int nr = (n + 7) & ~7;
  // 512-way on the 8 bulk waves (two per SIMD: the count is a latency-bound chain, so the second
  // wave per SIMD costs little), 6 rounds of 9 bits (2^-54 of the span): 3 us less than 256-way
  // on 4 waves in 7 rounds (DBG 64 keeps that, DBG 8 the two-ended count)
  constexpr int NCW = (DBG & 64) ? 4 : NWB;        // counting waves
  constexpr double NSIG = 64.0 * NCW + 1.0;
  for (int it = 0; it < ((DBG & 64) ? 7 : 6); ++it) {
    const double width = hi - lo;
    if (w < NCW) {
      const double sigma = lo + width * ((double)(tid + 1) / NSIG);
      const bool below = (DBG & 8) ? sturm_any_below2(sd, se, nr, sigma) : sturm_any_below(sd, se, nr, sigma);
      const unsigned long long mk = __ballot(below);
      if (lane == 0) masks[w] = mk;
    }
    __syncthreads();
    int f = -1;
    for (int q = 0; q < NCW && f < 0; ++q)
      if (masks[q]) f = q * 64 + __ffsll((long long)masks[q]) - 1;
    __syncthreads();
    if (f < 0) {
      lo = lo + width * ((NSIG - 1.0) / NSIG);
    } else {
      hi = lo + width * ((double)(f + 1) / NSIG);
      if (f > 0) lo = lo + width * ((double)f / NSIG);
    }
  }
  if (tid == 0) out[blockIdx.x] = __builtin_ldexp((lo + hi) * 0.5, bnd_ex + ex0);
#ifdef CLRSDP_EIGSPLIT_STAMPS
  ES_STAMP(7)
  if (lane == 0 && (chain || w == 4))
    for (int q = 0; q < 8; ++q)
      if ((chain && q < 3) || (!chain && q >= 3)) atomicAdd(&g_eigsplit_stamps[q], st_acc[q]);
#endif
#undef ES_STAMP
}

// ------------------------------------------------------------------------------------------
// eigmin_onebar (round 6): eigmin_split with ONE barrier per column.  eigmin_split runs per
// column k: the bulk's p = A_k v_k and its reductions -- barrier -- the chain wave's reflector
// v_{k+1} beside the bulk's rank-2 update -- barrier; the matrix-vector product and its
// reductions sit between the two barriers on the critical path.  Here they move under the
// chain's reflector: v_{k+1} = x~ + v0 e_{k+2}, where x~ = row k+1 of A_{k+1} beyond column
// k+2 is known as soon as K_k is (x_j = o_j - beta v_r p_j + g_r v_j, the chain's own formula on
// the same operands, so the bulk's copy has the chain's bits), and only the scalar v0 = x_{k+2}
// - alpha waits for the reflector.  So after the barrier of column k the bulk waves apply the
// rank-2 update of column k and at once form, with the updated registers,
//     q = A_{k+1} x~,   c = A_{k+1} e_{k+2}   (per row, in LDS)
//     S1 = x~^T q,      S2 = x~^T c           (per-wave partials)
// while the chain wave builds v0 and beta_{k+1} from the same row.  After the next barrier
//     p_{k+1} = q + v0 c,   v_{k+1}^T p_{k+1} = S1 + v0 S2 + v0 p_{k+1}[k+2]
// come out of LDS with no further cross-wave exchange.  Chain and bulk form p, K, w_r, g_r and
// x~ by identical expressions from identical LDS operands, so v_{k+1} is one vector everywhere.
// Same layout, scaling, Gershgorin bracket and 512-way multisection as eigmin_split.
// ------------------------------------------------------------------------------------------
template <int DBG = 0>
__global__ __launch_bounds__(576) void eigmin_onebar(const MatDesc<double>* __restrict__ descs,
                                                      double* __restrict__ out) {
  constexpr int NS = 16, NWB = 8, GS = 4;
  __shared__ __attribute__((aligned(16))) double rowb[2][128];
  __shared__ __attribute__((aligned(16))) double qb[2][128];
  __shared__ __attribute__((aligned(16))) double cb[2][128];
  __shared__ __attribute__((aligned(16))) double redw[2][2 * NWB];  // (S1, S2) of each bulk wave
  __shared__ __attribute__((aligned(16))) double scal[2][2];         // v0, beta of the reflector
  __shared__ double dg[128], e2[128];
  __shared__ __attribute__((aligned(16))) double sd[128], se[128];
  __shared__ double bnd[2];
  __shared__ unsigned long long masks[8];
  __shared__ double amaxw[NWB];
  const MatDesc<double> d = descs[blockIdx.x];
  const int n = d.n, lda = d.lda, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const bool chain = w == NWB;
  const int blk = w < 4 ? w : 11 - w;  // bulk row block (pairs 0/7, 1/6, 2/5, 3/4 per SIMD)
  const int c = lane >> 4, t16 = lane & 15;
  const int i = blk * 16 + t16;       // bulk: this lane's row
  const int j0 = 2 * c + 8 * t16;     // this lane's column pair (bulk: broadcast slot; chain: x_j)
  double a[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s) a[s][0] = a[s][1] = 0.0;
  if (!chain) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * c + 8 * s + e;
        const int ic = min(i, n - 1), jc = min(j, n - 1);
        const double v = gload(d.A + ic + (size_t)jc * lda);
        a[s][e] = (i < n && j < n) ? v : 0.0;
      }
    double amax = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) amax = fmax(amax, fmax(fabs(a[s][0]), fabs(a[s][1])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
    if (lane == 0) amaxw[w] = amax;
  }
  __syncthreads();
  int ex0;
  {
    double amax = amaxw[0];
#pragma unroll
    for (int r = 1; r < NWB; ++r) amax = fmax(amax, amaxw[r]);
    ex0 = (amax > 0.0 && amax < INFINITY) ? __builtin_amdgcn_frexp_exp(amax) : 0;
  }
  if (!chain) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      a[s][0] = __builtin_ldexp(a[s][0], -ex0);
      a[s][1] = __builtin_ldexp(a[s][1], -ex0);
    }
  }
  auto publish_row = [&](int r, double* dst) {  // the owners of row r write its 128 entries
    if (!chain && blk == (r >> 4) && t16 == (r & 15)) {
#pragma unroll
      for (int s = 0; s < NS; ++s)
        *reinterpret_cast<double2*>(dst + 2 * c + 8 * s) = make_double2(a[s][0], a[s][1]);
    }
  };
  // chain: v of the current step at the lane's column pair
  double cx = 0.0, cy = 0.0;
  // the reflector of row r from x = row r of the current matrix (chain wave only): v_j = 0
  // (j <= r), v0 (j = r+1), x_j (j > r+1), H = I - beta v v^T; v0 and beta go to scal[r & 1]
  auto reflector = [&](int r, double xj0, double xj1, double xr, double x0) {
    double tl = (j0 >= r + 2 ? xj0 * xj0 : 0.0);
    tl = fma(j0 + 1 >= r + 2 ? xj1 : 0.0, xj1, tl);
    tl = xsum32(xsum16(row16_sum(tl)));  // sum_{j >= r+2} x_j^2
    double bt = 0.0, v0 = x0, e2r = x0 * x0;
    if (tl > 0.0) {
      const double ss = fma(x0, x0, tl);
      double nrm;
      if (ss > 0x1p-900) {  // Newton-refined hardware rsq / rcp (~1 ulp)
        double rs = __builtin_amdgcn_rsq(ss);
        rs = rs * fma(-0.5 * ss, rs * rs, 1.5);
        nrm = ss * rs;
        nrm = fma(fma(-nrm, nrm, ss), 0.5 * rs, nrm);
      } else {
        nrm = sqrt(ss);
      }
      const double alpha = x0 > 0.0 ? -nrm : nrm;
      v0 = x0 - alpha;
      const double q = fma(v0, v0, tl);
      double rc = __builtin_amdgcn_rcp(q);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      bt = 2.0 * rc;
      e2r = alpha * alpha;
    }
    cx = j0 <= r ? 0.0 : (j0 == r + 1 ? v0 : xj0);
    cy = j0 + 1 <= r ? 0.0 : (j0 + 1 == r + 1 ? v0 : xj1);
    if (lane == 0) {
      *reinterpret_cast<double2*>(scal[r & 1]) = make_double2(v0, bt);
      dg[r] = xr;
      e2[r] = e2r;
    }
  };
  // bulk state carried from step to step: x~ at the column pair and at the own row, and the
  // own row's q and c (full sums, in every lane of the row)
  double xt0 = 0.0, xt1 = 0.0, xti = 0.0, qi = 0.0, ci = 0.0;
  // the bulk's product with the freshly updated registers: q = A x~ (x~ at the pair in xt0/xt1,
  // zero at columns < r + 2), c = column r + 1, the partials S1 = x~^T q, S2 = x~^T c; to LDS
  // buffer r & 1 (read by the step that applies reflector r)
  auto product = [&](int r, int lo, bool live) {
    double pa[4] = {0.0, 0.0, 0.0, 0.0};
    double cp = 0.0;
    const int sc = (r + 1) >> 3;
    // (the column's entry picked by weights, not by a select of a[s][0] / a[s][1]: a runtime
    // choice between them became an address select and put a[][] in scratch)
    const double m1 = ((r + 1) & 1) ? 1.0 : 0.0, m0 = 1.0 - m1;
    if (live && !(DBG & 2)) {
      static_for<0, NS / GS>([&](auto G) {
        constexpr int g = decltype(G)::value;
        if (GS * g + GS - 1 >= lo) {
          static_for<GS * g, GS * g + GS>([&](auto S) {
            constexpr int s = decltype(S)::value;
            fmac_bcast<s, s == GS * g>(pa[2 * (s & 1)], xt0, a[s][0]);
            fmac_bcast<s, false>(pa[2 * (s & 1) + 1], xt1, a[s][1]);
            if (s == sc) cp = fma(a[s][1], m1, a[s][0] * m0);
          });
        }
      });
    }
    cp = (c == (((r + 1) >> 1) & 3)) ? cp : 0.0;
    const double qq = xsum32(xsum16((pa[0] + pa[1]) + (pa[2] + pa[3])));
    const double cc = xsum32(xsum16(cp));
    double t1 = 0.0, t2 = 0.0;
    if (c == 0) {
      qb[r & 1][i] = qq;
      cb[r & 1][i] = cc;
      t1 = xti * qq;
      t2 = xti * cc;
    }
    t1 = row16_sum(t1);
    t2 = row16_sum(t2);
    if (lane == 0) *reinterpret_cast<double2*>(&redw[r & 1][2 * w]) = make_double2(t1, t2);
    qi = qq;
    ci = cc;
  };
  publish_row(0, rowb[0]);
  if (n >= 2) publish_row(1, rowb[1]);
  __syncthreads();
  if (chain) {
    __builtin_amdgcn_s_setprio(3);
    if (n >= 2) {
      const double2 xr = *reinterpret_cast<const double2*>(&rowb[0][j0]);
      reflector(0, xr.x, xr.y, rowb[0][0], rowb[0][1]);
    } else if (lane == 0) {
      dg[0] = rowb[0][0];
    }
  } else if (n >= 2) {
    // x~_0 = row 0 beyond column 1; q = A_0 x~_0, c = A_0 e_1
    const double2 o2 = *reinterpret_cast<const double2*>(&rowb[0][j0]);
    xt0 = j0 >= 2 ? o2.x : 0.0;
    xt1 = j0 + 1 >= 2 ? o2.y : 0.0;
    xti = i >= 2 ? rowb[0][i] : 0.0;
    product(0, 0, blk * 16 < n);
  }
  __syncthreads();
  for (int k = 0; k + 2 < n; ++k) {
    const int r = k + 1, par = k & 1, rp = r & 1;
    const int lo = (k + 1) >> 3;  // slots s < lo hold columns <= k only
    // ---- scalars of step k, identical in every wave: v0, beta, p_r, v^T p, K, w_r, g_r
    const double2 sv = *reinterpret_cast<const double2*>(scal[par]);
    const double v0 = sv.x, bk = sv.y;
    double rw[2 * NWB];
#pragma unroll
    for (int q = 0; q < 2 * NWB; q += 2) {
      const double2 v2 = *reinterpret_cast<const double2*>(&redw[par][q]);
      rw[q] = v2.x;
      rw[q + 1] = v2.y;
    }
    const double pr = fma(v0, cb[par][r], qb[par][r]);
    const double2 q2 = *reinterpret_cast<const double2*>(&qb[par][j0]);
    const double2 c2 = *reinterpret_cast<const double2*>(&cb[par][j0]);
    const double2 o = *reinterpret_cast<const double2*>(&rowb[rp][j0]);
    const double s1t = ((rw[0] + rw[2]) + (rw[4] + rw[6])) + ((rw[8] + rw[10]) + (rw[12] + rw[14]));
    const double s2t = ((rw[1] + rw[3]) + (rw[5] + rw[7])) + ((rw[9] + rw[11]) + (rw[13] + rw[15]));
    const double tot = fma(v0, pr, fma(v0, s2t, s1t));
    const double Kc = bk * bk * tot * 0.5;
    const double vr = v0;
    const double wr = fma(bk, pr, -(Kc * vr));
    const double gr = fma(Kc, vr, -wr), mhr = -(bk * vr);
    // p_k at the column pair (zero at the dead columns <= k)
    const double px = j0 > k ? fma(v0, c2.x, q2.x) : 0.0;
    const double py = j0 + 1 > k ? fma(v0, c2.y, q2.y) : 0.0;
    if (chain) {
      // ---- row r of A_{k+1} and the reflector v_{k+1} (cx, cy: v_k at the pair)
      const double orr = rowb[rp][r], or1 = rowb[rp][r + 1];
      const double pr1 = fma(v0, cb[par][r + 1], qb[par][r + 1]);
      const int ix = r + 1;  // v_k[r + 1] from the lane holding that column pair
      const double vr1 = readlane_d((ix & 1) ? cy : cx, 16 * ((ix >> 1) & 3) + (ix >> 3));
      const double xj0 = fma(cx, gr, fma(px, mhr, o.x));
      const double xj1 = fma(cy, gr, fma(py, mhr, o.y));
      const double xr = fma(vr, gr, fma(pr, mhr, orr));
      const double x0 = fma(vr1, gr, fma(pr1, mhr, or1));
      if constexpr (DBG & 4) {  // (timing only: no reflector)
        cx = xj0;
        cy = xj1;
        if (lane == 0) {
          *reinterpret_cast<double2*>(scal[r & 1]) = make_double2(x0, 0.0);
          dg[r] = xr;
          e2[r] = 1.0;
        }
      } else {
        reflector(r, xj0, xj1, xr, x0);
      }
    } else {
      const bool live = blk * 16 + 15 >= k + 2 && blk * 16 < n;
      if (live) {
        // v_k at the pair and the own row; p_k at the own row; w_i, g_i, h_i
        const double vx = j0 == r ? v0 : xt0;
        const double vy = j0 + 1 == r ? v0 : xt1;
        const double vi = i == r ? v0 : xti;
        const double pi = fma(v0, ci, qi);
        const double wi = fma(bk, pi, -(Kc * vi));
        const double gi = fma(Kc, vi, -wi), mhi = -(bk * vi);
        // x~_{k+1} = row r of A_{k+1} beyond column r + 1 (the chain's formula)
        const double oi = rowb[rp][i];
        const double nx0 = fma(vx, gr, fma(px, mhr, o.x));
        const double nx1 = fma(vy, gr, fma(py, mhr, o.y));
        const double nxi = fma(vi, gr, fma(pi, mhr, oi));
        // ---- A_{k+1} = A_k - v w^T - w v^T: a_ij += h_i p_j + g_i v_j
        if (!(DBG & 1)) static_for<0, NS / GS>([&](auto G) {
          constexpr int g = decltype(G)::value;
          if (GS * g + GS - 1 >= lo) {
            static_for<GS * g, GS * g + GS>([&](auto S) {
              constexpr int s = decltype(S)::value;
              fmac_bcast<s, s == GS * g>(a[s][0], px, mhi);
              fmac_bcast<s, false>(a[s][1], py, mhi);
            });
            static_for<GS * g, GS * g + GS>([&](auto S) {
              constexpr int s = decltype(S)::value;
              fmac_bcast<s, false>(a[s][0], vx, gi);
              fmac_bcast<s, false>(a[s][1], vy, gi);
            });
          }
        });
        xt0 = j0 >= r + 2 ? nx0 : 0.0;
        xt1 = j0 + 1 >= r + 2 ? nx1 : 0.0;
        xti = i >= r + 2 ? nxi : 0.0;
        // ---- q = A_{k+1} x~, c = A_{k+1} e_{r+1} and the partials for step k + 1
        product(r, lo, true);
        publish_row(k + 2, rowb[par]);
      } else {
        // no row beyond k + 1 here: zero q, c and partials (rows >= n stay exactly zero)
        xt0 = xt1 = xti = 0.0;
        product(r, lo, false);
      }
    }
    __syncthreads();
  }
  if (chain) __builtin_amdgcn_s_setprio(0);
  // the last diagonal entry: row n-1 as its owners published it at the last step (or at the start)
  if (tid == 0 && n >= 2) dg[n - 1] = rowb[(n - 1) & 1][n - 1];
  __syncthreads();
  // Gershgorin interval, scaling and 512-way multisection: as eigmin_split
  int bnd_ex = 0;
  {
    double lo = INFINITY, hi = -INFINITY;
    if (tid < n) {
      double rr = 0.0;
      if (tid > 0) rr += sqrt(e2[tid - 1]);
      if (tid + 1 < n) rr += sqrt(e2[tid]);
      lo = dg[tid] - rr;
      hi = dg[tid] + rr;
    }
    if (w < 2) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o));
        hi = fmax(hi, __shfl_xor(hi, o));
      }
      if (lane == 0) {
        reinterpret_cast<double*>(masks)[2 * w] = lo;
        reinterpret_cast<double*>(masks)[2 * w + 1] = hi;
      }
    }
    __syncthreads();
    const double* m = reinterpret_cast<const double*>(masks);
    const double l = fmin(m[0], m[2]), h = fmax(m[1], m[3]);
    const double mag = fmax(fabs(l), fabs(h));
    const int ex = (mag > 0.0 && mag < INFINITY) ? __builtin_amdgcn_frexp_exp(mag) : 0;
    bnd_ex = ex;
    if (tid < 128) {
      sd[tid] = tid < n ? __builtin_ldexp(dg[tid], -ex) : 4.0;
      se[tid] = (tid >= 1 && tid < n) ? fmax(__builtin_ldexp(e2[tid - 1], -2 * ex), 0x1p-900) : 0.0;
    }
    if (tid == 0) {
      const double ls = __builtin_ldexp(l, -ex), hs = __builtin_ldexp(h, -ex);
      const double span = hs - ls;
      bnd[0] = ls - span * 1e-3 - 1e-300;
      bnd[1] = hs + span * 1e-3 + 1e-300;
    }
  }
  __syncthreads();
  double lo = bnd[0], hi = bnd[1];
  const int nr = (n + 7) & ~7;
  constexpr double NSIG = 64.0 * NWB + 1.0;
  for (int it = 0; it < 6; ++it) {
    const double width = hi - lo;
    if (w < NWB) {
      const double sigma = lo + width * ((double)(tid + 1) / NSIG);
      const bool below = sturm_any_below(sd, se, nr, sigma);
      const unsigned long long mk = __ballot(below);
      if (lane == 0) masks[w] = mk;
    }
    __syncthreads();
    int f = -1;
    for (int q = 0; q < NWB && f < 0; ++q)
      if (masks[q]) f = q * 64 + __ffsll((long long)masks[q]) - 1;
    __syncthreads();
    if (f < 0) {
      lo = lo + width * ((NSIG - 1.0) / NSIG);
    } else {
      hi = lo + width * ((double)(f + 1) / NSIG);
      if (f > 0) lo = lo + width * ((double)f / NSIG);
    }
  }
  if (tid == 0) out[blockIdx.x] = __builtin_ldexp((lo + hi) * 0.5, bnd_ex + ex0);
}

#ifdef CLRSDP_EIG_STAMPS
__device__ unsigned long long g_eig_stamps[8];
#define EIG_STAMP(slot)                                                     \
  if (tid == 0) {                                                           \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                   \
    atomicAdd(&g_eig_stamps[slot], t_ - t_prev);                           \
    t_prev = t_;                                                            \
  }
#else
#define EIG_STAMP(slot)
#endif
// Wave sum of a (multi-word) value by DPP and permlane swaps, limb by limb, with the word
// type's own addition at every step (commutative, so partner lanes agree): against the
// ds_bpermute butterfly of wave_sum, whose six dependent LDS-unit round trips per limb set the
// reflector's critical path in eigmin_lds.
template <int CTRL, class T>
__device__ inline T dpp_mw(const T& v) {
  T o;
  const double* a = reinterpret_cast<const double*>(&v);
  double* b = reinterpret_cast<double*>(&o);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(T) / 8); ++q) b[q] = dpp_d<CTRL>(a[q]);
  return o;
}
__device__ inline double swap32_d(double x) {  // value of lane ^ 32
  const auto rl = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(x), false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(x), false, false);
  const bool low = __lane_id() < 32;
  return low ? __hiloint2double(rh[1], rl[1]) : __hiloint2double(rh[0], rl[0]);
}
template <int SW, class T>
__device__ inline T swap_mw(const T& v) {
  T o;
  const double* a = reinterpret_cast<const double*>(&v);
  double* b = reinterpret_cast<double*>(&o);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(T) / 8); ++q) b[q] = SW == 16 ? swap16_d(a[q]) : swap32_d(a[q]);
  return o;
}
template <class T>
__device__ inline T wave_sum_mw(T v) {
  v = v + dpp_mw<0xB1>(v);   // quad_perm [1,0,3,2]
  v = v + dpp_mw<0x4E>(v);   // quad_perm [2,3,0,1]
  v = v + dpp_mw<0x141>(v);  // row_half_mirror
  v = v + dpp_mw<0x140>(v);  // row_mirror
  v = v + swap_mw<16>(v);
  v = v + swap_mw<32>(v);
  return v;
}
// The same butterfly when only lane 0 needs the sum and only lanes 0..m-1 hold nonzero values:
// after level L lane 0 holds the sum of lanes 0..2^L - 1, so the levels past ceil(log2 m) would
// only add zeros (uniform branches on m).  eigmin_lds2's v^T p partials live on lanes 0-7 and
// its reflector norms on the first m = n - c - 1 lanes: half of the multi-word additions of
// those two sums are dropped from the per-column chain.
template <class T>
__device__ inline T lane0_sum_mw(T v, int m) {
  if (m > 1) v = v + dpp_mw<0xB1>(v);
  if (m > 2) v = v + dpp_mw<0x4E>(v);
  if (m > 4) v = v + dpp_mw<0x141>(v);
  if (m > 8) v = v + dpp_mw<0x140>(v);
  if (m > 16) v = v + swap_mw<16>(v);
  if (m > 32) v = v + swap_mw<32>(v);
  return v;
}

// exact power-of-two scaling of every limb
__device__ inline double scale2(double v, int e) { return ldexp(v, e); }
__device__ inline mw::dd scale2(const mw::dd& v, int e) { return mw::dd(ldexp(v.hi, e), ldexp(v.lo, e)); }
__device__ inline mw::qd scale2(const mw::qd& v, int e) {
  return mw::qd(ldexp(v.x[0], e), ldexp(v.x[1], e), ldexp(v.x[2], e), ldexp(v.x[3], e));
}
// The half-width word of a multi-word type and the rounding to it (the leading words of the
// non-overlapping representation).
template <class T> struct HalfWord;
template <> struct HalfWord<double> {
  using type = double;
  __device__ static double half(double v) { return v; }
};
template <> struct HalfWord<mw::dd> {
  using type = double;
  __device__ static double half(const mw::dd& v) { return v.hi; }
};
template <> struct HalfWord<mw::qd> {
  using type = mw::dd;
  __device__ static mw::dd half(const mw::qd& v) { return mw::dd(v.x[0], v.x[1]); }
};
// Multi-word "count >= 1" of the Sturm sequence (some eigenvalue of the tridiagonal below sigma),
// division-free as sturm_any_below: with p_0 = 1 the count is >= 1 iff some leading principal
// minor p_i = (d_i - sigma) p_{i-1} - e2_{i-1} p_{i-2} is negative (a zero minor is followed by a
// nonzero one of the sign opposite to its predecessor's, as the pivot form's q = 0 -> +tiny
// convention counts it; a zero last minor is not counted there either).  (p_{i-1}, p_i) is
// rescaled by the power of two of the larger every 4 rows (exact), so no minor overflows.  Per
// row two multi-word products and two differences, against a multi-word division in the pivot
// form (sturm_count), whose fp64 division sequences made the multi-word rounds of the
// multisection 56 % of eigmin_lds<dd>.
template <class T>
__device__ __forceinline__ bool sturm_any_below_mw(const T* __restrict__ dg, const T* __restrict__ e2, int n,
                                   const T& sigma) {
  T pm = T(0.0), pc = T(1.0);
  bool neg = false;
  // groups of 4 rows: the group's coefficients are read and d_i - sigma formed ahead of the
  // chain (LDS latency and the differences off the dependent path), then one rescale
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    T dv[4], fv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      dv[u] = dg[i + u] - sigma;
      fv[u] = sel(i + u > 0, e2[i + u > 0 ? i + u - 1 : 0], T(0.0));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      T pn = dv[u] * pc - fv[u] * pm;
      // a zero minor followed by e2_i = 0 (a decoupled tridiagonal) would keep the recurrence
      // at zero and hide every later sign change: count it as negative (LAPACK's -pivmin),
      // as the fp64 count floors e2 at 2^-900
      if (Num<T>::hi(pn) == 0.0) pn = T(-__builtin_ldexp(fabs(Num<T>::hi(pc)), -300));
      neg = neg || (pn < T(0.0));
      pm = pc;
      pc = pn;
    }
    const double mx = fmax(fabs(Num<T>::hi(pc)), fabs(Num<T>::hi(pm)));
    if (mx > 0.0 && mx < INFINITY) {
      const int ex = __builtin_amdgcn_frexp_exp(mx);
      pc = scale2(pc, -ex);
      pm = scale2(pm, -ex);
    }
  }
  for (; i < n; ++i) {
    T pn = (dg[i] - sigma) * pc - sel(i > 0, e2[i > 0 ? i - 1 : 0], T(0.0)) * pm;
    if (Num<T>::hi(pn) == 0.0) pn = T(-__builtin_ldexp(fabs(Num<T>::hi(pc)), -300));
    neg = neg || (pn < T(0.0));
    pm = pc;
    pc = pn;
  }
  return neg;
}

// the multi-word count >= 1 tests (CLRSDP_EIG_PIVOT_COUNT: the pivot form, for A/B timing)
#ifdef CLRSDP_EIG_PIVOT_COUNT
#define ANY_BELOW(sg) (sturm_count(dg, e2, n, (sg)) >= 1)
#else
#define ANY_BELOW(sg) sturm_any_below_mw(dg, e2, n, (sg))
#endif
// The multisection phase of eigmin_lds / eigmin_lds2 (512 threads): lambda_min of the
// tridiagonal (dg, e2 = squared off-diagonals) in LDS to the word's precision, into
// out[blockIdx.x].  A is LDS scratch (>= 2n + 14 doubles), Wv one word of LDS scratch.
template <class T, bool NEWTON>
__device__ __forceinline__ void eig_multisection(const T* __restrict__ dg, const T* __restrict__ e2, int n,
                                 T* __restrict__ A, T* __restrict__ Wv, T* __restrict__ out) {
  constexpr int NT = 512, NW = 8;
  const int tid = threadIdx.x;
  if (n == 1) {
    if (tid == 0) out[blockIdx.x] = dg[0];
    return;
  }
  // ---- multisection, 256-way on waves 0-3 (8 bits per round), in two phases:
  //  (1) fp64 on the leading limbs of the tridiagonal: Gershgorin bracket, 8 rounds;
  //  (2) multi-word, started from the fp64 eigenvalue +- delta, where delta bounds the effect of
  //      the rounding to fp64 (Weyl: |dlambda| <= ||dT|| <= ~3 eps64 ||T||) and of the fp64 Sturm
  //      counts (exact for a matrix perturbed by a few eps64 relative), with a wide margin.  The
  //      bracket is checked with two multi-word counts (no eigenvalue below it, one below its top)
  //      and replaced by the Gershgorin bracket if the check fails.  About half the multi-word
  //      rounds of a multisection from the Gershgorin bracket.
  // The matrix image in LDS is no longer needed: it holds the fp64 copy and the round masks.
  double* dgh = reinterpret_cast<double*>(A);
  double* e2h = dgh + n;
  double* bnd = e2h + n;  // [0,1] Gershgorin bracket, [2,3] multi-word start bracket, [4] ok
  unsigned long long* masks = reinterpret_cast<unsigned long long*>(bnd + 6);
  for (int i = tid; i < n; i += NT) {
    dgh[i] = Num<T>::hi(dg[i]);
    e2h[i] = Num<T>::hi(e2[i]);
  }
  __syncthreads();
  if (tid == 0) {
    double glo = 0.0, ghi = 0.0;
    for (int i = 0; i < n; ++i) {
      double r = 0.0;
      if (i > 0) r += sqrt(e2h[i - 1]);
      if (i + 1 < n) r += sqrt(e2h[i]);
      const double a = dgh[i] - r, b = dgh[i] + r;
      if (i == 0 || a < glo) glo = a;
      if (i == 0 || b > ghi) ghi = b;
    }
    // the leading limbs and the fp64 sqrt differ from the exact bounds by ~eps64 relative
    const double span = ghi - glo, mag = fmax(fabs(glo), fabs(ghi));
    bnd[0] = glo - span * 1e-3 - mag * 1e-12 - 1e-300;
    bnd[1] = ghi + span * 1e-3 + mag * 1e-12 + 1e-300;
  }
  __syncthreads();
  const int w = tid >> 6, lane = tid & 63;
  // one 512-way round: the first of the 512 interior points with a count >= 1 (every thread
  // gets the same answer); returns its index, or -1 if none
  auto first_hit = [&](bool hit) -> int {
    const unsigned long long mk = __ballot(hit);
    if (lane == 0) masks[w] = mk;
    __syncthreads();
    int f = -1;
    for (int q = 0; q < NW && f < 0; ++q)
      if (masks[q]) f = q * 64 + __ffsll((long long)masks[q]) - 1;
    __syncthreads();
    return f;
  };
  {
    // 8 rounds of 256 division-free counts on waves 0-3 (64 bits of the Gershgorin span)
    double lo = bnd[0], hi = bnd[1];
    for (int it = 0; it < 8; ++it) {
      const double width = hi - lo;
      bool hit = false;
      if (tid < 256) hit = sturm_any_below_mw(dgh, e2h, n, lo + width * ((double)(tid + 1) / 257.0));
      const int f = first_hit(hit);
      if (f < 0) {
        lo = lo + width * (256.0 / 257.0);
      } else {
        hi = lo + width * ((double)(f + 1) / 257.0);
        if (f > 0) lo = lo + width * ((double)f / 257.0);
      }
    }
    if (tid == 0) {
      const double c = 0.5 * (lo + hi);
      const double mag = fmax(fabs(bnd[0]), fabs(bnd[1]));
      const double delta = 64.0 * (double)n * 2.3e-16 * mag + (hi - lo) + 1e-300;
      bnd[2] = c - delta;
      bnd[3] = c + delta;
    }
  }
  __syncthreads();
  if constexpr (NEWTON && Num<T>::BITS > 60) {  // (multi-word words only)
    // (2') Newton on det(T - sigma I) from the fp64 centre.  (Before round 3 only at qd: at dd the
    // 11 parallel multisection rounds were as fast as the sequential chain of divisions.)  With the pivots of
    // T - sigma I = L D L^T, q_i = (d_i - sigma) - e2_{i-1} / q_{i-1}, and s_i = dq_i/dsigma =
    // -1 + e2_{i-1} s_{i-1} / q_{i-1}^2, the Newton step is 1 / sum_i s_i / q_i.  It converges
    // quadratically from the fp64 estimate (3 steps for a simple eigenvalue, a 4th confirms).
    // The result is accepted only if it converged AND two multi-word Sturm counts bracket it
    // (no eigenvalue below sigma - delta, one at most sigma + delta, delta = 2^(12-BITS)
    // magnitudes); otherwise the multisection below runs as before.
    // Division-free (round 3): the step is p_n / p_n' with the three-term recurrence of the
    // leading principal minors and of their derivatives, p_i = (d_i - s) p_{i-1} - e2_{i-1}
    // p_{i-2}, p_i' = (d_i - s) p_{i-1}' - p_{i-1} - e2_{i-1} p_{i-2}', the four values rescaled
    // by one power of two per row (exact, the ratio is unchanged): four multi-word products per
    // row and one division per step, against a division and three products per row.  A step
    // below 2^(-BITS/2 - 24) of the magnitude is the last one (quadratic convergence puts the
    // next correction far below the word); the two Sturm counts below accept the result.
    // Mixed precision (round 3, late): the derivative recurrence runs in the half-width word H
    // (dd for qd, fp64 for dd).  The step p/p' is a correction of the current error e, so a
    // relative error eta of p' only adds eta * e to the next error (quadratic convergence becomes
    // e^2 + eta e); p itself stays at full width.  At qd the first steps run entirely at dd
    // (from the fp64 centre to ~2^-100 of the magnitude), so only the last two steps carry qd
    // products, two per row instead of four.  The two Sturm counts below still decide.
    using H = typename HalfWord<T>::type;
    T* nres = Wv;  // free after the reduction: [0] = sigma
    const double mag = fmax(fabs(bnd[0]), fabs(bnd[1]));
    if (tid == 0) {
      T s = T(0.5 * (bnd[2] + bnd[3]));
      if constexpr (Num<T>::BITS > 150) {  // qd: dd pre-iterations on the dd-rounded tridiagonal
        H sh = H(0.5 * (bnd[2] + bnd[3]));
        const double tolh = ldexp(mag, -(Num<H>::BITS / 2 + 24)) + 1e-300;
        for (int it = 0; it < 3; ++it) {
          H pm = H(1.0), pc = HalfWord<T>::half(dg[0]) - sh, dm = H(0.0), dc = H(-1.0);
          for (int i = 1; i < n; ++i) {
            const H t = HalfWord<T>::half(dg[i]) - sh, e = HalfWord<T>::half(e2[i - 1]);
            const H pn = t * pc - e * pm;
            const H dn = (t * dc - pc) - e * dm;
            pm = pc;
            pc = pn;
            dm = dc;
            dc = dn;
            const double mx = fmax(fmax(fabs(Num<H>::hi(pc)), fabs(Num<H>::hi(pm))),
                                   fmax(fabs(Num<H>::hi(dc)), fabs(Num<H>::hi(dm))));
            if (mx > 0.0 && mx < INFINITY) {
              const int ex = __builtin_amdgcn_frexp_exp(mx);
              pc = scale2(pc, -ex);
              pm = scale2(pm, -ex);
              dc = scale2(dc, -ex);
              dm = scale2(dm, -ex);
            }
          }
          if (Num<H>::hi(dc) == 0.0) break;
          const H step = pc / dc;
          const double as = fabs(Num<H>::hi(step));
          if (!(as == as)) break;  // NaN: keep the last finite estimate
          sh = sh - step;
          if (as <= tolh) break;
        }
        s = T(sh);
      }
      const double tol = ldexp(mag, -(Num<T>::BITS / 2 + 24)) + 1e-300;
      int conv = 0;
      for (int it = 0; it < 4; ++it) {
        T pm = T(1.0), pc = dg[0] - s;
        H dm = H(0.0), dc = H(-1.0);
        for (int i = 1; i < n; ++i) {
          const T t = dg[i] - s;
          const T pn = t * pc - e2[i - 1] * pm;
          const H dn = (HalfWord<T>::half(t) * dc - HalfWord<T>::half(pc)) -
                       HalfWord<T>::half(e2[i - 1]) * dm;
          pm = pc;
          pc = pn;
          dm = dc;
          dc = dn;
          const double mx = fmax(fmax(fabs(Num<T>::hi(pc)), fabs(Num<T>::hi(pm))),
                                 fmax(fabs(Num<H>::hi(dc)), fabs(Num<H>::hi(dm))));
          if (mx > 0.0 && mx < INFINITY) {
            const int ex = __builtin_amdgcn_frexp_exp(mx);
            pc = scale2(pc, -ex);
            pm = scale2(pm, -ex);
            dc = scale2(dc, -ex);
            dm = scale2(dm, -ex);
          }
        }
        if (Num<H>::hi(dc) == 0.0) break;
        const T step = pc / T(dc);
        s = s - step;
        const double as = fabs(Num<T>::hi(step));
        if (!(as == as)) break;  // NaN: leave conv = 0
        if (as <= tol) { conv = 1; break; }
      }
      nres[0] = s;
      masks[2] = (unsigned long long)conv;
    }
    __syncthreads();
    const T s = nres[0];
    const T dl = T(ldexp(mag, 12 - Num<T>::BITS) + 1e-300);
    int c = 0;
    if (tid == 0) c = masks[2] && !ANY_BELOW(s - dl);
    if (tid == 64) c = ANY_BELOW(s + dl);
    __syncthreads();
    if (tid == 0 || tid == 64) masks[tid >> 6] = (unsigned long long)c;
    __syncthreads();
    const bool ok = masks[0] && masks[1];
    __syncthreads();
    if (ok) {
      if (tid == 0) out[blockIdx.x] = s;
      return;
    }
  }
  T lo = T(bnd[2]), hi = T(bnd[3]);
  // check the start bracket at full width: count(lo) == 0 and count(hi) >= 1
  {
    int c = 0;
    if (tid == 0) c = !ANY_BELOW(lo);
    if (tid == 64) c = ANY_BELOW(hi);
    if (tid == 0 || tid == 64) masks[tid >> 6] = (unsigned long long)c;
    __syncthreads();
    const bool ok = masks[0] && masks[1];
    __syncthreads();
    if (!ok) {
      lo = T(bnd[0]);
      hi = T(bnd[1]);
    }
    // rounds to shrink the bracket to ~2^-BITS of the spectrum's magnitude.  The multi-word
    // counts are VALU-issue bound, so they run 256-way on waves 0-3 (one wave per SIMD: 8 bits
    // per round) rather than 512-way on two waves per SIMD (9 bits per round at twice the issue)
#ifdef CLRSDP_EIG_MW512
    constexpr int MS = 512, MB = 9;
#else
    constexpr int MS = 256, MB = 8;
#endif
    constexpr double MD = MS + 1.0;
    // rounds to take the bracket below 2^-(BITS+2) of the magnitude (from its actual width:
    // the checked fp64 start bracket is ~64 n eps64 wide, so about 40 of the bits are known)
    int rounds = Num<T>::BITS / MB + 3;
    {
      const double wd = Num<T>::hi(hi - lo);
      const double mag = fmax(fabs(bnd[0]), fabs(bnd[1]));
      const double tgt = ldexp(mag, -(Num<T>::BITS + 2)) + 1e-300;
      if (wd > 0.0 && wd < INFINITY)
        rounds = min(rounds, max(1, (int)ceil(log2(wd / tgt) / (double)MB) + 1));
    }
    for (int it = 0; it < rounds; ++it) {
      const T width = hi - lo;
      bool hit = false;
      if (tid < MS) {  // wave-uniform
        const T sigma = lo + width * T((double)(tid + 1) / MD);
        hit = ANY_BELOW(sigma);
      }
      const int f = first_hit(hit);
      if (f < 0) {
        lo = lo + width * T((double)MS / MD);
      } else {
        hi = lo + width * T((double)(f + 1) / MD);
        if (f > 0) lo = lo + width * T((double)f / MD);
      }
    }
  }
  if (tid == 0) out[blockIdx.x] = (lo + hi) * T(0.5);
}

template <class T, bool NEWTON = true>
__global__ __launch_bounds__(512) void eigmin_lds(const MatDesc<T>* __restrict__ descs,
                                                  T* __restrict__ out) {
#ifdef CLRSDP_EIG_STAMPS
  unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#endif
  constexpr int NT = 512, NW = 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const MatDesc<T> d = descs[blockIdx.x];
  const int n = d.n, tid = threadIdx.x;
  // rows per pass and column classes of the matrix-vector product and the rank-2 update: every
  // wave holds rows when n <= 64 (64 rows x 8 classes), else 128 rows x 4 classes
  const int RW = n <= 64 ? 64 : 128, NC = NT / RW;
  T* A = reinterpret_cast<T*>(smem_raw);  // n x n
  T* v = A + (size_t)n * n;               // n
  T* p = v + n;                            // NC * n partials (eig_lds_bytes)
  T* dg = p + NC * n;                      // n
  T* e2 = dg + n;                          // n
  // coalesced load, then symmetrise in LDS: A = (A + A^T)/2
  for (int j = tid >> 6; j < n; j += NT / 64)
    for (int i = tid & 63; i < n; i += 64) A[i + (size_t)j * n] = d.A[i + (size_t)j * d.lda];
  __syncthreads();
  for (int j = tid >> 6; j < n; j += NT / 64)
    for (int i = tid & 63; i < j; i += 64) {
      const T sv = (A[i + (size_t)j * n] + A[j + (size_t)i * n]) * T(0.5);
      A[i + (size_t)j * n] = sv;
      A[j + (size_t)i * n] = sv;
    }
  __syncthreads();
  T* Wv = e2 + n;        // w vector (n)            -- carved after e2
  T* scal = Wv + n;      // [0] = beta, [1] = tail flag
  T* redw = scal + 4;    // NW partials of v^T A' v
  for (int k = 0; k + 2 < n; ++k) {
    const int m = n - k - 1;
    T* Ak = A + (k + 1) + (size_t)(k + 1) * n;  // trailing m x m, ld n
    // ---- (A) wave 0: reflector of column k
    if (tid < 64) {
      T s = T(0.0);
      for (int i = tid; i < m; i += 64) {
        const T xi = A[(k + 1 + i) + (size_t)k * n];
        v[i] = xi;
        s += xi * xi;
      }
      s = wave_sum_mw(s);
      const T x0 = A[(k + 1) + (size_t)k * n];
      const T tail = s - x0 * x0;
      if (tid == 0) {
        dg[k] = A[k + (size_t)k * n];
        if (!(tail > T(0.0))) {
          e2[k] = x0 * x0;
          scal[0] = T(0.0);  // beta = 0: no reflection
        } else {
          T nrm, rnrm;
          pivot_sqrt(s, nrm, rnrm);  // (dd: off the IEEE sqrt/division sequences)
          const T alpha = sel(x0 > T(0.0), -nrm, nrm);
          const T v0 = x0 - alpha;
          e2[k] = alpha * alpha;
          v[0] = v0;
          scal[0] = recip_fast(tail + v0 * v0) * T(2.0);
        }
      }
    }
    __syncthreads();
    EIG_STAMP(0)
    const T beta = scal[0];
    if (beta == T(0.0)) continue;  // uniform: nothing to update
    // ---- (B) partial rows of A'v (NC column classes) and v^T A' v
    const int ri = tid & (RW - 1), cq = tid / RW;
    T vav = T(0.0);
    for (int ii = ri; ii < m; ii += RW) {
      T a0 = T(0.0), a1 = T(0.0), a2 = T(0.0), a3 = T(0.0);
      int j = cq;
      for (; j + 3 * NC < m; j += 4 * NC) {
        a0 += Ak[ii + (size_t)j * n] * v[j];
        a1 += Ak[ii + (size_t)(j + NC) * n] * v[j + NC];
        a2 += Ak[ii + (size_t)(j + 2 * NC) * n] * v[j + 2 * NC];
        a3 += Ak[ii + (size_t)(j + 3 * NC) * n] * v[j + 3 * NC];
      }
      for (; j < m; j += NC) a0 += Ak[ii + (size_t)j * n] * v[j];
      const T part = (a0 + a1) + (a2 + a3);
      p[cq * n + ii] = part;
      vav += part * v[ii];
    }
    EIG_STAMP(1)
    vav = wave_sum_mw(vav);
    if ((tid & 63) == 0) redw[tid >> 6] = vav;
    __syncthreads();
    EIG_STAMP(2)
    // ---- (C) w = beta A'v - K v,  K = beta^2 v^T A' v / 2
    {
      // pairwise (three dependent multi-word additions instead of seven)
      const T tot = ((redw[0] + redw[1]) + (redw[2] + redw[3])) + ((redw[4] + redw[5]) + (redw[6] + redw[7]));
      const T Kc = beta * beta * tot * T(0.5);
      for (int i = tid; i < m; i += NT) {
        T ps = (p[i] + p[n + i]) + (p[2 * n + i] + p[3 * n + i]);
        if (NC == 8) ps = ps + ((p[4 * n + i] + p[5 * n + i]) + (p[6 * n + i] + p[7 * n + i]));
        Wv[i] = ps * beta - Kc * v[i];
      }
    }
    __syncthreads();
    EIG_STAMP(3)
    // ---- (D) A' -= v w^T + w v^T
    for (int ii = ri; ii < m; ii += RW) {
      const T vi = v[ii], wi = Wv[ii];
      int j = cq;
      for (; j + 3 * NC < m; j += 4 * NC) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          T* a = Ak + ii + (size_t)(j + u * NC) * n;
          *a = *a - (vi * Wv[j + u * NC] + wi * v[j + u * NC]);
        }
      }
      for (; j < m; j += NC) {
        T* a = Ak + ii + (size_t)j * n;
        *a = *a - (vi * Wv[j] + wi * v[j]);
      }
    }
    __syncthreads();
    EIG_STAMP(4)
  }
  EIG_STAMP(5)
  if (tid == 0) {
    if (n >= 2) {
      dg[n - 2] = A[(n - 2) + (size_t)(n - 2) * n];
      dg[n - 1] = A[(n - 1) + (size_t)(n - 1) * n];
      const T e = A[(n - 1) + (size_t)(n - 2) * n];
      e2[n - 2] = e * e;
    } else {
      dg[0] = A[0];
    }
  }
  __syncthreads();
  eig_multisection<T, NEWTON>(dg, e2, n, A, Wv, out);
  EIG_STAMP(6)
}

// ------------------------------------------------------------------------------------------
// eigmin_lds2: the Householder tridiagonalisation of eigmin_lds with two barriers per column
// instead of four, and the next reflector off the critical path.  The matrix is in LDS with a
// padded leading dimension (ld = 16 ceil(n/16) + 8, so the 16 lanes of an LDS pass hit distinct
// banks); thread (wave w, lane r + 8 c) owns row 64 q + 8 w + r (every pass q) and the column
// class j = c mod 8.  Per column k (trailing block k+1.., reflector v, beta):
//   (B) p_i = (A v)_i: the row's 8 class partials summed by DPP / permlane swaps inside the wave,
//       p -> LDS, the per-wave parts of v^T p -> LDS                              -- barrier
//   (D) with K = beta^2 v^T p / 2, g_i = beta p_i - 2K v_i and h_i = beta v_i (the row's own
//       values): a_ij -= h_i p_j + g_i v_j for every j > k of the thread's class (LDS reads of
//       p_j, v_j only; no w vector, no third barrier).  Column k+1 is skipped there: wave 0
//       forms its updated entries in registers and builds the next reflector from them (multi-
//       word norm, rsqrt pivot, reciprocal) while the other waves update     -- barrier
// The rows/columns <= k+1 are never read again, so column k+1 is not written back.
// ------------------------------------------------------------------------------------------
template <class T> __host__ __device__ constexpr int eig2_ld(int n) { return ((n + 15) / 16) * 16 + 8; }
template <class T> size_t eig2_lds_bytes(int n) {
  // A (n x ld), v (2 x ld), p (ld), dg, e2, scal (4), redw (2 x 8), + the tail's fp64 scratch
  return sizeof(T) * ((size_t)n * eig2_ld<T>(n) + 3 * (size_t)eig2_ld<T>(n) + 2 * (size_t)n + 4 + 16) + 64;
}
// The tridiagonalisation loop of eigmin_lds2 on the symmetric image A (n x ld in LDS, n >= 2,
// 512 threads): dg, e2 (and the last diagonal entry) when it returns.  KEEPV (fp64, eigmin_mx)
// also keeps every reflector: v_c in column c of V (n x n, rows c+1..n-1), beta_c in bet[c] and
// the signed off-diagonal T(c+1, c) in eo[c], so that A = Q T Q^T with Q = H_0 H_1 ... H_{n-2}.
template <class T, bool KEEPV>
__device__ __forceinline__ void tridiag_lds2(T* __restrict__ A, int ld, int n, T* __restrict__ vb,
                                             T* __restrict__ p, T* __restrict__ dg,
                                             T* __restrict__ e2, T* __restrict__ scal,
                                             T* __restrict__ redw, T* __restrict__ V,
                                             T* __restrict__ bet, T* __restrict__ eo) {
  // column slots per lane (j = cls + 8 t) and rows per lane in the reflector: a quad-double
  // image fits LDS only for n <= 64 (the launch checks it), so qd carries 8 slots and one row,
  // which keeps its per-lane words out of scratch
  constexpr int NSL = sizeof(T) > 16 ? 8 : 16, NH = sizeof(T) > 16 ? 1 : 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 7, cls = lane >> 3;
  const int npass = (n + 63) / 64;
  // reflector of column c from its entries x_i = col[i] (i > c; lane l holds rows c+1+l and
  // c+65+l), by wave 0: v into vb[c & 1], beta into scal[c & 1], dg[c] = diag, e2[c]
  auto reflector = [&](int c, const T (&x)[NH], const T& diag) {
    T s = T(0.0);
#pragma unroll
    for (int h = 0; h < NH; ++h) s += x[h] * x[h];
    s = lane0_sum_mw(s, n - c - 1);  // (only lane 0 uses s: beta, v0, e2[c])
    const T x0 = x[0];  // row c+1 (lane 0 is the only lane that uses x0, s and tail)
    const T tail = s - x0 * x0;
    T* v = vb + (c & 1) * ld;
    T beta = T(0.0), v0 = x0, e2c = x0 * x0, offd = x0;
    if (tail > T(0.0)) {
      T nrm, rnrm;
      if constexpr (std::is_same<T, double>::value) {  // (eigmin_mx) as eigmin_split's reflector
        if (s > 0x1p-900) {
          double rs = __builtin_amdgcn_rsq(s);
          rs = rs * fma(-0.5 * s, rs * rs, 1.5);
          nrm = s * rs;
          nrm = fma(fma(-nrm, nrm, s), 0.5 * rs, nrm);
        } else {
          nrm = sqrt(s);
        }
      } else {
        pivot_sqrt(s, nrm, rnrm);
      }
      const T alpha = sel(x0 > T(0.0), -nrm, nrm);
      v0 = x0 - alpha;
      e2c = alpha * alpha;
      offd = alpha;
      if constexpr (std::is_same<T, double>::value) {
        const double q = fma(v0, v0, tail);
        double rc = __builtin_amdgcn_rcp(q);
        rc = fma(fma(-q, rc, 1.0), rc, rc);
        rc = fma(fma(-q, rc, 1.0), rc, rc);
        beta = 2.0 * rc;
      } else {
        beta = recip_fast(tail + v0 * v0) * T(2.0);
      }
    }
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int i = c + 1 + lane + 64 * h;
      if (i < n) {
        const T vi = sel(i == c + 1, v0, x[h]);
        v[i] = vi;
        if constexpr (KEEPV) V[i + (size_t)c * n] = vi;
      }
    }
    if (lane < c + 1 && lane < ld) v[lane] = T(0.0);
    if (NH > 1 && lane + 64 < c + 1) v[lane + 64] = T(0.0);
    if (lane == 0) {
      dg[c] = diag;
      e2[c] = e2c;
      scal[c & 1] = beta;
      if constexpr (KEEPV) {
        bet[c] = beta;
        eo[c] = offd;
      }
    }
  };
  if (w == 0) {  // the reflector of column 0 from the input
    T x[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int i = 1 + lane + 64 * h;
      x[h] = T(0.0);
      if (i < n) x[h] = A[i];
    }
    reflector(0, x, A[0]);
  }
  __syncthreads();
  for (int k = 0; k + 2 < n; ++k) {
    const T* v = vb + (k & 1) * ld;
    const T beta = scal[k & 1];
    // ---- (B) p = A' v on the trailing block (rows and columns > k)
    T vp = T(0.0);
    for (int q = 0; q < npass; ++q) {
      const int i = 64 * q + 8 * w + r;
      // the class's columns j = cls + 8 t > k, t < 16 (n <= 128): compile-time slots, so the
      // independent multi-word products interleave (a runtime loop serialised their chains)
      T acc[4] = {T(0.0), T(0.0), T(0.0), T(0.0)};
      if (i > k && i < n) {
#pragma unroll
        for (int t = 0; t < NSL; ++t) {
          const int j = cls + 8 * t;
          if (j > k && j < n) acc[t & 3] += A[i + (size_t)j * ld] * v[j];
        }
      }
      T pi = (acc[0] + acc[1]) + (acc[2] + acc[3]);
      pi = pi + dpp_mw<0x128>(pi);   // row_ror:8  -> classes c, c^1
      pi = pi + swap_mw<16>(pi);     // classes c ^ 2
      pi = pi + swap_mw<32>(pi);     // classes c ^ 4
      if (cls == 0 && i < n) {
        p[i] = sel(i > k, pi, T(0.0));
        if (i > k) vp += v[i] * pi;
      }
    }
    vp = lane0_sum_mw(vp, 8);  // (nonzero on the class-0 lanes 0-7 only)
    if (lane == 0) redw[(k & 1) * 8 + w] = vp;
    __syncthreads();
    // ---- (D) A' -= v w^T + w v^T on rows/columns > k+1; wave 0: column k+1 and its reflector
    const T* rw = redw + (k & 1) * 8;
    const T tot = ((rw[0] + rw[1]) + (rw[2] + rw[3])) + ((rw[4] + rw[5]) + (rw[6] + rw[7]));
    const T K2 = beta * beta * tot;  // 2K
    const int c1 = k + 1;
    const T pc = p[c1], vc = v[c1];
    if (w == 0) {  // column c1 (rows > c1) and its diagonal, updated in registers
      T x[NH];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int i = c1 + 1 + lane + 64 * h;
        x[h] = T(0.0);
        if (i < n) {
          const T pi = p[i], vi = v[i];
          const T gi = beta * pi - K2 * vi, hi = beta * vi;
          x[h] = A[i + (size_t)c1 * ld] - (hi * pc + gi * vc);
        }
      }
      const T gc = beta * pc - K2 * vc, hc = beta * vc;
      const T diag = A[c1 + (size_t)c1 * ld] - (hc * pc + gc * vc);
      reflector(c1, x, diag);
    }
    for (int q = 0; q < npass; ++q) {
      const int i = 64 * q + 8 * w + r;
      if (i > c1 && i < n) {
        const T pi = p[i], vi = v[i];
        const T gi = beta * pi - K2 * vi, hi = beta * vi;
        // groups of 4 slots: all loads, then the 4 independent updates, then the stores (the
        // stores may alias later loads of the same LDS image, which would order every chain)
#pragma unroll
        for (int t0 = 0; t0 < NSL; t0 += 4) {
          if (cls + 8 * t0 >= n) break;  // (this lane has no live slot from t0 on)
          T av[4], pj[4], vj[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = cls + 8 * (t0 + u);
            const int jc = j < n ? j : n - 1;
            av[u] = A[i + (size_t)jc * ld];
            pj[u] = p[jc];
            vj[u] = v[jc];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) av[u] = av[u] - (hi * pj[u] + gi * vj[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = cls + 8 * (t0 + u);
            if (j > c1 && j < n) A[i + (size_t)j * ld] = av[u];
          }
        }
      }
    }
    __syncthreads();
  }
  // the last diagonal entry (updated by the last step's (D))
  if (tid == 0) dg[n - 1] = A[(n - 1) + (size_t)(n - 1) * ld];
  __syncthreads();
}

// DBG (timing experiments, tools/micro/eig2_mw.hip): 1 = stop after the tridiagonalisation
template <class T, bool NEWTON, int DBG>
__device__ __forceinline__ void eigmin_lds2_dev(const MatDesc<T>& d, T* __restrict__ out,
                                                char* __restrict__ smem_raw) {
  constexpr int NT = 512;
  const int n = d.n, tid = threadIdx.x, lane = tid & 63;
  const int ld = eig2_ld<T>(n);
  T* A = reinterpret_cast<T*>(smem_raw);      // n x ld, column-major
  T* vb = A + (size_t)n * ld;                 // 2 x ld: v of step k in vb[(k & 1) * ld]
  T* p = vb + 2 * ld;                          // ld
  T* dg = p + ld;                              // n
  T* e2 = dg + n;                              // n
  T* scal = e2 + n;                            // [0..1] beta of the two v buffers
  T* redw = scal + 4;                          // 2 x 8 per-wave parts of v^T p
  // coalesced load, then symmetrise: A = (A + A^T)/2
  for (int j = tid >> 6; j < n; j += NT / 64)
    for (int i = lane; i < n; i += 64) A[i + (size_t)j * ld] = d.A[i + (size_t)j * d.lda];
  __syncthreads();
  for (int j = tid >> 6; j < n; j += NT / 64)
    for (int i = lane; i < j; i += 64) {
      const T sv = (A[i + (size_t)j * ld] + A[j + (size_t)i * ld]) * T(0.5);
      A[i + (size_t)j * ld] = sv;
      A[j + (size_t)i * ld] = sv;
    }
  __syncthreads();
  if (n == 1) {
    if (tid == 0) out[blockIdx.x] = A[0];
    return;
  }
  tridiag_lds2<T, false>(A, ld, n, vb, p, dg, e2, scal, redw, nullptr, nullptr, nullptr);
  if constexpr (DBG == 1) {
    if (tid == 0) out[blockIdx.x] = dg[n - 1] + e2[0];
    return;
  }
  eig_multisection<T, NEWTON>(dg, e2, n, A, p, out);
}

// redo (eigmin_mx's fallback launch): only the blocks with redo[block] != 0
template <class T, bool NEWTON = true, int DBG = 0>
__global__ __launch_bounds__(512) void eigmin_lds2(const MatDesc<T>* __restrict__ descs,
                                                   T* __restrict__ out,
                                                   const int* __restrict__ redo = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if (redo && redo[blockIdx.x] == 0) return;
  eigmin_lds2_dev<T, NEWTON, DBG>(descs[blockIdx.x], out, smem_raw);
}
#undef ANY_BELOW

// ------------------------------------------------------------------------------------------
// eigmin_mx (round 4): multi-word lambda_min (n <= 64) from an fp64 eigenpair refined at the
// word's width, instead of a multi-word tridiagonalisation.  The reference computes lambda_min
// of L^-1 dM L^-T at BigFloat precision (compute_step_length, MPMP.jl:1857-1870); eigmin_lds2
// does so in double-double / quad-double arithmetic throughout, where every one of the n - 2
// columns is a chain of multi-word reductions, square roots and reciprocals (~5 us per column
// at dd).  Here:
//   1. A_h = the leading words of A_s = (A + A^T)/2, tridiagonalised in fp64 (tridiag_lds2,
//      keeping the reflectors): A_h = Q T Q^T.  T is rescaled by a power of two (|T| < 1).
//   2. fp64 lambda of T (512-way multisection) and a lower bound of its second eigenvalue: one
//      512-way round of full Sturm counts at lambda + span 2^(-t/8) (count <= 1 => lambda_2 >= ..).
//   3. z = its eigenvector (inverse iteration, tridiagonal LU with partial pivoting), x = Q z.
//   4. R refinement steps (1 at dd, 2 at qd): r = A_s x - rho x with rho = x^T A_s x / x^T x at
//      the full width (the only multi-word work: two or three n^2 matrix-vector products), then
//      the Newton correction (A - rho I) d = -r, d orthogonal to x, solved in fp64 through the
//      same Q and T: d = Q P (T - lambda I)^-1 P Q^T (-r), P = I - z z^T; x <- x + d (each step
//      multiplies the eigenvector error by ~eps64 ||A|| / gap).
//   5. rho of the final x.  Temple's bound: with ||r||^2 / ||x||^2 = eta and lambda_2 > rho,
//      rho - eta / (lambda_2 - rho) <= lambda_min <= rho.  rho is accepted when that width is
//      below 2^-(BITS+2) of the spectrum's magnitude; otherwise (a multiple or tightly
//      clustered lambda_min, or no separated lambda_2) the block is flagged and the launch
//      that follows (eigmin_lds2 with the flags) runs the multi-word path on it alone
//      (g_eigmx_fallbacks counts those).
// ------------------------------------------------------------------------------------------
__device__ unsigned int g_eigmx_fallbacks = 0;
template <class T> __host__ __device__ constexpr int eigmx_refine() { return 6; }
template <class T> size_t eigmx_own_bytes(int n) {
  const size_t ld = eig2_ld<double>(n), W = sizeof(T) / 8;
  return 8 * (128 + (size_t)n * ld + 3 * ld + 2 * (size_t)n + 4 + 16 + (size_t)n * n +
              2 * (size_t)n + 6 * (size_t)n + 64 + 8 + W * (size_t)n + 8 * W * (size_t)n) + 64;
}
// static LDS of split_tridiag_keepv (rowb, pb, vb, redw, betab, amaxw), on top of the dynamic size
constexpr size_t EIGMX_STATIC_LDS = 6400;
template <class T> size_t eigmx_lds_bytes(int n) { return eigmx_own_bytes<T>(n); }
// Sturm count of the (scaled, |T| < 1) tridiagonal in pivot form, pivots floored at 2^-900
__device__ __forceinline__ int sturm_count_piv(const double* __restrict__ dg,
                                               const double* __restrict__ e2, int n, double sigma) {
  constexpr double PIVMIN = 0x1p-900;
  int cnt = 0;
  double q = dg[0] - sigma;
  if (fabs(q) < PIVMIN) q = -PIVMIN;
  cnt += q < 0.0;
  for (int i = 1; i < n; ++i) {
    q = (dg[i] - sigma) - e2[i - 1] / q;
    if (fabs(q) < PIVMIN) q = -PIVMIN;
    cnt += q < 0.0;
  }
  return cnt;
}
// T - mu I = L D L^T for the (scaled) tridiagonal with mu just below lambda_1, so every pivot is
// positive in exact arithmetic (floored at 2^-900 against rounding): one thread, the pivot
// chain in registers, reciprocals by the hardware rcp and two Newton steps.  rd = 1 / D,
// ll = the subdiagonal of L.
__device__ __forceinline__ double rcp_nr(double q) {
  double r = __builtin_amdgcn_rcp(q);
  r = fma(fma(-q, r, 1.0), r, r);
  return fma(fma(-q, r, 1.0), r, r);
}
__device__ __forceinline__ void tri_ldl(const double* __restrict__ dg, const double* __restrict__ eo,
                                        int n, double mu, double* __restrict__ rd,
                                        double* __restrict__ ll) {
  constexpr double PIVMIN = 0x1p-900;
  double dcur = dg[0] - mu;
#pragma unroll 8
  for (int i = 0; i + 1 < n; ++i) {
    const double e = eo[i], an = dg[i + 1] - mu;
    const double r = rcp_nr(fmax(dcur, PIVMIN)), l = e * r;
    rd[i] = r;
    ll[i] = l;
    dcur = fma(-l, e, an);
  }
  rd[n - 1] = rcp_nr(fmax(dcur, PIVMIN));
}
// b <- (L D L^T)^-1 b, one thread
__device__ __forceinline__ void tri_ldl_solve(const double* __restrict__ rd,
                                              const double* __restrict__ ll, int n,
                                              double* __restrict__ b) {
  double y = b[0];
#pragma unroll 8
  for (int i = 1; i < n; ++i) {
    y = fma(-ll[i - 1], y, b[i]);
    b[i] = y;
  }
  double x = y * rd[n - 1];
  b[n - 1] = x;
#pragma unroll 8
  for (int i = n - 2; i >= 0; --i) {
    x = fma(b[i], rd[i], -ll[i] * x);
    b[i] = x;
  }
}
// eigmin_split's register-resident tridiagonalisation (576 threads: 8 bulk waves holding the
// matrix, one chain wave building each reflector once) on the fp64 image Ah (n x ld in LDS,
// n <= 128), keeping the reflectors for eigmin_mx: v_r in column r of V (n x n), beta_r in
// bet[r], the signed coupling T(r+1, r) in eo[r] and the diagonal in dg.  The image is scaled by
// 2^-ex0 (its largest entry below 1, as eigmin_split) and T comes out scaled alike; returns ex0.
// The DBG knobs and stamps of eigmin_split are left out; the arithmetic is the same.
__device__ __forceinline__ int split_tridiag_keepv(const double* __restrict__ Ah, int ld, int n,
                                                   double* __restrict__ dg, double* __restrict__ V,
                                                   double* __restrict__ bet,
                                                   double* __restrict__ eo) {
  constexpr int NS = 16, NWB = 8, GS = 4;
  __shared__ __attribute__((aligned(16))) double rowb[2][128];
  __shared__ __attribute__((aligned(16))) double pb[2][128];
  __shared__ __attribute__((aligned(16))) double vb[2][128];
  __shared__ __attribute__((aligned(16))) double redw[2][NWB];
  __shared__ double betab[2];
  __shared__ double amaxw[NWB];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const bool chain = w == NWB;
  const int blk = w < 4 ? w : 11 - w;
  const int c = lane >> 4, t16 = lane & 15;
  const int i = blk * 16 + t16;
  const int j0 = 2 * c + 8 * t16;
  double a[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s) a[s][0] = a[s][1] = 0.0;
  if (!chain) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * c + 8 * s + e;
        const int ic = min(i, n - 1), jc = min(j, n - 1);
        const double v = Ah[ic + (size_t)jc * ld];
        a[s][e] = (i < n && j < n) ? v : 0.0;
      }
    double amax = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) amax = fmax(amax, fmax(fabs(a[s][0]), fabs(a[s][1])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
    if (lane == 0) amaxw[w] = amax;
  }
  __syncthreads();
  int ex0;
  {
    double amax = amaxw[0];
#pragma unroll
    for (int r = 1; r < NWB; ++r) amax = fmax(amax, amaxw[r]);
    ex0 = (amax > 0.0 && amax < INFINITY) ? __builtin_amdgcn_frexp_exp(amax) : 0;
  }
  if (!chain) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      a[s][0] = __builtin_ldexp(a[s][0], -ex0);
      a[s][1] = __builtin_ldexp(a[s][1], -ex0);
    }
  }
  auto publish_row = [&](int r, double* dst) {
    if (!chain && blk == (r >> 4) && t16 == (r & 15)) {
#pragma unroll
      for (int s = 0; s < NS; ++s)
        *reinterpret_cast<double2*>(dst + 2 * c + 8 * s) = make_double2(a[s][0], a[s][1]);
    }
  };
  double cx = 0.0, cy = 0.0, beta = 0.0, vi = 0.0;
  auto reflector = [&](int r, double xj0, double xj1, double xr, double x0) {
    double tl = (j0 >= r + 2 ? xj0 * xj0 : 0.0);
    tl = fma(j0 + 1 >= r + 2 ? xj1 : 0.0, xj1, tl);
    tl = xsum32(xsum16(row16_sum(tl)));
    double bt = 0.0, v0 = x0, offd = x0;
    if (tl > 0.0) {
      const double ss = fma(x0, x0, tl);
      double nrm;
      if (ss > 0x1p-900) {
        double rs = __builtin_amdgcn_rsq(ss);
        rs = rs * fma(-0.5 * ss, rs * rs, 1.5);
        nrm = ss * rs;
        nrm = fma(fma(-nrm, nrm, ss), 0.5 * rs, nrm);
      } else {
        nrm = sqrt(ss);
      }
      const double alpha = x0 > 0.0 ? -nrm : nrm;
      v0 = x0 - alpha;
      const double q = fma(v0, v0, tl);
      double rc = __builtin_amdgcn_rcp(q);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      bt = 2.0 * rc;
      offd = alpha;
    }
    cx = j0 <= r ? 0.0 : (j0 == r + 1 ? v0 : xj0);
    cy = j0 + 1 <= r ? 0.0 : (j0 + 1 == r + 1 ? v0 : xj1);
    beta = bt;
    *reinterpret_cast<double2*>(&vb[r & 1][j0]) = make_double2(cx, cy);
    if (j0 < n) V[j0 + (size_t)r * n] = cx;
    if (j0 + 1 < n) V[j0 + 1 + (size_t)r * n] = cy;
    if (lane == 0) {
      dg[r] = xr;
      betab[r & 1] = bt;
      bet[r] = bt;
      eo[r] = offd;
    }
  };
  publish_row(0, rowb[0]);
  publish_row(1, rowb[1]);
  __syncthreads();
  if (chain) {
    __builtin_amdgcn_s_setprio(3);
    const double2 xr = *reinterpret_cast<const double2*>(&rowb[0][j0]);
    reflector(0, xr.x, xr.y, rowb[0][0], rowb[0][1]);
  }
  __syncthreads();
  if (!chain) {
    const double2 v2 = *reinterpret_cast<const double2*>(&vb[0][j0]);
    cx = v2.x;
    cy = v2.y;
    vi = vb[0][i];
    beta = betab[0];
  }
  for (int k = 0; k + 2 < n; ++k) {
    const int lo = (k + 1) >> 3;
    const int r = k + 1;
    double pp = 0.0;
    if (!chain) {
      const bool live = blk * 16 + 15 > k && blk * 16 < n;
      double pa[4] = {0.0, 0.0, 0.0, 0.0};
      if (live) {
        static_for<0, NS / GS>([&](auto G) {
          constexpr int g = decltype(G)::value;
          if (GS * g + GS - 1 >= lo) {
            static_for<GS * g, GS * g + GS>([&](auto S) {
              constexpr int s = decltype(S)::value;
              fmac_bcast<s, s == GS * g>(pa[2 * (s & 1)], cx, a[s][0]);
              fmac_bcast<s, false>(pa[2 * (s & 1) + 1], cy, a[s][1]);
            });
          }
        });
      }
      pp = xsum32(xsum16((pa[0] + pa[1]) + (pa[2] + pa[3])));
      double t = 0.0;
      if (c == 0) {
        pb[k & 1][i] = i > k ? pp : 0.0;
        t = vi * pp;
      }
      t = row16_sum(t);
      if (lane == 0) redw[k & 1][w] = t;
    }
    __syncthreads();
    if (chain) {
      double rw[NWB];
#pragma unroll
      for (int q = 0; q < NWB; q += 2) {
        const double2 v2 = *reinterpret_cast<const double2*>(&redw[k & 1][q]);
        rw[q] = v2.x;
        rw[q + 1] = v2.y;
      }
      const double* old = rowb[r & 1];
      const double2 pj = *reinterpret_cast<const double2*>(&pb[k & 1][j0]);
      const double2 o = *reinterpret_cast<const double2*>(old + j0);
      const double orr = old[r], or1 = old[r + 1];
      const double vr = vb[k & 1][r], vr1 = vb[k & 1][r + 1];
      const double pr = pb[k & 1][r], pr1 = pb[k & 1][r + 1];
      const double tot = ((rw[0] + rw[1]) + (rw[2] + rw[3])) + ((rw[4] + rw[5]) + (rw[6] + rw[7]));
      const double Kc = beta * beta * tot * 0.5;
      const double wr = fma(beta, pr, -(Kc * vr));
      const double gr = fma(Kc, vr, -wr), mhr = -(beta * vr);
      const double xj0 = fma(cx, gr, fma(pj.x, mhr, o.x));
      const double xj1 = fma(cy, gr, fma(pj.y, mhr, o.y));
      const double xr = fma(vr, gr, fma(pr, mhr, orr));
      const double x0 = fma(vr1, gr, fma(pr1, mhr, or1));
      reflector(r, xj0, xj1, xr, x0);
    } else if (blk * 16 + 15 > k + 1 && blk * 16 < n) {
      double rw[NWB];
#pragma unroll
      for (int q = 0; q < NWB; q += 2) {
        const double2 v2 = *reinterpret_cast<const double2*>(&redw[k & 1][q]);
        rw[q] = v2.x;
        rw[q + 1] = v2.y;
      }
      const double2 pv = *reinterpret_cast<const double2*>(&pb[k & 1][j0]);
      const double tot = ((rw[0] + rw[1]) + (rw[2] + rw[3])) + ((rw[4] + rw[5]) + (rw[6] + rw[7]));
      const double Kc = beta * beta * tot * 0.5;
      const double wi = fma(beta, pp, -(Kc * vi));
      const double gi = fma(Kc, vi, -wi), mhi = -(beta * vi);
      static_for<0, NS / GS>([&](auto G) {
        constexpr int g = decltype(G)::value;
        if (GS * g + GS - 1 >= lo) {
          static_for<GS * g, GS * g + GS>([&](auto S) {
            constexpr int s = decltype(S)::value;
            fmac_bcast<s, s == GS * g>(a[s][0], pv.x, mhi);
            fmac_bcast<s, false>(a[s][1], pv.y, mhi);
          });
          static_for<GS * g, GS * g + GS>([&](auto S) {
            constexpr int s = decltype(S)::value;
            fmac_bcast<s, false>(a[s][0], cx, gi);
            fmac_bcast<s, false>(a[s][1], cy, gi);
          });
        }
      });
      publish_row(k + 2, rowb[k & 1]);
    }
    __syncthreads();
    if (!chain) {
      const double2 v2 = *reinterpret_cast<const double2*>(&vb[r & 1][j0]);
      cx = v2.x;
      cy = v2.y;
      vi = vb[r & 1][i];
      beta = betab[r & 1];
    }
  }
  if (chain) __builtin_amdgcn_s_setprio(0);
  if (tid == 0) dg[n - 1] = rowb[(n - 1) & 1][n - 1];
  __syncthreads();
  return ex0;
}
// DBG: per-block diagnostics and phase stamps (s_memtime) in g_eigmx_dbg[block * 24 + slot]
__device__ double g_eigmx_dbg[256 * 24];
// DBG 2: block 0's fp64 data for a host check (V n x n, then dg, eo, bet, z, x, r, s, d', d by n)
__device__ double g_eigmx_dump[64 * 64 + 12 * 64];
// TRI = 1: the register-resident tridiagonalisation (split_tridiag_keepv, 576 threads; the
// ninth wave only builds reflectors), TRI = 0: tridiag_lds2 on 512 threads
template <class T, int DBG = 0, int TRI = 1>
__global__ __launch_bounds__(TRI ? 576 : 512) void eigmin_mx(const MatDesc<T>* __restrict__ descs,
                                                             T* __restrict__ out,
                                                             int* __restrict__ redo) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int NT = 512, NW = 8, R = eigmx_refine<T>();
  const MatDesc<T> d = descs[blockIdx.x];
  const int n = d.n, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double* dbg = DBG ? g_eigmx_dbg + (size_t)(blockIdx.x & 255) * 24 : nullptr;
  unsigned long long t_prev = DBG ? __builtin_amdgcn_s_memtime() : 0ull;
  auto stamp = [&](int slot) {
    if constexpr (DBG != 0) {
      if (tid == 0 && slot < 16) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        dbg[slot] = (double)(t - t_prev);
        t_prev = t;
      }
    }
  };
  bool ok = n >= 3;
  if (ok) {
    const int ld = eig2_ld<double>(n);
    double* sd = reinterpret_cast<double*>(smem_raw);  // 64 padded diagonal for the counts
    double* se = sd + 64;                              // 64 padded squared couplings
    double* A = se + 64;                               // n x ld
    double* vb = A + (size_t)n * ld;                   // 2 x ld
    double* p = vb + 2 * ld;                           // ld
    double* dg = p + ld;                               // n
    double* e2 = dg + n;                               // n
    double* scal = e2 + n;                             // 4
    double* redw = scal + 4;                           // 16
    double* V = redw + 16;                             // n x n reflectors
    double* bet = V + (size_t)n * n;                   // n
    double* eo = bet + n;                              // n signed off-diagonal
    double* rd = eo + n;                               // n  1 / D of T - mu I = L D L^T
    double* ll = rd + n;                               // n  L's subdiagonal
    double* wv = ll + 4 * n;                           // n  right-hand side / solution
    double* sc = wv + n;                               // 64 scalars
    unsigned long long* masks = reinterpret_cast<unsigned long long*>(sc + 64);  // 8
    T* xv = reinterpret_cast<T*>(masks + 8);           // n   the eigenvector estimate
    T* part = xv + n;                                  // 8 x n  row partials of A_s x
    // the symmetrised entries (row lane, columns j = w + NW u) of the lane, every load issued
    // before any is used (a loop over j waited on each strided load in turn, ~n / NW global
    // latencies per pass; n <= 64 so one row per lane and at most JM columns per wave)
    // (quad-double: in two halves of JH columns, registers)
    constexpr int JM = 64 / NW, JH = sizeof(T) > 16 ? JM / 2 : JM;
    auto load_sym = [&](T* sv, int u0) {
#pragma unroll
      for (int u = 0; u < JH; ++u) {
        const int j = w + NW * (u0 + u), jc = min(j, n - 1), ic = min(lane, n - 1);
        const T a1 = d.A[ic + (size_t)jc * d.lda], a2 = d.A[jc + (size_t)ic * d.lda];
        sv[u] = (a1 + a2) * T(0.5);
      }
    };
    // (1) leading words of the symmetrised block, then the fp64 tridiagonalisation
    if (w < NW && lane < n) {
#pragma unroll
      for (int u0 = 0; u0 < JM; u0 += JH) {
        T sv[JH];
        load_sym(sv, u0);
#pragma unroll
        for (int u = 0; u < JH; ++u) {
          const int j = w + NW * (u0 + u);
          if (j < n && lane >= j) {
            A[lane + (size_t)j * ld] = Num<T>::hi(sv[u]);
            A[j + (size_t)lane * ld] = Num<T>::hi(sv[u]);
          }
        }
      }
    }
    __syncthreads();
    stamp(0);
    int ex0 = 0;  // (TRI 1: T comes out scaled by 2^-ex0)
    if constexpr (TRI == 1) {
      ex0 = split_tridiag_keepv(A, ld, n, dg, V, bet, eo);
      for (int i = tid; i + 1 < n; i += NT) e2[i] = eo[i] * eo[i];
      __syncthreads();
    } else {
      tridiag_lds2<double, true>(A, ld, n, vb, p, dg, e2, scal, redw, V, bet, eo);
    }
    stamp(1);
    // Gershgorin bracket of T and the power of two that scales it below 1
    if (tid == 0) {
      double glo = 0.0, ghi = 0.0;
      for (int i = 0; i < n; ++i) {
        const double rr = (i > 0 ? fabs(eo[i - 1]) : 0.0) + (i + 1 < n ? fabs(eo[i]) : 0.0);
        const double a = dg[i] - rr, b = dg[i] + rr;
        if (i == 0 || a < glo) glo = a;
        if (i == 0 || b > ghi) ghi = b;
      }
      const double mag = fmax(fabs(glo), fabs(ghi));
      const bool fin = mag > 0.0 && mag < INFINITY;
      const int ex = fin ? __builtin_amdgcn_frexp_exp(mag) : 0;
      sc[0] = fin ? 1.0 : 0.0;
      sc[1] = (double)ex;
      sc[6] = (double)(ex + ex0);  // A's units -> the scaled T's
      const double span = ldexp(ghi - glo, -ex);
      sc[2] = ldexp(glo, -ex) - span * 1e-3 - 1e-300;
      sc[3] = ldexp(ghi, -ex) + span * 1e-3 + 1e-300;
    }
    __syncthreads();
    ok = sc[0] != 0.0;
    if (ok) {
      const int ex = (int)sc[1];
      for (int i = tid; i < n; i += NT) {
        dg[i] = ldexp(dg[i], -ex);
        e2[i] = ldexp(e2[i], -2 * ex);
        eo[i] = ldexp(eo[i], -ex);
      }
      __syncthreads();
      auto first_hit = [&](bool hit) -> int {
        const unsigned long long mk = __ballot(hit && tid < NT);
        if (lane == 0 && w < NW) masks[w] = mk;
        __syncthreads();
        int f = -1;
        for (int q = 0; q < NW && f < 0; ++q)
          if (masks[q]) f = q * 64 + __ffsll((long long)masks[q]) - 1;
        __syncthreads();
        return f;
      };
      // (2) lambda of T: eigmin_split's multisection (the padded fp64 arrays, 512-way on all 8
      // waves, 6 rounds of 9 bits = 2^-54 of the span)
      const int nr = (n + 7) & ~7;
      if (tid < nr) {
        sd[tid] = tid < n ? dg[tid] : 4.0;
        se[tid] = (tid >= 1 && tid < n) ? fmax(e2[tid - 1], 0x1p-900) : 0.0;
      }
      __syncthreads();
      double lo = sc[2], hi = sc[3];
      for (int it = 0; it < 6; ++it) {
        const double width = hi - lo;
        const bool hit = sturm_any_below(sd, se, nr, lo + width * ((double)(tid + 1) / 513.0));
        const int f = first_hit(hit);
        if (f < 0) {
          lo = lo + width * (512.0 / 513.0);
        } else {
          hi = lo + width * ((double)(f + 1) / 513.0);
          if (f > 0) lo = lo + width * ((double)f / 513.0);
        }
      }
      const double lam = 0.5 * (lo + hi), span = sc[3] - sc[2];
      // lower bound of lambda_2: the largest lam + span 2^(-t/4) (t < 256) with at most one
      // eigenvalue below it
      bool le1 = false;
      if (tid < 256) le1 = sturm_count_piv(dg, e2, n, lam + span * exp2(-(double)tid * 0.25)) <= 1;
      const int f2 = first_hit(le1);
      // the fp64 tridiagonal is within ~n eps64 |T| of A_s (backward stable, plus the rounding
      // of A_s to its leading words): a margin of 2^-40 of the scaled magnitude
      const double lam2 = f2 < 0 ? -INFINITY : lam + span * exp2(-(double)f2 * 0.25) - 0x1p-40;
      stamp(2);
      // (3) L D L^T of T - mu I, mu = lambda - 2^-48 span (below lambda_1: the bracket is 2^-54
      // span wide), and two inverse-iteration solves from the all-ones vector (thread 0; each
      // solve grows the vector by at most ~2^48, so no rescaling in between)
      const double mu = lam - span * 0x1p-48;
      if (tid == 0) {
        tri_ldl(dg, eo, n, mu, rd, ll);
        for (int i = 0; i < n; ++i) wv[i] = 1.0;
        tri_ldl_solve(rd, ll, n, wv);
        tri_ldl_solve(rd, ll, n, wv);
      }
      __syncthreads();
      stamp(3);
      // (3') wave 0: z = wv / ||wv||, x = Q z (reflectors n-3 .. 0), x / ||x||
      double zl = 0.0;  // (wave 0, lane l < n: z_l; kept in the register for the projections)
      // x <- Q x (H_{n-2} first) or Q^T x (H_0 first), lane l holding x_l: the next reflector's
      // entry is loaded ahead of the current one's wave sum.  (The last "reflector" H_{n-2} acts
      // on one entry: it is the identity unless the contracted tail s - x0^2 came out positive,
      // in which case it flips the sign of row n-1 and T's last coupling is -x0.)
      auto apply_q = [&](double xl, bool transpose) -> double {
        const int m = n - 1, dk = transpose ? 1 : -1;
        int k = transpose ? 0 : n - 2;
        double vk = lane > k && lane < n ? V[lane + (size_t)k * n] : 0.0, bk = bet[k];
        for (int s = 0; s < m; ++s) {
          const int kn = k + dk;
          double vn = 0.0, bn = 0.0;
          if (s + 1 < m) {
            vn = lane > kn && lane < n ? V[lane + (size_t)kn * n] : 0.0;
            bn = bet[kn];
          }
          const double t = wave_sum_mw<double>(vk * xl);
          xl -= (bk * t) * vk;
          vk = vn;
          bk = bn;
          k = kn;
        }
        return xl;
      };
      if (w == 0) {
        double zz = lane < n ? wv[lane] : 0.0;
        double mz = fabs(zz);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mz = fmax(mz, __shfl_xor(mz, o));
        zz = mz > 0.0 && mz < INFINITY ? zz / mz : 0.0;
        const double nz = sqrt(wave_sum_mw<double>(zz * zz));
        zl = nz > 0.0 ? zz / nz : 0.0;
        double xl = apply_q(zl, false);
        const double nx = sqrt(wave_sum_mw<double>(xl * xl));
        xl = nx > 0.0 ? xl / nx : 0.0;
        if (lane < n) xv[lane] = T(xl);
        if constexpr (DBG == 2) {
          if (blockIdx.x == 0 && lane < n) {
            double* dm = g_eigmx_dump + (size_t)n * n;
            dm[lane] = dg[lane];
            dm[n + lane] = eo[lane];
            dm[2 * n + lane] = bet[lane];
            dm[3 * n + lane] = zl;
            dm[4 * n + lane] = xl;
            for (int k = 0; k < n; ++k) g_eigmx_dump[lane + (size_t)k * n] = V[lane + (size_t)k * n];
            if (lane == 0) { dm[10 * n] = mu; dm[10 * n + 1] = sc[6]; }
          }
        }
        if (lane == 0) sc[4] = nz > 0.0 && nx > 0.0 ? 1.0 : 0.0;
      }
      __syncthreads();
      stamp(4);
      ok = sc[4] != 0.0;
      // (4)-(5) Rayleigh quotient and residual of x; accepted as soon as Temple's width is below
      // 2^-(BITS+2) of |T| < 1, else a refinement step (at most R = 6: a close lambda_2 slows
      // the refinement to ~2^-50 |T| / gap per step, and a few more steps of ~25 us are far
      // cheaper than the multi-word fallback)
      for (int it = 0; ok && it <= R; ++it) {
        // row partials of y = A_s x: row lane, columns j = w (mod 8)
        if (lane < n && w < NW) {
          T acc = T(0.0);
#pragma unroll
          for (int u0 = 0; u0 < JM; u0 += JH) {
            T sv[JH];
            load_sym(sv, u0);
#pragma unroll
            for (int u = 0; u < JH; ++u) {
              const int j = w + NW * (u0 + u);
              if (j < n) acc = acc + sv[u] * xv[j];
            }
          }
          part[w * n + lane] = acc;
        }
        __syncthreads();
        stamp(5 + 3 * it);
        if (w == 0) {
          T y = T(0.0), xl = T(0.0);
          if (lane < n) {
            xl = xv[lane];
            y = ((part[lane] + part[n + lane]) + (part[2 * n + lane] + part[3 * n + lane])) +
                ((part[4 * n + lane] + part[5 * n + lane]) + (part[6 * n + lane] + part[7 * n + lane]));
          }
          const T num = wave_sum_mw<T>(xl * y), den = wave_sum_mw<T>(xl * xl);
          const T rho = num / den;
          const T rr = y - rho * xl;
          const double rh = ldexp(Num<T>::hi(rr), -(int)sc[6]);  // scaled residual
          const double eta = wave_sum_mw<double>(rh * rh) / Num<T>::hi(den);
          if constexpr (DBG != 0) {
            if (lane == 0 && it < 4) dbg[16 + it] = eta;
          }
          const double rhs = ldexp(Num<T>::hi(rho), -(int)sc[6]);
          const double tw = lam2 > rhs ? eta / (lam2 - rhs) : INFINITY;
          const bool acc = tw <= 0x1p-3 * Num<T>::eps();  // 2^-(BITS+2) of |T| < 1
          if (lane == 0) {
            // accepted / rejected (the last step, or no lambda_2 bound above rho: Temple's bound
            // cannot hold however far x is refined) / refine
            sc[5] = acc ? 1.0 : ((it == R || !(lam2 > rhs)) ? -1.0 : 0.0);
            if (acc) out[blockIdx.x] = rho;
            if constexpr (DBG != 0) {
              dbg[20] = lam;
              dbg[21] = lam2;
              dbg[22] = rhs;
              dbg[23] = tw;
            }
          }
          if (!acc && it < R && lam2 > rhs) {
            // s = P Q^T (-r) in fp64 (scaled) -> wv for the solve
            double s = apply_q(-rh, true);
            s -= wave_sum_mw<double>(zl * s) * zl;
            if (lane < n) wv[lane] = s;
            if constexpr (DBG == 2) {
              if (blockIdx.x == 0 && it == 0 && lane < n) {
                double* dm = g_eigmx_dump + (size_t)n * n;
                dm[5 * n + lane] = rh;
                dm[6 * n + lane] = s;
              }
            }
          }
        }
        __syncthreads();
        if (sc[5] != 0.0) {
          ok = sc[5] > 0.0;
          break;
        }
        if (tid == 0) tri_ldl_solve(rd, ll, n, wv);  // (T - mu I) d' = s
        __syncthreads();
        stamp(6 + 3 * it);
        if (w == 0) {  // x += Q P d' (unscaled: the residual was scaled by 2^-ex)
          double dl = lane < n ? wv[lane] : 0.0;
          dl -= wave_sum_mw<double>(zl * dl) * zl;
          dl = apply_q(dl, false);
          if constexpr (DBG == 2) {
            if (blockIdx.x == 0 && it == 0 && lane < n) {
              double* dm = g_eigmx_dump + (size_t)n * n;
              dm[7 * n + lane] = wv[lane];
              dm[8 * n + lane] = dl;
            }
          }
          if (lane < n) xv[lane] = xv[lane] + T(dl);
        }
        __syncthreads();
        stamp(7 + 3 * it);
      }
    }
  }
  // redo[block] = 1: the multi-word path (eigmin_lds2, the next launch) takes this block (a
  // clustered lambda_min, or n < 3)
  if (tid == 0) {
    redo[blockIdx.x] = ok ? 0 : 1;
    if (!ok && n >= 3) atomicAdd(&g_eigmx_fallbacks, 1u);
  }
}

}  // namespace clrsdp

namespace clrsdp {

// ------------------------------------------------------------------------------------------
// Cholesky + inverse of one fp64 block on chip with MFMA (chol_inv_tiles, below) and its
// diagonal-tile step.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// One wave: Cholesky factor and inverse of the 16x16 diagonal tile at (k0, k0) of the LDS image,
// with no LDS round trip inside the column chain.  Lane l holds row i = l & 15 of A (-> L) and
// of X (-> L^-1) in full (each of the four 16-lane DPP rows is a replica).  Per column j the
// pivot comes by v_readlane and every l_k / x_jm by row_newbcast from the lane that owns it, so
// a column costs ~50 VALU instructions and one dependent chain (broadcast -> fma -> readlane ->
// rsq).  Writes L_kk back into the image and L_kk^-1 column-major into Dinv; a non-positive
// pivot sets *flag = k0 + 1.
// IDX(i, j) = offset of tile element (i, j) in the image (only i >= j is read and written).
template <class IDX>
__device__ inline void chol_diag16_bc(double* __restrict__ A, IDX idx, int k0,
                                     double* __restrict__ Dinv, int* flag, int lane) {
  const int i = lane & 15;
  double a[16], x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {  // symmetric tile from its lower triangle
    a[k] = A[idx(max(i, k), min(i, k))];
    x[k] = (k == i) ? 1.0 : 0.0;
  }
  // X = diag(r) Y: the rows of Y are left unscaled (y_i -= l_ij r_j y_j), and each lane
  // scales its own row by its pivot's 1/l_ii at the end
  int bad = 0;
  double rmine = 1.0;
  static_for<0, 16>([&](auto J) {
    constexpr int j = decltype(J)::value;
    const double d = readlane_d(a[j], j);
    bad |= !(d > 0.0);
    double r = __builtin_amdgcn_rsq(d);
    r = r * (1.5 - 0.5 * d * r * r);  // Newton step: r = 1/sqrt(d) to ~1 ulp
    const double lv = a[j] * r;       // l_ij (row j: sqrt(d))
    const double nl = (i > j) ? -lv : 0.0;
    const double nlr = nl * r;
    rmine = (i == j) ? r : rmine;
    a[j] = lv;
    // a_ik -= l_i l_k (k > j; the next pivot column first).  Only the first reads lv right
    // after its VALU write; the y sources were last written a column ago.
    static_for<j + 1, 16>([&](auto K) {
      constexpr int k = decltype(K)::value;
      fmac_bcast<k, k == j + 1>(a[k], lv, nl);
    });
    static_for<0, j + 1>([&](auto M) {
      constexpr int m = decltype(M)::value;
      fmac_bcast<j, j == 15 && m == 0>(x[m], x[m], nlr);
    });
  });
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] *= rmine;
  if (lane < 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k <= i) A[idx(i, k)] = a[k];
      Dinv[k * 16 + i] = x[k];  // column-major L_kk^-1 (zero above the diagonal)
    }
    if (lane == 0 && bad) *flag = k0 + 1;
  }
}

// chol_diag16_bc software-pipelined (same arithmetic, bit for bit): each column's pivot chain
// (readlane -> rsq -> Newton -> l_j -> the next pivot column's update) is the critical path, and
// the rest of the previous column's rank-1 update is issued inside it, in four pieces between
// its dependent steps (in-order issue: those FMAs fill the chain's latency instead of following
// it).  The inverse rows are split over the four 16-lane DPP rows: register s of DPP row g holds
// column 4s + g of this lane's row of X, so a column's inverse update is ceil((j+1)/4) FMAs,
// not j+1.
// LD(i, k): element (i, k) of the symmetric input tile (default: the lower triangle of the image)
template <class IDX, class LD>
__device__ inline void chol_diag16_pipe(double* __restrict__ A, IDX idx, LD ld, int k0,
                                        double* __restrict__ Dinv, int* flag, int lane) {
  const int i = lane & 15, g = lane >> 4;
  double a[16], x[4];
#pragma unroll
  for (int k = 0; k < 16; ++k) a[k] = ld(i, k);
#pragma unroll
  for (int s = 0; s < 4; ++s) x[s] = (4 * s + g == i) ? 1.0 : 0.0;
  int bad = 0;
  double rmine = 1.0, lvp = 0.0, nlp = 0.0, nlrp = 0.0;  // column j-1's l, -l and -l r
  // piece C (of 4) of column JP's bulk: a[JP+2 ..] -= l l_k, then x[s] (4s <= JP)
  auto bulk = [&](auto JP, auto C, auto NOP) {
    constexpr int jp = decltype(JP)::value, c = decltype(C)::value;
    constexpr int NA = jp < 14 ? 14 - jp : 0, N = NA + jp / 4 + 1;
    static_for<c * N / 4, (c + 1) * N / 4>([&](auto T) {
      constexpr int t = decltype(T)::value;
      if constexpr (t < NA) fmac_bcast<jp + 2 + t, false>(a[jp + 2 + t], lvp, nlp);
      else fmac_bcast<jp, decltype(NOP)::value && t == c * N / 4>(x[t - NA], x[t - NA], nlrp);
    });
  };
  using F = std::false_type;
  static_for<0, 16>([&](auto J) {
    constexpr int j = decltype(J)::value;
    constexpr auto JP = std::integral_constant<int, (j > 0 ? j - 1 : 0)>{};
    const double d = readlane_d(a[j], j);
    bad |= !(d > 0.0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (j > 0) bulk(JP, std::integral_constant<int, 0>{}, F{});
    __builtin_amdgcn_sched_barrier(0);
    double r = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (j > 0) bulk(JP, std::integral_constant<int, 1>{}, F{});
    __builtin_amdgcn_sched_barrier(0);
    const double t1 = hd * r;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (j > 0) bulk(JP, std::integral_constant<int, 2>{}, F{});
    __builtin_amdgcn_sched_barrier(0);
    const double t2 = 1.5 - t1 * r;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (j > 0) bulk(JP, std::integral_constant<int, 3>{}, F{});
    __builtin_amdgcn_sched_barrier(0);
    r = r * t2;
    const double lv = a[j] * r;
    const double nl = (i > j) ? -lv : 0.0;
    const double nlr = nl * r;
    rmine = (i == j) ? r : rmine;
    a[j] = lv;
    if constexpr (j < 15) fmac_bcast<j + 1, true>(a[j + 1], lv, nl);
    lvp = lv;
    nlp = nl;
    nlrp = nlr;
  });
  // column 15's bulk: the inverse update only
  static_for<0, 4>([&](auto C) { bulk(std::integral_constant<int, 15>{}, C, std::true_type{}); });
#pragma unroll
  for (int s = 0; s < 4; ++s) x[s] *= rmine;
  if (lane < 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k <= i) A[idx(i, k)] = a[k];
    if (lane == 0 && bad) *flag = k0 + 1;
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) Dinv[(4 * s + g) * 16 + i] = x[s];
}
template <class IDX>
__device__ inline void chol_diag16_pipe(double* __restrict__ A, IDX idx, int k0,
                                        double* __restrict__ Dinv, int* flag, int lane) {
  chol_diag16_pipe(A, idx, [&](int i, int k) { return A[idx(max(i, k), min(i, k))]; }, k0, Dinv, flag,
                   lane);
}

// ------------------------------------------------------------------------------------------
// chol_inv_tiles: A = L L^T and L^-1 for n <= NP (fp64), one 512-thread workgroup per matrix,
// with the off-diagonal 16x16 tiles resident in the worker waves' MFMA accumulators for the
// whole factorisation (no LDS round trip of the trailing matrix).  Tile (i, j), i > j, of the
// lower triangle belongs to worker (t mod 7), slot t / 7 (t = its row-major index); the slot
// holds A_ij^T in accumulator layout (register r of lane l = A_ij[l&15][(l>>4) + 4r]) until
// panel j turns it into L_ij, and X_ij = (L^-1)_ij (register r = X_ij[(l>>4) + 4r][l&15]) from
// then on.  Only the diagonal tiles, one 16-column panel of L, one 16-row block of X and the
// two diagonal inverses live in LDS (57 KB at NP = 128).  Per panel k:
//   (b) workers: L_ik^T = Linv_kk A_ik^T (the accumulator is exactly the B operand) -> LDS
//       panel; X_kj <- Linv_kk X_kj and X_kk = Linv_kk -> LDS row block;
//   (c) workers: A_ij^T -= L_jk L_ik^T, X_ij -= L_ik X_kj, diagonal tiles D_i -= L_ik L_ik^T;
//   wave 0, concurrently (look-ahead): as soon as L_{k+1,k} is in the panel, D_{k+1} -=
//       L L^T and its Cholesky + inverse (chol_diag16_bc, no LDS inside the column chain).
// The critical path per panel is one MFMA tile + the 16-column diagonal factorisation.
// ------------------------------------------------------------------------------------------
#ifdef CLRSDP_CHOL_TRACE
// [block][wave (up to 16)][point (up to 128)]
__device__ unsigned long long g_chol2_trace[256 * 16 * 128];
#define CT_TRACE() do { if ((threadIdx.x & 63) == 0 && tr_i < 128) g_chol2_trace[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 128 + tr_i] = __builtin_amdgcn_s_memtime(); ++tr_i; } while (0)
#else
#define CT_TRACE()
#endif
#ifndef CLRSDP_CHOL256_NTH
#define CLRSDP_CHOL256_NTH 768
#endif
template <int NP>
struct CholTiles {
  // NTH threads: one chain wave and NWK workers (512 up to NP = 128; 768 at NP = 256).  Wave 4
  // (a worker) shares SIMD 0 with the chain wave, and its f64 MFMAs slow the chain's VALU
  // chain by half (tools/micro/diag16_bench.hip); measured and rejected: no tiles on it (the
  // MFMA work then has three SIMDs: 32.7 vs 31.3 us at n = 128) or its trailing update held
  // back until the chain's diagonal factor is done (35.0 vs 31.4 us)
  static constexpr int NTH = NP > 128 ? CLRSDP_CHOL256_NTH : 512;
  static constexpr int NT = NP / 16, NOFF = NT * (NT - 1) / 2, NWK = NTH / 64 - 1;
  static constexpr int SLOTS = (NOFF + NWK - 1) / NWK, DSLOTS = (NT + NWK - 1) / NWK;
  static constexpr int LDD = 18;        // diagonal tiles: column-major 16 x 18
  static constexpr int XLD = NP + 16;   // X row block: 16 x XLD row-major
  static constexpr int DT = 0, PN = DT + NT * 16 * LDD, XR = PN + NT * 256, DI = XR + 16 * XLD,
                       END = DI + 512;  // doubles; the int flags follow
  static __device__ __forceinline__ void tile(int t, int& i, int& j) {  // row-major lower
    i = 1;
    while (i * (i + 1) / 2 <= t) ++i;
    j = t - i * (i - 1) / 2;
  }
};
template <int NP>
size_t chol_inv_tiles_lds() { return sizeof(double) * CholTiles<NP>::END + 16; }

template <int NP>
__global__ __launch_bounds__(CholTiles<NP>::NTH) void chol_inv_tiles(const MatDesc<double>* __restrict__ in,
                                                      const MatDesc<double>* __restrict__ out_inv,
                                                      int* __restrict__ info, int prio = 0) {
  using CT = CholTiles<NP>;
  // prio: the diagonal chain (wave 0) at priority 3, the workers at 2, above co-resident waves
  // of other launches (which stay at 0)
  if (prio) {
    if (threadIdx.x < 64) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(2);
  }
  constexpr int NT = CT::NT, NWK = CT::NWK, SLOTS = CT::SLOTS, DSLOTS = CT::DSLOTS;
  constexpr int LDD = CT::LDD, XLD = CT::XLD;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  double* Dt = reinterpret_cast<double*>(smem_raw) + CT::DT;  // diagonal tiles
  double* Pn = reinterpret_cast<double*>(smem_raw) + CT::PN;  // panel: L_ik column-major 16x16
  double* Xr = reinterpret_cast<double*>(smem_raw) + CT::XR;  // X row block k
  double* Di = reinterpret_cast<double*>(smem_raw) + CT::DI;  // Linv_kk by parity, col-major
  int* flag = reinterpret_cast<int*>(reinterpret_cast<double*>(smem_raw) + CT::END);
#ifdef CLRSDP_CHOL_TRACE
  int tr_i = 0;
#endif
  CT_TRACE();
  const MatDesc<double> d = in[blockIdx.x];
  // (the wave index through readfirstlane: the slot coordinates and every branch on them are
  // scalar, not per-lane registers)
  const int n = d.n, tid = threadIdx.x, lane = tid & 63,
            w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = (n + 15) / 16;
  const int lr = lane & 15, lk = lane >> 4;
  const int wk = w - 1;  // worker index, -1 for wave 0
  // The chain wave and the workers run separate copies of the panel loop (the same barriers in
  // the same order): the workers' accumulator slots are not live in the chain wave's code, so
  // the register allocation is the larger of the two paths, not their sum (NP = 256: 18 slots
  // per worker next to the chain's 32-register rows).
  const MatDesc<double> o = out_inv[blockIdx.x];
  // prologue: the diagonal tiles 1.. into LDS with identity padding (tile 0 is the chain wave's:
  // it factors D_0 straight from global memory while the other waves load); L^-1's tiles are
  // written as they become final (tile row k after panel k), so no store tail is left for the
  // end; the zero tiles above the diagonal first (never read: the input is read on and below the
  // diagonal only, so in place is safe).  All loads of the diagonal tiles are issued before the
  // first LDS store: one memory latency, not one per pass of the loop.
  constexpr int DPER = (NT * 256 + CT::NTH - 1) / CT::NTH;
  double dv[DPER];
  auto prologue_load = [&]() {
#pragma unroll
    for (int q = 0; q < DPER; ++q) {
      const int e = tid + q * CT::NTH;
      const int t = e >> 8, c = (e >> 4) & 15, r = e & 15;
      const int gi = min(16 * t + r, n - 1), gj = min(16 * t + c, n - 1);
      dv[q] = gload(d.A + gi + (size_t)gj * d.lda);
    }
    asm volatile("" ::: "memory");  // (the loads stay above: not sunk into the selects below)
  };
  auto prologue_store = [&]() {
#pragma unroll
    for (int q = 0; q < DPER; ++q) {
      const int e = tid + q * CT::NTH;
      if (e < 256 || e >= NT * 256) continue;
      const int t = e >> 8, c = (e >> 4) & 15, r = e & 15;
      const int gi = 16 * t + r, gj = 16 * t + c;
      double v = gi == gj ? 1.0 : 0.0;
      if (t < nt && gi < n && gj < n && r >= c) v = dv[q];
      Dt[t * 16 * LDD + c * LDD + r] = v;
    }
    for (int j = tid >> 4; j < n; j += CT::NTH / 16)
      for (int i = (tid & 15); i < (j & ~15); i += 16) o.A[i + (size_t)j * o.lda] = 0.0;
    lds_barrier();
    CT_TRACE();
  };
  if (wk < 0) {
    // ======================= the chain wave: the diagonal tiles, one panel ahead
    if (lane == 0) {  // (before D_0's factorisation, which may set flag[0])
      flag[0] = 0;  // first failing pivot + 1
      flag[1] = 0;  // panels whose L_{k+1,k} is in the panel buffer
      flag[2] = 0;  // worker arrivals at the (b) -> (c) barrier
    }
    prologue_load();
    chol_diag16_pipe(Dt, [](int i, int j) { return j * LDD + i; },
                     [&](int i, int k) {  // D_0 from global memory, identity-padded past n
                       const int r = max(i, k), c = min(i, k);
                       return r < n ? gload(d.A + r + (size_t)c * d.lda) : (i == k ? 1.0 : 0.0);
                     },
                     0, Di, flag, lane);
    prologue_store();
    lds_barrier();
    CT_TRACE();
    for (int k = 0; k < nt; ++k) {
      if (*flag) break;
      if (k + 1 < nt) {
        // D_{k+1} -= L L^T (L = L_{k+1,k}) and its factorisation
        // (the flags order LDS data only: relaxed LDS atomics and compiler fences, so neither
        // side waits for the workers' outstanding global stores of final L^-1 tiles)
        while (__hip_atomic_load(flag + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= k)
          __builtin_amdgcn_s_sleep(1);
        __atomic_signal_fence(__ATOMIC_ACQUIRE);
        CT_TRACE();
        const double* P = Pn + 256 * (k + 1);
        double* D = Dt + (k + 1) * 16 * LDD;
        d4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = D[lr * LDD + lk + 4 * r];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double f = P[(4 * r + lk) * 16 + lr];
          acc = mfma64(-f, f, acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) D[lr * LDD + lk + 4 * r] = acc[r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        chol_diag16_pipe(D, [](int i, int j) { return j * LDD + i; }, 16 * (k + 1),
                         Di + 256 * ((k + 1) & 1), flag, lane);
        CT_TRACE();
      }
      lds_barrier();
      CT_TRACE();
    }
  } else {
    // ======================= the workers
    // ---- tile coordinates of this worker's slots (wave-uniform)
    int TI[SLOTS], TJ[SLOTS];
#pragma unroll
    for (int q = 0; q < SLOTS; ++q) {
      const int t = wk + NWK * q;
      int ti = NT, tj = 0;  // empty slot: row NT is never active
      if (t < CT::NOFF) CT::tile(t, ti, tj);
      TI[q] = ti;
      TJ[q] = tj;
    }
    // ---- off-diagonal tiles straight into the accumulators (A_ij^T layout, coalesced along rows)
    d4 T[SLOTS];
#pragma unroll
    for (int q = 0; q < SLOTS; ++q) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 16 * TI[q] + lr, gj = 16 * TJ[q] + lk + 4 * r;
        T[q][r] = (TI[q] < nt && gi < n && gj < n) ? gload(d.A + gi + (size_t)gj * d.lda) : 0.0;
      }
    }
    d4 XD[DSLOTS];
#pragma unroll
    for (int q = 0; q < DSLOTS; ++q) XD[q] = d4{0.0, 0.0, 0.0, 0.0};
    prologue_load();
    prologue_store();
    lds_barrier();  // (the chain wave's first diagonal factor)
    CT_TRACE();
    for (int k = 0; k < nt; ++k) {
      if (*flag) break;
      // an opaque zero per panel: the per-slot LDS and store addresses below are formed where
      // they are used, not hoisted out of the loop (NP = 256: dozens of loop-invariant
      // addresses kept live across the panels spilled to scratch)
      int opq = 0;
      if constexpr (SLOTS > 6) asm volatile("" : "+s"(opq));
      double* const Pn_ = Pn + opq;
      double* const Xr_ = Xr + opq;
      double* const Dt_ = Dt + opq;
      double* const oA = o.A + opq;
      const double* Dk = Di + 256 * (k & 1);
      // ---------------- (b): Linv_kk as the A operand: a[r] = Linv[lr][4r+lk]
      double lopA[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) lopA[r] = Dk[(4 * r + lk) * 16 + lr];
      // the look-ahead tile L_{k+1,k} first (wave 0 waits for it)
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int q = 0; q < SLOTS; ++q) {
          if (TI[q] >= nt || TJ[q] != k) continue;
          if ((TI[q] == k + 1) != (pass == 0)) continue;
          d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int r = 0; r < 4; ++r) acc = mfma64(lopA[r], T[q][r], acc);  // L_ik^T
          double* P = Pn_ + 256 * TI[q];
#pragma unroll
          for (int r = 0; r < 4; ++r) P[(lk + 4 * r) * 16 + lr] = acc[r];  // L_ik[lr][lk+4r]
          if (pass == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __atomic_signal_fence(__ATOMIC_RELEASE);
            if (lane == 0) __hip_atomic_store(flag + 1, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < SLOTS; ++q) {  // X row block: X_kj <- Linv_kk X_kj (j < k)
        if (TI[q] != k) continue;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma64(lopA[r], T[q][r], acc);
        T[q] = acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Xr_[(lk + 4 * r) * XLD + 16 * TJ[q] + lr] = acc[r];
          const int gi = 16 * k + lk + 4 * r, gj = 16 * TJ[q] + lr;  // final: (L^-1)_kj
          if (gi < n && gj < n) oA[gi + (size_t)gj * o.lda] = acc[r];
        }
      }
      if (wk == k % NWK) {  // X_kk = Linv_kk (accumulator layout: register r = Linv[lk+4r][lr])
#pragma unroll
        for (int q = 0; q < DSLOTS; ++q)
          if (q == k / NWK) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              XD[q][r] = Dk[lr * 16 + lk + 4 * r];
              Xr_[(lk + 4 * r) * XLD + 16 * k + lr] = XD[q][r];
              const int gi = 16 * k + lk + 4 * r, gj = 16 * k + lr;  // final: (L^-1)_kk
              if (gi < n && gj < n) oA[gi + (size_t)gj * o.lda] = XD[q][r];
            }
          }
      }
      CT_TRACE();
      // workers-only barrier (wave 0 is busy with the next diagonal tile)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __atomic_signal_fence(__ATOMIC_RELEASE);
      if (lane == 0) __hip_atomic_fetch_add(flag + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      while (__hip_atomic_load(flag + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < NWK * (k + 1))
        __builtin_amdgcn_s_sleep(1);
      __atomic_signal_fence(__ATOMIC_ACQUIRE);
      CT_TRACE();
      // ---------------- (c) trailing update of the rows below k
      const double* Pk = Pn_;
#pragma unroll
      for (int q = 0; q < SLOTS; ++q) {
        const int ti = TI[q], tj = TJ[q];
        if (ti >= nt || ti <= k) continue;
        const double* Pi = Pk + 256 * ti;
        if (tj > k) {  // A_ij^T -= L_jk L_ik^T
          const double* Pj = Pk + 256 * tj;
          d4 acc = T[q];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc = mfma64(-Pj[(4 * r + lk) * 16 + lr], Pi[(4 * r + lk) * 16 + lr], acc);
          T[q] = acc;
        } else {  // X_ij -= L_ik X_kj (tj == k: the slot turns from L_ik into X_ik = -L_ik X_kk)
          d4 acc = tj == k ? d4{0.0, 0.0, 0.0, 0.0} : T[q];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc = mfma64(-Pi[(4 * r + lk) * 16 + lr], Xr_[(4 * r + lk) * XLD + 16 * tj + lr], acc);
          T[q] = acc;
        }
      }
      // diagonal tiles below the look-ahead one: D_i -= L_ik L_ik^T (in LDS)
#pragma unroll
      for (int q = 0; q < DSLOTS; ++q) {
        const int di = wk + NWK * q;
        if (di >= nt || di <= k + 1) continue;
        const double* Pi = Pk + 256 * di;
        double* D = Dt_ + di * 16 * LDD;
        d4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = D[lr * LDD + lk + 4 * r];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double f = Pi[(4 * r + lk) * 16 + lr];
          acc = mfma64(-f, f, acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) D[lr * LDD + lk + 4 * r] = acc[r];
      }
      CT_TRACE();
      lds_barrier();
      CT_TRACE();
    }
  }
  if (tid == 0 && info) info[blockIdx.x] = *flag;
  CT_TRACE();
}
#undef CT_TRACE


// ------------------------------------------------------------------------------------------
// The cluster part of the block solve (MPMP.jl:1751-1768) at fp64 with the explicit inverses, as
// two launches around slab_qsolve instead of four batched GEMVs (q_t, p_Wt | q_Wdy, q_dx):
//   cl_solve_t:  t = L^-1 rhs and this row block's share of W^T t   (one partial slab per block)
//   cl_solve_dx: u = t + W dy and dx = L^-T u                        (one column block of dx)
// L^-1 is the lower triangle of S_j in place (chol_inv_tiles; 2x2-blocked with X21 or not): row
// i only uses columns <= i, so the stale S12 above the diagonal is never read.  64-row / 64-column
// blocks, 4 waves; sums in a fixed order (deterministic).
// ------------------------------------------------------------------------------------------
struct ClSolveDesc {
  const double* L;    // D x D, column-major, ld D: L^-1 in the lower triangle
  const double* W;    // D x n_y, ld D: W = L^-1 B
  const double* rhs;  // D
  double* t;          // D: t = L^-1 rhs
  double* dx;         // D: dx = L^-T (t + W dy)
  int D, pad;
};

// Sum over the 64 lanes of each of the N values every lane holds, transposed: log2(N) halving
// steps (lane bit 5, 4, ... picks the half a lane keeps and adds its partner's copy of) and plain
// butterfly steps after that, so lane l ends with the total of value l >> (6 - log2 N) in
// N - 1 + (6 - log2 N) shuffles instead of 6 N.  Fixed order.
template <int N>
__device__ __forceinline__ double xpose_sum(double (&v)[N], int lane) {
  static_for<0, 6>([&](auto Lv) {
    constexpr int lev = decltype(Lv)::value;
    constexpr int o = 32 >> lev;
    constexpr int H = N >> (lev + 1);
    if constexpr (H >= 1) {
      const bool hi = (lane & o) != 0;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const double send = hi ? v[j] : v[j + H];
        const double keep = hi ? v[j + H] : v[j];
        v[j] = keep + __shfl_xor(send, o);
      }
    } else {
      v[0] = v[0] + __shfl_xor(v[0], o);
    }
  });
  return v[0];
}

// grid: clusters x nrb row blocks; slabs[(cluster * nrb + block) * ny + c] (zeros past D)
__global__ __launch_bounds__(256) void cl_solve_t(const ClSolveDesc* __restrict__ ds, int nrb,
                                                  int ny, double* __restrict__ slabs) {
  __shared__ double part[4][64];
  const int c = blockIdx.x / nrb, rb = blockIdx.x - c * nrb;
  const ClSolveDesc d = ds[c];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int D = d.D, r0 = 64 * rb, i = r0 + lane, ic = min(i, D - 1);
  double* out = slabs + (size_t)blockIdx.x * ny;
  if (r0 >= D) {  // (clusters of different sizes)
    for (int e = tid; e < ny; e += 256) out[e] = 0.0;
    return;
  }
  // (1) t_i = sum_{k <= i} L_ik rhs_k, wave w over k in [64 w, 64 w + 64)
  const int k0 = 64 * w, k1 = min(k0 + 64, min(r0 + 64, D));
  double acc = 0.0;
  for (int kb = k0; kb < k1; kb += 16) {
    double lv[16], rv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = min(kb + u, k1 - 1);
      lv[u] = d.L[ic + (size_t)k * D];
      rv[u] = d.rhs[k];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (kb + u < k1 && kb + u <= i) acc = fma(lv[u], rv[u], acc);
  }
  part[w][lane] = acc;
  __syncthreads();
  double t = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
  if (i >= D) t = 0.0;
  else if (w == 0) d.t[i] = t;
  // (2) sum over this block's rows of W_ic t_i: wave w takes 32 of every 128 columns
  for (int cb = 32 * w; cb < ny; cb += 128) {
    double v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const double wv = d.W[ic + (size_t)min(cb + j, ny - 1) * D];
      v[j] = i < D ? wv * t : 0.0;
    }
    const double sm = xpose_sum<32>(v, lane);
    const int cc = cb + (lane >> 1);
    if ((lane & 1) == 0 && cc < ny) out[cc] = sm;
  }
}

// grid: clusters x nrb column blocks (64 columns of dx each, 16 per wave)
__global__ __launch_bounds__(256) void cl_solve_dx(const ClSolveDesc* __restrict__ ds, int nrb,
                                                   int ny, const double* __restrict__ dy) {
  __shared__ double part[4][64];
  const int c = blockIdx.x / nrb, cbk = blockIdx.x - c * nrb;
  const ClSolveDesc d = ds[c];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int D = d.D, j0 = 64 * cbk + 16 * w;
  if (64 * cbk >= D) return;
  const int cw0 = (int)((long long)ny * w / 4), cw1 = (int)((long long)ny * (w + 1) / 4);
  double accx = 0.0;
  for (int rb = cbk; 64 * rb < D; ++rb) {  // the rows i >= 64 cbk, in order
    const int i = 64 * rb + lane, ic = min(i, D - 1);
    // u_i = t_i + W_i dy (this wave's share of the columns; the four shares in order)
    double sm = 0.0;
    for (int cb = cw0; cb < cw1; cb += 16) {
      double wv[16], yv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int cc = min(cb + u, cw1 - 1);
        wv[u] = d.W[ic + (size_t)cc * D];
        yv[u] = dy[cc];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (cb + u < cw1) sm = fma(wv[u], yv[u], sm);
    }
    part[w][lane] = sm;
    __syncthreads();
    const double ui =
        i < D ? d.t[ic] + ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane])) : 0.0;
    __syncthreads();  // (part is rewritten for the next row block)
    // dx_j += sum over this block's rows i >= j of L_ij u_i, the wave's 16 columns
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j = j0 + q;
      const double l = d.L[ic + (size_t)min(j, D - 1) * D];
      v[q] = (i < D && j < D && i >= j) ? l * ui : 0.0;
    }
    accx += xpose_sum<16>(v, lane);  // lane l: column j0 + (l >> 2)
  }
  const int j = j0 + (lane >> 2);
  if ((lane & 3) == 0 && j < D) d.dx[j] = accx;
}


}  // namespace clrsdp
