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
__device__ T wave_sum(T v) {
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
__device__ T block_sum_w(T v, T* red) {
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
// Right-looking: step j broadcasts column j of L and row j of L^-1 through LDS (2 barriers).
// In-place safe (out == A): every thread reads its own tile before anything is written.
// ------------------------------------------------------------------------------------------
template <class T, int TR, int TC, int GR, int GC>
__global__ __launch_bounds__(GR * GC) void chol_inv_reg(const MatDesc<T>* __restrict__ in,
                                                        const MatDesc<T>* __restrict__ out_inv,
                                                        const MatDesc<T>* __restrict__ out_l,
                                                        int* __restrict__ info) {
  constexpr int NMAX = TR * GR;
  static_assert(TR * GR == TC * GC, "square tile grid");
  __shared__ T col[NMAX];
  __shared__ T row[NMAX];
  __shared__ T sd;
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
      a[i][c] = (gi < n && gc < n && gc <= gi) ? d.A[gi + (size_t)gc * d.lda] : T(0.0);
      x[i][c] = (gi == gc) ? T(1.0) : T(0.0);
    }
  if (t == 0) {
    fail = 0;
    const T d0 = d.A[0];
    if (!(d0 > T(0.0))) fail = 1;
    sd = Num<T>::sqrt_(d0);
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    if (fail) break;
    const T s = sd;
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
              const T l = (gi == j) ? s : a[i][c] / s;
              a[i][c] = l;
              col[gi] = l;
            }
          }
        }
      }
    }
    if (tr == j / TR) {
#pragma unroll
      for (int i = 0; i < TR; ++i) {
        if (i == jr) {
#pragma unroll
          for (int c = 0; c < TC; ++c) {
            x[i][c] = x[i][c] / s;
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
      for (int i = 0; i < TR; ++i) ci[i] = (r0 + i > j && r0 + i < n) ? col[r0 + i] : T(0.0);
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
      if (c0 <= j) {
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
      sd = Num<T>::sqrt_(dn);
    }
    __syncthreads();
  }
  if (t == 0 && info) info[blockIdx.x] = fail;
  const MatDesc<T> o = out_inv[blockIdx.x];
#pragma unroll
  for (int i = 0; i < TR; ++i)
#pragma unroll
    for (int c = 0; c < TC; ++c) {
      const int gi = r0 + i, gc = c0 + c;
      if (gi < n && gc < n) o.A[gi + (size_t)gc * o.lda] = x[i][c];
    }
  if (out_l) {
    const MatDesc<T> ol = out_l[blockIdx.x];
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int c = 0; c < TC; ++c) {
        const int gi = r0 + i, gc = c0 + c;
        if (gi < n && gc < n) ol.A[gi + (size_t)gc * ol.lda] = (gc <= gi) ? a[i][c] : T(0.0);
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
// (replaces approx_eig_qr! in compute_step_length, MPMP.jl:1857-1860).  512 threads; wave w
// owns rows 16w..16w+15 (lane r = l & 15), lane class c = l >> 4 owns the column pairs
// j = 2c + 8s + {0,1}, s = 0..15: 32 entries per thread.  Householder tridiagonalisation with
// two barriers per column:
//   (B) every wave rebuilds the reflector of column k redundantly from the column buffer
//       (wave reduction, no barrier), p_i = sum_j A_ij v_j in registers (+ 2 shuffles across
//       the column classes), per-wave v^T p to LDS                                 -- barrier
//   (C) w = beta p - K v; A -= v w^T + w v^T in registers; the owners of column k+1 publish it
//       to the other column buffer                                                -- barrier
// then 512-way multisection with Sturm counts on the tridiagonal matrix.  No LDS image of A:
// the only LDS traffic per column is the broadcast of v and p (two ds_read_b128 per pair).
// ------------------------------------------------------------------------------------------
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

__global__ __launch_bounds__(512) void eigmin_reg(const MatDesc<double>* __restrict__ descs,
                                                  double* __restrict__ out) {
  constexpr int NS = 16;
#ifdef CLRSDP_EIGREG_STAMPS
  unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#define ER_STAMP(slot) if (threadIdx.x == 0) { unsigned long long t_ = __builtin_amdgcn_s_memtime(); atomicAdd(&g_eigreg_stamps[slot], t_ - t_prev); t_prev = t_; }
#else
#define ER_STAMP(slot)
#endif
  // colb[k&1] = column k of the current matrix with rows <= k-1 zeroed; pb = A'v with inactive
  // rows zeroed; rows/columns >= n stay zero.  So v and w need no masking per element.
  // entries 128..255 stay zero: the slots past the last column read zeros there
  __shared__ __attribute__((aligned(16))) double colb[2][256];
  __shared__ __attribute__((aligned(16))) double pb[256];
  __shared__ double redw[8];
  __shared__ double dg[128], e2[128];
  __shared__ __attribute__((aligned(16))) double sd[128], se[128];
  __shared__ double bnd[2];
  __shared__ unsigned long long masks[8];
  const MatDesc<double> d = descs[blockIdx.x];
  const int n = d.n, lda = d.lda, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int c = lane >> 4, i = w * 16 + (lane & 15);
  const bool rowok = i < n;
  // slot s holds columns j = 2c + 8(s + q) + {0,1}; q advances (the slots shift down by one)
  // each time column k+1 enters a new group of 8, so column k+1 always sits in slot 0.
  double a[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 2 * c + 8 * s + e;
      const int ic = min(i, n - 1), jc = min(j, n - 1);  // unconditional loads, masked after
      const double v = (gload(d.A + ic + (size_t)jc * lda) + gload(d.A + jc + (size_t)ic * lda)) * 0.5;
      a[s][e] = (rowok && j < n) ? v : 0.0;
    }
  // scale the block by 2^-ex0 so that its largest entry lies in [0.5, 1): the column norms of the
  // Householder reduction neither overflow nor underflow for any block norm in fp64 range (exact,
  // undone on the result)
  int ex0 = 0;
  {
    double amax = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) amax = fmax(amax, fmax(fabs(a[s][0]), fabs(a[s][1])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
    if (lane == 0) redw[w] = amax;
    __syncthreads();
    amax = redw[0];
#pragma unroll
    for (int r = 1; r < 8; ++r) amax = fmax(amax, redw[r]);
    ex0 = (amax > 0.0 && amax < INFINITY) ? __builtin_amdgcn_frexp_exp(amax) : 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      a[s][0] = __builtin_ldexp(a[s][0], -ex0);
      a[s][1] = __builtin_ldexp(a[s][1], -ex0);
    }
  }
#define EIG_SHIFT_SLOTS()                                                 \
  do {                                                                       \
    _Pragma("unroll") for (int s = 0; s + 1 < NS; ++s) {                     \
      a[s][0] = a[s + 1][0];                                                 \
      a[s][1] = a[s + 1][1];                                                 \
    }                                                                        \
    a[NS - 1][0] = a[NS - 1][1] = 0.0;                                       \
  } while (0)
  if (tid < 256) {
    pb[tid] = 0.0;
    colb[1][tid] = 0.0;
    if (tid >= n) colb[0][tid] = 0.0;
  }
  if (c == 0 && rowok) colb[0][i] = a[0][0];  // column 0
  __syncthreads();
  ER_STAMP(0)
  int q = 0;
  for (int k = 0; k + 2 < n; ++k) {
    if (((k + 1) & 7) == 0) { EIG_SHIFT_SLOTS(); ++q; }
    const double* col = colb[k & 1];
    const int ns = NS - q;  // slots that hold existing columns
    // ---- LDS reads: the column tail for the norm first (rows > k+128 read the zero padding),
    // then the slot values, so the norm's wait does not cover the slot reads
    const double xa = col[k + 1 + lane], xb = col[k + 65 + lane];
    double2 cv[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s)
      cv[s] = *reinterpret_cast<const double2*>(col + 2 * c + 8 * (s + q));
    const double xi = col[i < 128 ? i : 0];
    // ---- reflector of column k (every wave, redundantly)
    double ss = fma(xa, xa, xb * xb);
    ss = wave_sum_dpp(ss);
    const double x0 = col[k + 1];
    const double tail = ss - x0 * x0;
    double beta = 0.0, v0 = x0;
    if (tail > 0.0) {
      const double nrm = sqrt(ss);
      const double alpha = x0 > 0.0 ? -nrm : nrm;
      v0 = x0 - alpha;
      beta = 2.0 / (tail + v0 * v0);
      if (tid == 0) e2[k] = alpha * alpha;
    } else if (tid == 0) {
      e2[k] = x0 * x0;
    }
    if (tid == 0) dg[k] = col[k];
    ER_STAMP(6)
    if (beta != 0.0) {
      // ---- (B) p = A' v.  v_j = col[j] for j > k+1, v0 at k+1 (slot 0, element (k+1)&1 of
      // class ((k+1)>>1)&3), 0 for j <= k (zeroed rows of the column buffer)
      const int jn = k + 1;
      const bool own = c == ((jn >> 1) & 3);
      if (own) {
        if (jn & 1) cv[0].y = v0; else cv[0].x = v0;
      }
      // the pivot entry j = k holds the diagonal in the column buffer: v_k = 0.  Column k is in
      // slot 0 unless the slots were just shifted past it.
      if (((k + 1) & 7) != 0 && c == ((k >> 1) & 3)) {
        if (k & 1) cv[0].y = 0.0; else cv[0].x = 0.0;
      }
      const double vi = i > k ? (i == jn ? v0 : xi) : 0.0;
      const bool wave_live = w * 16 + 15 > k;  // wave-uniform: some row of this wave is active
      double pp = 0.0, pq = 0.0;  // two FMA chains
      // slots in groups of 4 behind one uniform branch each (a per-slot condition gets
      // if-converted into computing everything plus selects)
      if (wave_live) {
#pragma unroll
        for (int g = 0; g < NS / 4; ++g) {
          if (4 * g < ns) {
#pragma unroll
            for (int s = 4 * g; s < 4 * g + 4; ++s) {
              pp = fma(a[s][0], cv[s].x, pp);
              pq = fma(a[s][1], cv[s].y, pq);
            }
          }
        }
      }
      pp += pq;
      ER_STAMP(7)
      pp = xsum32(xsum16(pp));
      double t = 0.0;
      if (c == 0) {
        if (i < 128) pb[i] = i > k ? pp : 0.0;
        t = vi * pp;
      }
      t = wave_sum_dpp(t);
      if (lane == 0) redw[w] = t;
      ER_STAMP(1)
      __syncthreads();
      ER_STAMP(2)
      // ---- (C) w = beta p - K v;  A' -= v w^T + w v^T
      double tot = redw[0];
#pragma unroll
      for (int r = 1; r < 8; ++r) tot += redw[r];
      const double Kc = beta * beta * tot * 0.5;
      double2 pv[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s)
        pv[s] = *reinterpret_cast<const double2*>(pb + 2 * c + 8 * (s + q));
      // a_ij -= v_i w_j + w_i v_j with w = beta p - K v:  a_ij += g_i v_j - h_i p_j,
      // g_i = K v_i - w_i, h_i = beta v_i
      const double wi = beta * pp - Kc * vi;
      const double gi = Kc * vi - wi, hi = beta * vi;
      if (wave_live) {
#pragma unroll
        for (int g = 0; g < NS / 4; ++g) {
          if (4 * g < ns) {
#pragma unroll
            for (int s = 4 * g; s < 4 * g + 4; ++s) {
              a[s][0] = fma(gi, cv[s].x, fma(-hi, pv[s].x, a[s][0]));
              a[s][1] = fma(gi, cv[s].y, fma(-hi, pv[s].y, a[s][1]));
            }
          }
        }
      }
    }
    // ---- publish column k+1 from slot 0 of its owners; rows <= k+1-1 written as 0
    {
      const int jn = k + 1;
      if (c == ((jn >> 1) & 3) && i < 128) colb[jn & 1][i] = (i >= jn && rowok) ? ((jn & 1) ? a[0][1] : a[0][0]) : 0.0;
    }
    ER_STAMP(3)
    __syncthreads();
    ER_STAMP(4)
  }
  // trailing 2x2 (or 1x1): column n-1 from slot 0 of its owners (after the last shift)
  if (n >= 2) {
    const int j1 = n - 1;
    if (n >= 3 && ((n - 2 + 1) & 7) == 0) EIG_SHIFT_SLOTS();
    if (c == ((j1 >> 1) & 3) && rowok && i >= n - 2) pb[i] = (j1 & 1) ? a[0][1] : a[0][0];
  }
#undef EIG_SHIFT_SLOTS
  __syncthreads();
  if (tid == 0) {
    if (n >= 2) {
      const double* col = colb[(n - 2) & 1];  // column n-2 (published at k = n-3, or initial)
      dg[n - 2] = col[n - 2];
      dg[n - 1] = pb[n - 1];
      const double e = col[n - 1];
      e2[n - 2] = e * e;
    } else {
      dg[0] = colb[0][0];
    }
  }
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
  // ---- 512-way multisection: 6 rounds of 9 bits bracket lambda_min to 2^-54 of the Gershgorin
  // span, below the Sturm count's own backward error (~n eps ||T||), so a 7th round adds noise
  double lo = bnd[0], hi = bnd[1];
  const int nr = (n + 7) & ~7;
  for (int it = 0; it < 6; ++it) {
    const double width = hi - lo;
    const double sigma = lo + width * ((double)(tid + 1) / 513.0);
    const unsigned long long mk = __ballot(sturm_any_below(sd, se, nr, sigma));
    if (lane == 0) masks[w] = mk;
    __syncthreads();
    int f = -1;
    for (int q = 0; q < 8 && f < 0; ++q)
      if (masks[q]) f = q * 64 + __ffsll((long long)masks[q]) - 1;
    __syncthreads();
    if (f < 0) {
      lo = lo + width * (512.0 / 513.0);
    } else {
      hi = lo + width * ((double)(f + 1) / 513.0);
      if (f > 0) lo = lo + width * ((double)f / 513.0);
    }
  }
  ER_STAMP(5)
  if (tid == 0) out[blockIdx.x] = __builtin_ldexp((lo + hi) * 0.5, bnd_ex + ex0);
#undef ER_STAMP
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
  T* A = reinterpret_cast<T*>(smem_raw);  // n x n
  T* v = A + (size_t)n * n;               // n
  T* p = v + n;                            // 4 * n partials, then p
  T* dg = p + 4 * n;                       // n
  T* e2 = dg + n;                          // n
  T* red = e2 + 3 * n + 12;                // NW + 4 (after w, scalars and partials)
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
      s = wave_sum(s);
      const T x0 = A[(k + 1) + (size_t)k * n];
      const T tail = s - x0 * x0;
      if (tid == 0) {
        dg[k] = A[k + (size_t)k * n];
        if (!(tail > T(0.0))) {
          e2[k] = x0 * x0;
          scal[0] = T(0.0);  // beta = 0: no reflection
        } else {
          const T nrm = Num<T>::sqrt_(s);
          const T alpha = (x0 > T(0.0)) ? -nrm : nrm;
          const T v0 = x0 - alpha;
          e2[k] = alpha * alpha;
          v[0] = v0;
          scal[0] = T(2.0) / (tail + v0 * v0);
        }
      }
    }
    __syncthreads();
    EIG_STAMP(0)
    const T beta = scal[0];
    if (beta == T(0.0)) continue;  // uniform: nothing to update
    // ---- (B) partial rows of A'v (4 column classes) and v^T A' v
    const int ri = tid & 127, cq = tid >> 7;
    T vav = T(0.0);
    for (int ii = ri; ii < m; ii += 128) {
      T a0 = T(0.0), a1 = T(0.0), a2 = T(0.0), a3 = T(0.0);
      int j = cq;
      for (; j + 12 < m; j += 16) {
        a0 += Ak[ii + (size_t)j * n] * v[j];
        a1 += Ak[ii + (size_t)(j + 4) * n] * v[j + 4];
        a2 += Ak[ii + (size_t)(j + 8) * n] * v[j + 8];
        a3 += Ak[ii + (size_t)(j + 12) * n] * v[j + 12];
      }
      for (; j < m; j += 4) a0 += Ak[ii + (size_t)j * n] * v[j];
      const T part = (a0 + a1) + (a2 + a3);
      p[cq * n + ii] = part;
      vav += part * v[ii];
    }
    EIG_STAMP(1)
    vav = wave_sum(vav);
    if ((tid & 63) == 0) redw[tid >> 6] = vav;
    __syncthreads();
    EIG_STAMP(2)
    // ---- (C) w = beta A'v - K v,  K = beta^2 v^T A' v / 2
    {
      T tot = redw[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) tot += redw[q];
      const T Kc = beta * beta * tot * T(0.5);
      for (int i = tid; i < m; i += NT)
        Wv[i] = ((p[i] + p[n + i]) + (p[2 * n + i] + p[3 * n + i])) * beta - Kc * v[i];
    }
    __syncthreads();
    EIG_STAMP(3)
    // ---- (D) A' -= v w^T + w v^T
    for (int ii = ri; ii < m; ii += 128) {
      const T vi = v[ii], wi = Wv[ii];
      int j = cq;
      for (; j + 12 < m; j += 16) {
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
          T* a = Ak + ii + (size_t)(j + u) * n;
          *a = *a - (vi * Wv[j + u] + wi * v[j + u]);
        }
      }
      for (; j < m; j += 4) {
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
  (void)red;
  if (n == 1) {
    if (tid == 0) out[blockIdx.x] = dg[0];
    return;
  }
  // ---- multisection with all 512 threads (9 bits per round), in two phases:
  //  (1) fp64 on the leading limbs of the tridiagonal: Gershgorin bracket, 7 rounds;
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
    double lo = bnd[0], hi = bnd[1];
    for (int it = 0; it < 7; ++it) {
      const double width = hi - lo;
      const double sigma = lo + width * ((double)(tid + 1) / 513.0);
      const int f = first_hit(sturm_count_fast(dgh, e2h, n, sigma) >= 1);
      if (f < 0) {
        lo = lo + width * (512.0 / 513.0);
      } else {
        hi = lo + width * ((double)(f + 1) / 513.0);
        if (f > 0) lo = lo + width * ((double)f / 513.0);
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
  if constexpr (NEWTON && Num<T>::BITS > 120) {
    // (2') quad-double: Newton on det(T - sigma I) from the fp64 centre (at dd the 11 parallel
    // multisection rounds are as fast as the sequential Newton chain, so dd keeps them).  With the pivots of
    // T - sigma I = L D L^T, q_i = (d_i - sigma) - e2_{i-1} / q_{i-1}, and s_i = dq_i/dsigma =
    // -1 + e2_{i-1} s_{i-1} / q_{i-1}^2, the Newton step is 1 / sum_i s_i / q_i.  It converges
    // quadratically from the fp64 estimate (3 steps for a simple eigenvalue, a 4th confirms).
    // The result is accepted only if it converged AND two multi-word Sturm counts bracket it
    // (no eigenvalue below sigma - delta, one at most sigma + delta, delta = 2^(12-BITS)
    // magnitudes); otherwise the multisection below runs as before.
    T* nres = Wv;  // free after the reduction: [0] = sigma
    const double mag = fmax(fabs(bnd[0]), fabs(bnd[1]));
    if (tid == 0) {
      T s = T(0.5 * (bnd[2] + bnd[3]));
      const double tol = ldexp(mag, -(Num<T>::BITS + 2)) + 1e-300;
      int conv = 0;
      for (int it = 0; it < 4; ++it) {
        T q = dg[0] - s;
        if (q == T(0.0)) q = T(1e-300);
        T r = T(1.0) / q, sd = T(-1.0), g = -r;
        for (int i = 1; i < n; ++i) {
          const T t = e2[i - 1] * r;
          sd = (t * r) * sd - T(1.0);
          q = (dg[i] - s) - t;
          if (q == T(0.0)) q = T(1e-300);
          r = T(1.0) / q;
          g = g + sd * r;
        }
        const T step = T(1.0) / g;
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
    if (tid == 0) c = masks[2] && sturm_count(dg, e2, n, s - dl) == 0;
    if (tid == 64) c = sturm_count(dg, e2, n, s + dl) >= 1;
    __syncthreads();
    if (tid == 0 || tid == 64) masks[tid >> 6] = (unsigned long long)c;
    __syncthreads();
    const bool ok = masks[0] && masks[1];
    __syncthreads();
    if (ok) {
      if (tid == 0) out[blockIdx.x] = s;
      EIG_STAMP(6)
      return;
    }
  }
  T lo = T(bnd[2]), hi = T(bnd[3]);
  // check the start bracket at full width: count(lo) == 0 and count(hi) >= 1
  {
    int c = 0;
    if (tid == 0) c = sturm_count(dg, e2, n, lo) == 0;
    if (tid == 64) c = sturm_count(dg, e2, n, hi) >= 1;
    if (tid == 0 || tid == 64) masks[tid >> 6] = (unsigned long long)c;
    __syncthreads();
    const bool ok = masks[0] && masks[1];
    __syncthreads();
    if (!ok) {
      lo = T(bnd[0]);
      hi = T(bnd[1]);
    }
    // rounds to shrink the bracket to ~2^-BITS of the spectrum's magnitude
    const int rounds = ok ? (Num<T>::BITS - 25) / 9 + 2 : Num<T>::BITS / 9 + 3;
    for (int it = 0; it < rounds; ++it) {
      const T width = hi - lo;
      const T sigma = lo + width * T((double)(tid + 1) / 513.0);
      const int f = first_hit(sturm_count(dg, e2, n, sigma) >= 1);
      if (f < 0) {
        lo = lo + width * T(512.0 / 513.0);
      } else {
        hi = lo + width * T((double)(f + 1) / 513.0);
        if (f > 0) lo = lo + width * T((double)f / 513.0);
      }
    }
  }
  if (tid == 0) out[blockIdx.x] = (lo + hi) * T(0.5);
  EIG_STAMP(6)
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
__device__ unsigned long long g_chol2_trace[256 * 8 * 64];
#define CT_TRACE() do { if ((threadIdx.x & 63) == 0 && tr_i < 64) g_chol2_trace[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + tr_i] = __builtin_amdgcn_s_memtime(); ++tr_i; } while (0)
#else
#define CT_TRACE()
#endif
template <int NP>
struct CholTiles {
  static constexpr int NT = NP / 16, NOFF = NT * (NT - 1) / 2, NWK = 7;
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
__global__ __launch_bounds__(512) void chol_inv_tiles(const MatDesc<double>* __restrict__ in,
                                                      const MatDesc<double>* __restrict__ out_inv,
                                                      int* __restrict__ info) {
  using CT = CholTiles<NP>;
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
  const int n = d.n, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nt = (n + 15) / 16;
  const int lr = lane & 15, lk = lane >> 4;
  const int wk = w - 1;  // worker index, -1 for wave 0
  // ---- tile coordinates of this worker's slots (wave-uniform)
  int TI[SLOTS], TJ[SLOTS];
#pragma unroll
  for (int q = 0; q < SLOTS; ++q) {
    const int t = wk + NWK * q;
    TI[q] = NT; TJ[q] = 0;  // empty slot: row NT is never active
    if (wk >= 0 && t < CT::NOFF) CT::tile(t, TI[q], TJ[q]);
  }
  // ---- off-diagonal tiles straight into the accumulators (A_ij^T layout, coalesced along
  // rows), diagonal tiles into LDS with identity padding
  d4 T[SLOTS];
#pragma unroll
  for (int q = 0; q < SLOTS; ++q) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = 16 * TI[q] + lr, gj = 16 * TJ[q] + lk + 4 * r;
      T[q][r] = (TI[q] < nt && gi < n && gj < n) ? gload(d.A + gi + (size_t)gj * d.lda) : 0.0;
    }
  }
  for (int e = tid; e < NT * 256; e += 512) {
    const int t = e >> 8, c = (e >> 4) & 15, r = e & 15;
    const int gi = 16 * t + r, gj = 16 * t + c;
    double v = gi == gj ? 1.0 : 0.0;
    if (t < nt && gi < n && gj < n && r >= c) v = gload(d.A + gi + (size_t)gj * d.lda);
    Dt[t * 16 * LDD + c * LDD + r] = v;
  }
  d4 XD[DSLOTS];
#pragma unroll
  for (int q = 0; q < DSLOTS; ++q) XD[q] = d4{0.0, 0.0, 0.0, 0.0};
  if (tid == 0) {
    flag[0] = 0;  // first failing pivot + 1
    flag[1] = 0;  // panels whose L_{k+1,k} is in the panel buffer
    flag[2] = 0;  // worker arrivals at the (b) -> (c) barrier
  }
  __syncthreads();
  CT_TRACE();
  if (w == 0)
    chol_diag16_bc(Dt, [](int i, int j) { return j * LDD + i; }, 0, Di, flag, lane);
  __syncthreads();
  CT_TRACE();
  for (int k = 0; k < nt; ++k) {
    if (*flag) break;
    const double* Dk = Di + 256 * (k & 1);
    if (wk >= 0) {
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
          double* P = Pn + 256 * TI[q];
#pragma unroll
          for (int r = 0; r < 4; ++r) P[(lk + 4 * r) * 16 + lr] = acc[r];  // L_ik[lr][lk+4r]
          if (pass == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(flag + 1, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
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
        for (int r = 0; r < 4; ++r) Xr[(lk + 4 * r) * XLD + 16 * TJ[q] + lr] = acc[r];
      }
      if (wk == k % NWK) {  // X_kk = Linv_kk (accumulator layout: register r = Linv[lk+4r][lr])
#pragma unroll
        for (int q = 0; q < DSLOTS; ++q)
          if (q == k / NWK) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              XD[q][r] = Dk[lr * 16 + lk + 4 * r];
              Xr[(lk + 4 * r) * XLD + 16 * k + lr] = XD[q][r];
            }
          }
      }
      CT_TRACE();
      // workers-only barrier (wave 0 is busy with the next diagonal tile)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(flag + 2, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      while (__hip_atomic_load(flag + 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < NWK * (k + 1))
        __builtin_amdgcn_s_sleep(1);
      CT_TRACE();
      // ---------------- (c) trailing update of the rows below k
      const double* Pk = Pn;
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
            acc = mfma64(-Pi[(4 * r + lk) * 16 + lr], Xr[(4 * r + lk) * XLD + 16 * tj + lr], acc);
          T[q] = acc;
        }
      }
      // diagonal tiles below the look-ahead one: D_i -= L_ik L_ik^T (in LDS)
#pragma unroll
      for (int q = 0; q < DSLOTS; ++q) {
        const int di = wk + NWK * q;
        if (di >= nt || di <= k + 1) continue;
        const double* Pi = Pk + 256 * di;
        double* D = Dt + di * 16 * LDD;
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
    } else if (k + 1 < nt) {
      // ---------------- wave 0: D_{k+1} -= L L^T (L = L_{k+1,k}) and its factorisation
      while (__hip_atomic_load(flag + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= k)
        __builtin_amdgcn_s_sleep(1);
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
      chol_diag16_bc(D, [](int i, int j) { return j * LDD + i; }, 16 * (k + 1),
                     Di + 256 * ((k + 1) & 1), flag, lane);
      CT_TRACE();
    }
    __syncthreads();
    CT_TRACE();
  }
  if (tid == 0 && info) info[blockIdx.x] = *flag;
  // ---- write L^-1: off-diagonal and diagonal X tiles from the registers, zeros above
  const MatDesc<double> o = out_inv[blockIdx.x];
  if (wk >= 0) {
#pragma unroll
    for (int q = 0; q < SLOTS; ++q) {
      if (TI[q] >= nt) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 16 * TI[q] + lk + 4 * r, gj = 16 * TJ[q] + lr;
        if (gi < n && gj < n) o.A[gi + (size_t)gj * o.lda] = T[q][r];
      }
    }
#pragma unroll
    for (int q = 0; q < DSLOTS; ++q) {
      const int di = wk + NWK * q;
      if (di >= nt) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 16 * di + lk + 4 * r, gj = 16 * di + lr;
        if (gi < n && gj < n) o.A[gi + (size_t)gj * o.lda] = XD[q][r];
      }
    }
  }
  for (int j = tid >> 4; j < n; j += 32)
    for (int i = (tid & 15); i < (j & ~15); i += 16) o.A[i + (size_t)j * o.lda] = 0.0;  // tiles above
  CT_TRACE();
}
#undef CT_TRACE


}  // namespace clrsdp


