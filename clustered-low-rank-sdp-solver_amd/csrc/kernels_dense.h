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
template <class T>
__global__ __launch_bounds__(512) void eigmin_lds(const MatDesc<T>* __restrict__ descs,
                                                  T* __restrict__ out) {
  constexpr int NT = 512, NW = 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const MatDesc<T> d = descs[blockIdx.x];
  const int n = d.n, tid = threadIdx.x;
  T* A = reinterpret_cast<T*>(smem_raw);  // n x n
  T* v = A + (size_t)n * n;               // n
  T* p = v + n;                            // 4 * n partials, then p
  T* dg = p + 4 * n;                       // n
  T* e2 = dg + n;                          // n
  T* red = e2 + n;                         // NW + 4
  for (int e = tid; e < n * n; e += NT) {
    const int i = e % n, j = e / n;
    A[e] = (d.A[i + (size_t)j * d.lda] + d.A[j + (size_t)i * d.lda]) * T(0.5);
  }
  __syncthreads();
  for (int k = 0; k + 2 < n; ++k) {
    const int m = n - k - 1;
    T* Ak = A + (k + 1) + (size_t)(k + 1) * n;  // trailing m x m, ld n
    T s = T(0.0);
    for (int i = tid; i < m; i += NT) {
      const T xi = A[(k + 1 + i) + (size_t)k * n];
      v[i] = xi;
      s += xi * xi;
    }
    s = block_sum_w<T, NW>(s, red);
    const T x0 = v[0];
    if (tid == 0) dg[k] = A[k + (size_t)k * n];
    const T tail = s - x0 * x0;
    if (!(tail > T(0.0))) {
      if (tid == 0) e2[k] = x0 * x0;
      __syncthreads();
      continue;
    }
    const T nrm = Num<T>::sqrt_(s);
    const T alpha = (x0 > T(0.0)) ? -nrm : nrm;
    const T v0 = x0 - alpha;
    const T beta = T(2.0) / (tail + v0 * v0);
    if (tid == 0) {
      e2[k] = alpha * alpha;
      v[0] = v0;
    }
    __syncthreads();
    // p = beta A' v : thread (i, q) sums columns j = q, q+4, ... (4 partials per row)
    {
      const int i = tid & 127, q = tid >> 7;
      for (int ii = i; ii < m; ii += 128) {
        T acc = T(0.0);
        for (int j = q; j < m; j += 4) acc += Ak[ii + (size_t)j * n] * v[j];
        p[q * n + ii] = acc;
      }
    }
    __syncthreads();
    T pv = T(0.0);
    for (int i = tid; i < m; i += NT) {
      const T pi = (p[i] + p[n + i] + p[2 * n + i] + p[3 * n + i]) * beta;
      p[i] = pi;
      pv += pi * v[i];
    }
    pv = block_sum_w<T, NW>(pv, red);
    const T Kc = beta * pv * T(0.5);
    for (int i = tid; i < m; i += NT) p[i] = p[i] - Kc * v[i];
    __syncthreads();
    for (int e = tid; e < m * m; e += NT) {
      const int i = e % m, j = e / m;
      Ak[i + (size_t)j * n] = Ak[i + (size_t)j * n] - (v[i] * p[j] + p[i] * v[j]);
    }
    __syncthreads();
  }
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
  if (tid < 64) {
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

}  // namespace clrsdp
