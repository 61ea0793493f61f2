// Host check of eigmin_mx's fp64 intermediates (DBG = 2 dump of block 0): the reflectors
// reproduce T (Q^T A_h Q), z is an eigenvector of T, x = Q z, the residual r, s = P Q^T (-r),
// the solve (T - lam I) d' = s, and d = Q P d'.  Norms printed per check.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 eig_mx_dump.hip -o microbin/eig_mx_dump
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <random>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
using mw::dd;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)
typedef long double LD;

static void run(int n) {
  std::mt19937_64 g(11 + n);
  std::uniform_real_distribution<double> ud(-0.5, 0.5);
  std::vector<dd> A((size_t)n * n);
  std::vector<double> Ah((size_t)n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i <= j; ++i) {
      const double v = ud(g) + (i == j ? 0.1 * (j % 7) : 0.0);
      A[i + (size_t)j * n] = A[j + (size_t)i * n] = dd(v);
      Ah[i + (size_t)j * n] = Ah[j + (size_t)i * n] = v;
    }
  dd *dA, *dE;
  int* redo;
  CK(hipMalloc(&redo, sizeof(int)));
  CK(hipMalloc(&dA, A.size() * sizeof(dd)));
  CK(hipMalloc(&dE, sizeof(dd)));
  CK(hipMemcpy(dA, A.data(), A.size() * sizeof(dd), hipMemcpyHostToDevice));
  MatDesc<dd> h{dA, n, n}, *dd_;
  CK(hipMalloc(&dd_, sizeof(h)));
  CK(hipMemcpy(dd_, &h, sizeof(h), hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)eigmin_mx<dd, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - EIGMX_STATIC_LDS));
  eigmin_mx<dd, 2><<<1, 576, eigmx_lds_bytes<dd>(n)>>>(dd_, dE, redo);
  CK(hipDeviceSynchronize());
  std::vector<double> dm(64 * 64 + 12 * 64);
  CK(hipMemcpyFromSymbol(dm.data(), HIP_SYMBOL(g_eigmx_dump), dm.size() * sizeof(double)));
  const double* V = dm.data();
  const double* X = dm.data() + (size_t)n * n;
  const double *dg = X, *eo = X + n, *bet = X + 2 * n, *z = X + 3 * n, *x = X + 4 * n, *rh = X + 5 * n,
               *s = X + 6 * n, *dp = X + 7 * n, *d = X + 8 * n;
  const double lam = X[10 * n];  // (the LDL shift mu)
  const int ex = (int)X[10 * n + 1];
  // Q explicitly: Q = H_0 ... H_{n-2}, applied to the identity from the right end
  std::vector<LD> Q((size_t)n * n, 0.0L);
  for (int i = 0; i < n; ++i) Q[i + (size_t)i * n] = 1.0L;
  for (int k = n - 2; k >= 0; --k)  // Q <- H_k Q
    for (int c = 0; c < n; ++c) {
      LD t = 0;
      for (int i = k + 1; i < n; ++i) t += (LD)V[i + (size_t)k * n] * Q[i + (size_t)c * n];
      for (int i = k + 1; i < n; ++i) Q[i + (size_t)c * n] -= (LD)bet[k] * t * V[i + (size_t)k * n];
    }
  // step by step: A_{k+1} = H_k A_k H_k with the stored reflectors; the first step whose column k
  // is not [.., dg_k, eo_k, 0 ..]
  {
    std::vector<LD> M((size_t)n * n);
    for (size_t q = 0; q < M.size(); ++q) M[q] = Ah[q];
    int shown = 0;
    for (int k = 0; k + 2 < n && shown < 3; ++k) {
      // M <- H_k M H_k
      std::vector<LD> v(n, 0.0L);
      for (int i = k + 1; i < n; ++i) v[i] = V[i + (size_t)k * n];
      for (int c = 0; c < n; ++c) {  // columns
        LD t = 0;
        for (int i = 0; i < n; ++i) t += v[i] * M[i + (size_t)c * n];
        for (int i = 0; i < n; ++i) M[i + (size_t)c * n] -= (LD)bet[k] * t * v[i];
      }
      for (int r = 0; r < n; ++r) {  // rows
        LD t = 0;
        for (int i = 0; i < n; ++i) t += v[i] * M[r + (size_t)i * n];
        for (int i = 0; i < n; ++i) M[r + (size_t)i * n] -= (LD)bet[k] * t * v[i];
      }
      double ez0 = 0.0;
      for (int i = k + 2; i < n; ++i) ez0 = fmax(ez0, fabs((double)M[i + (size_t)k * n]));
      const double dd0 = fabs((double)M[k + (size_t)k * n] - ldexp(dg[k], ex));
      const double de0 = fabs((double)fabsl(M[k + 1 + (size_t)k * n]) - fabs(ldexp(eo[k], ex)));
      if (fabs((double)M[k + 1 + (size_t)k * n] - ldexp(eo[k], ex)) > 1e-12 && shown < 3) {
        ++shown;
        printf("  step %d: signed subdiag %.17g against eo %.17g\n", k, (double)M[k + 1 + (size_t)k * n], ldexp(eo[k], ex));
      }
      if (ez0 > 1e-12 || dd0 > 1e-12 || de0 > 1e-12) {
        ++shown;
        printf("  step %d: below-subdiag %.2e, diag err %.2e, |subdiag| err %.2e (sub %.6g eo %.6g) bet %.6g v[k+1] %.6g\n",
               k, ez0, dd0, de0, (double)M[k + 1 + (size_t)k * n], ldexp(eo[k], ex), bet[k], V[k + 1 + (size_t)k * n]);
      }
    }
  }
  // T' = Q^T A_h Q against the tridiagonal (unscaled)
  double et = 0.0, at = 0.0;
  int ei = -1, ej = -1;
  double etv = 0.0, erf = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      LD t = 0;
      for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) t += Q[a + (size_t)i * n] * (LD)Ah[a + (size_t)b * n] * Q[b + (size_t)j * n];
      double ref = 0.0;
      if (i == j) ref = ldexp(dg[i], ex);
      else if (i == j + 1) ref = ldexp(eo[j], ex);
      else if (j == i + 1) ref = ldexp(eo[i], ex);
      if (fabs((double)t - ref) > et) { ei = i; ej = j; etv = (double)t; erf = ref; }
      et = fmax(et, fabs((double)t - ref));
      at = fmax(at, fabs((double)t));
    }
  printf("  max |Q^T A Q - T| at (%d, %d): %.17g against %.17g\n", ei, ej, etv, erf);
  // (T_s - lam) z
  double ez = 0.0;
  for (int i = 0; i < n; ++i) {
    LD t = ((LD)dg[i] - lam) * z[i];
    if (i > 0) t += (LD)eo[i - 1] * z[i - 1];
    if (i + 1 < n) t += (LD)eo[i] * z[i + 1];
    ez = fmax(ez, fabs((double)t));
  }
  // x - Q z
  double ex_ = 0.0;
  for (int i = 0; i < n; ++i) {
    LD t = 0;
    for (int k = 0; k < n; ++k) t += Q[i + (size_t)k * n] * z[k];
    ex_ = fmax(ex_, fabs((double)(t - x[i])));
  }
  // r = A x - rho x (long double), scaled, against rh
  LD num = 0, den = 0;
  std::vector<LD> y(n);
  for (int i = 0; i < n; ++i) {
    y[i] = 0;
    for (int j = 0; j < n; ++j) y[i] += (LD)Ah[i + (size_t)j * n] * x[j];
  }
  for (int i = 0; i < n; ++i) { num += x[i] * y[i]; den += (LD)x[i] * x[i]; }
  const LD rho = num / den;
  double er = 0.0, nr = 0.0;
  for (int i = 0; i < n; ++i) {
    const LD r = ldexpl(y[i] - rho * x[i], -ex);
    er = fmax(er, fabs((double)(r - rh[i])));
    nr = fmax(nr, fabs((double)r));
  }
  // s = P Q^T (-rh)
  std::vector<LD> qs(n);
  LD zs = 0;
  for (int k = 0; k < n; ++k) {
    qs[k] = 0;
    for (int i = 0; i < n; ++i) qs[k] += Q[i + (size_t)k * n] * -(LD)rh[i];
    zs += qs[k] * z[k];
  }
  double es = 0.0, ns = 0.0;
  for (int k = 0; k < n; ++k) {
    es = fmax(es, fabs((double)(qs[k] - zs * z[k] - s[k])));
    ns = fmax(ns, fabs(s[k]));
  }
  // (T_s - lam) d' - s
  double ed = 0.0, nd = 0.0;
  for (int i = 0; i < n; ++i) {
    LD t = ((LD)dg[i] - lam) * dp[i];
    if (i > 0) t += (LD)eo[i - 1] * dp[i - 1];
    if (i + 1 < n) t += (LD)eo[i] * dp[i + 1];
    ed = fmax(ed, fabs((double)(t - s[i])));
    nd = fmax(nd, fabs(dp[i]));
  }
  // d - Q P d'
  LD zd = 0;
  for (int k = 0; k < n; ++k) zd += (LD)z[k] * dp[k];
  double eqd = 0.0;
  for (int i = 0; i < n; ++i) {
    LD t = 0;
    for (int k = 0; k < n; ++k) t += Q[i + (size_t)k * n] * ((LD)dp[k] - zd * z[k]);
    eqd = fmax(eqd, fabs((double)(t - d[i])));
  }
  // the corrected residual in long double: A (x + d) - rho' (x + d)
  std::vector<LD> x2(n), y2(n);
  for (int i = 0; i < n; ++i) x2[i] = (LD)x[i] + d[i];
  LD num2 = 0, den2 = 0;
  for (int i = 0; i < n; ++i) {
    y2[i] = 0;
    for (int j = 0; j < n; ++j) y2[i] += (LD)Ah[i + (size_t)j * n] * x2[j];
  }
  for (int i = 0; i < n; ++i) { num2 += x2[i] * y2[i]; den2 += x2[i] * x2[i]; }
  double nr2 = 0.0;
  for (int i = 0; i < n; ++i) nr2 = fmax(nr2, fabs((double)(y2[i] - num2 / den2 * x2[i])));
  printf("n=%d ex=%d lam=%.17g: |Q^T A Q - T| %.2e (|T| %.2e), |(T-lam)z| %.2e, |x-Qz| %.2e, |r| %.2e "
         "(dev err %.2e), |s| %.2e (err %.2e), |d'| %.2e solve res %.2e, |d - QPd'| %.2e, |z^T s| %.2e, "
         "corrected |r| (long double) %.2e\n",
         n, ex, lam, et, at, ez, ex_, nr, er, ns, es, nd, ed, eqd, (double)fabsl(zs), nr2);
  CK(hipFree(dA));
  CK(hipFree(dE));
  CK(hipFree(dd_));
}

int main() {
  run(18);
  run(40);
  run(64);
  return 0;
}
