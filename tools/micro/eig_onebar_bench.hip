// eigmin_onebar (one barrier per column, round 6) against eigmin_split<0, 24> (the round-5
// default) on batches of symmetric fp64 blocks: time per launch (best of 5), the largest
// |difference| of lambda_min relative to the block's max-norm, and a host Jacobi spot check,
// over the structures of eig_split_bench.hip (random, near-diagonal, tridiagonal, decoupled
// 16-blocks), several n, batches and scalings.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form eig_onebar_bench.hip \
//     -o ../../microbin/eig_onebar_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

template <class K>
float timeit(K k) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  k();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    float ms;
    CK(hipEventRecord(e0));
    k();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = fminf(best, ms * 1e3f);
  }
  return best;
}

static double jacobi_min(std::vector<double> A, int n) {
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int p = 0; p < n; ++p) for (int q = p + 1; q < n; ++q) off += A[p + q * n] * A[p + q * n];
    if (off < 1e-300) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p + q * n];
        if (apq == 0.0) continue;
        const double th = (A[q + q * n] - A[p + p * n]) / (2 * apq);
        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
        const double cs = 1 / sqrt(t * t + 1), sn = t * cs;
        for (int k = 0; k < n; ++k) {
          const double akp = A[k + p * n], akq = A[k + q * n];
          A[k + p * n] = cs * akp - sn * akq;
          A[k + q * n] = sn * akp + cs * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = A[p + k * n], aqk = A[q + k * n];
          A[p + k * n] = cs * apk - sn * aqk;
          A[q + k * n] = sn * apk + cs * aqk;
        }
      }
  }
  double m = INFINITY;
  for (int i = 0; i < n; ++i) m = fmin(m, A[i + i * n]);
  return m;
}

int run(int n, int nb, double scale, int kind, int nhost) {
  std::vector<double> h((size_t)nb * n * n);
  srand(11 + n + nb + kind);
  for (int b = 0; b < nb; ++b) {
    double* M = h.data() + (size_t)b * n * n;
    for (int j = 0; j < n; ++j)
      for (int i = j; i < n; ++i) {
        double v = rand() / (double)RAND_MAX - 0.5;
        if (kind == 1) v = (i == j) ? 1.0 + 0.1 * v : 1e-3 * v;
        if (kind == 2) v = (i == j) ? (double)(i % 7) : (i == j + 1 ? 1.0 : 0.0);
        if (kind == 3 && ((i / 16) != (j / 16))) v = 0.0;
        M[i + j * n] = M[j + i * n] = v * scale;
      }
  }
  double *dA, *dE;
  CK(hipMalloc(&dA, h.size() * 8));
  CK(hipMalloc(&dE, 2 * nb * 8));
  CK(hipMemcpy(dA, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  std::vector<MatDesc<double>> din(nb);
  for (int b = 0; b < nb; ++b) din[b] = {dA + (size_t)b * n * n, n, n};
  MatDesc<double>* ddin;
  CK(hipMalloc(&ddin, nb * sizeof(MatDesc<double>)));
  CK(hipMemcpy(ddin, din.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
  const float t_old = timeit([&] { eigmin_split<0, 24><<<nb, 576>>>(ddin, dE); });
  const float t_new = timeit([&] { eigmin_onebar<0><<<nb, 576>>>(ddin, dE + nb); });
  CK(hipDeviceSynchronize());
  std::vector<double> ev(2 * nb);
  CK(hipMemcpy(ev.data(), dE, 2 * nb * 8, hipMemcpyDeviceToHost));
  double dmax = 0;
  for (int b = 0; b < nb; ++b) {
    double amax = 0;
    for (size_t q = 0; q < (size_t)n * n; ++q) amax = fmax(amax, fabs(h[(size_t)b * n * n + q]));
    if (amax > 0) dmax = fmax(dmax, fabs(ev[b] - ev[nb + b]) / amax);
  }
  printf("n=%3d batch=%3d kind=%d scale=%8.1e  eigmin_split<0,24> %7.1f us  eigmin_onebar %7.1f us  "
         "max|diff|/|A| %.2e", n, nb, kind, scale, t_old, t_new, dmax);
  int bad = dmax > 1e-13;
  double eh = 0;
  for (int b = 0; b < nhost && b < nb; ++b) {
    std::vector<double> A0(h.begin() + (size_t)b * n * n, h.begin() + (size_t)(b + 1) * n * n);
    double amax = 0;
    for (double x : A0) amax = fmax(amax, fabs(x));
    const double ref = jacobi_min(A0, n);
    if (amax > 0) eh = fmax(eh, fabs(ev[nb + b] - ref) / amax);
  }
  if (nhost) {
    printf("  host-Jacobi(%d) |diff|/|A| %.2e", nhost, eh);
    bad |= eh > 1e-12;
  }
  printf("%s\n", bad ? "  MISMATCH" : "");
  CK(hipFree(dA));
  CK(hipFree(dE));
  CK(hipFree(ddin));
  return bad;
}

int main() {
  {  // timing experiments on the C3 batch (DBG variants: wrong results, timing only)
    const int n = 128, nb = 128;
    std::vector<double> h((size_t)nb * n * n);
    srand(5);
    for (int b = 0; b < nb; ++b)
      for (int j = 0; j < n; ++j)
        for (int i = j; i < n; ++i) h[(size_t)b * n * n + i + j * n] = h[(size_t)b * n * n + j + i * n] = rand() / (double)RAND_MAX - 0.5;
    double *dA, *dE;
    CK(hipMalloc(&dA, h.size() * 8));
    CK(hipMalloc(&dE, nb * 8));
    CK(hipMemcpy(dA, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<MatDesc<double>> din(nb);
    for (int b = 0; b < nb; ++b) din[b] = {dA + (size_t)b * n * n, n, n};
    MatDesc<double>* dd;
    CK(hipMalloc(&dd, nb * sizeof(MatDesc<double>)));
    CK(hipMemcpy(dd, din.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
    printf("onebar DBG (n=128, batch=128): full %.1f | no update %.1f | no matvec %.1f | no update+matvec %.1f | no reflector %.1f | nothing %.1f  (split %.1f)\n",
           timeit([&] { eigmin_onebar<0><<<nb, 576>>>(dd, dE); }),
           timeit([&] { eigmin_onebar<1><<<nb, 576>>>(dd, dE); }),
           timeit([&] { eigmin_onebar<2><<<nb, 576>>>(dd, dE); }),
           timeit([&] { eigmin_onebar<3><<<nb, 576>>>(dd, dE); }),
           timeit([&] { eigmin_onebar<4><<<nb, 576>>>(dd, dE); }),
           timeit([&] { eigmin_onebar<7><<<nb, 576>>>(dd, dE); }),
           timeit([&] { eigmin_split<0, 24><<<nb, 576>>>(dd, dE); }));
    CK(hipFree(dA));
    CK(hipFree(dE));
    CK(hipFree(dd));
  }
  int bad = 0;
  bad += run(128, 128, 1.0, 0, 2);
  bad += run(128, 16, 1.0, 0, 2);
  bad += run(128, 256, 1.0, 0, 0);
  bad += run(128, 128, 1e-200, 0, 0);
  bad += run(128, 128, 1e200, 0, 0);
  for (int kind = 1; kind <= 3; ++kind) bad += run(128, 64, 1.0, kind, 2);
  for (int n : {1, 2, 3, 4, 5, 8, 9, 17, 33, 64, 100, 127})
    for (int kind = 0; kind <= 3; ++kind) bad += run(n, 64, 1.0, kind, n <= 64 ? 3 : 1);
  printf("%s\n", bad ? "FAILED" : "all match");
  return bad ? 1 : 0;
}
