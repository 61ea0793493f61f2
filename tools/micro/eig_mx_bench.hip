// eigmin_mx (fp64 eigenpair + multi-word refinement) against eigmin_lds2 (multi-word
// tridiagonalisation) on batches of symmetric n x n blocks: time per batch, the largest
// difference of the two lambda_min relative to the block's magnitude, and the number of blocks
// eigmin_mx handed to its multi-word fallback.  Three families: random symmetric (separated
// lambda_min), lambda_min with a close second eigenvalue (gap 2^-g, g = 10, 30, 45: Q diag Q^T
// with a random orthogonal Q built at fp64 and rounded, so the gap is only approximately 2^-g),
// and c I (a multiple eigenvalue: every block falls back).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 eig_mx_bench.hip -o microbin/eig_mx_bench
//   microbin/eig_mx_bench [n] [batch]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <random>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
using mw::dd;
using mw::qd;
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

// random orthogonal Q (n x n, column-major) by Gram-Schmidt twice
static std::vector<double> rand_orth(int n, std::mt19937_64& g) {
  std::normal_distribution<double> nd;
  std::vector<double> Q((size_t)n * n);
  for (auto& v : Q) v = nd(g);
  for (int j = 0; j < n; ++j)
    for (int pass = 0; pass < 2; ++pass) {
      for (int k = 0; k < j; ++k) {
        double s = 0;
        for (int i = 0; i < n; ++i) s += Q[i + (size_t)k * n] * Q[i + (size_t)j * n];
        for (int i = 0; i < n; ++i) Q[i + (size_t)j * n] -= s * Q[i + (size_t)k * n];
      }
      double s = 0;
      for (int i = 0; i < n; ++i) s += Q[i + (size_t)j * n] * Q[i + (size_t)j * n];
      s = 1.0 / sqrt(s);
      for (int i = 0; i < n; ++i) Q[i + (size_t)j * n] *= s;
    }
  return Q;
}

template <class T>
void run(const char* name, int n, int nb, int family, int gexp) {
  std::vector<T> ht((size_t)n * n * nb);
  std::mt19937_64 g(7 + family * 100 + gexp);
  std::uniform_real_distribution<double> ud(-0.5, 0.5);
  for (int b = 0; b < nb; ++b) {
    T* A = ht.data() + (size_t)b * n * n;
    if (family == 0) {
      for (int j = 0; j < n; ++j)
        for (int i = 0; i <= j; ++i) {
          // a multi-word entry: fp64 value plus a lower word
          const T v = T(ud(g) + (i == j ? 0.1 * (j % 7) : 0.0)) + T(ud(g) * 0x1p-60);
          A[i + (size_t)j * n] = v;
          A[j + (size_t)i * n] = v;
        }
    } else if (family == 1) {
      const std::vector<double> Q = rand_orth(n, g);
      std::vector<double> lam(n);
      lam[0] = -0.5;
      lam[1] = -0.5 + ldexp(1.0, -gexp);
      for (int i = 2; i < n; ++i) lam[i] = -0.4 + 0.8 * (double)i / n;
      for (int j = 0; j < n; ++j)
        for (int i = 0; i <= j; ++i) {
          T s = T(0.0);
          for (int k = 0; k < n; ++k) s = s + T(Q[i + (size_t)k * n]) * T(Q[j + (size_t)k * n]) * T(lam[k]);
          A[i + (size_t)j * n] = s;
          A[j + (size_t)i * n] = s;
        }
    } else {
      for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) A[i + (size_t)j * n] = T(i == j ? 0.75 : 0.0);
    }
  }
  T *dA, *dE;
  int* redo;
  CK(hipMalloc(&redo, nb * sizeof(int)));
  CK(hipMalloc(&dA, ht.size() * sizeof(T)));
  CK(hipMalloc(&dE, 2 * nb * sizeof(T)));
  CK(hipMemcpy(dA, ht.data(), ht.size() * sizeof(T), hipMemcpyHostToDevice));
  std::vector<MatDesc<T>> din(nb);
  for (int b = 0; b < nb; ++b) din[b] = {dA + (size_t)b * n * n, n, n};
  MatDesc<T>* dd_;
  CK(hipMalloc(&dd_, nb * sizeof(MatDesc<T>)));
  CK(hipMemcpy(dd_, din.data(), nb * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  const size_t l2 = eig2_lds_bytes<T>(n), lm = eigmx_lds_bytes<T>(n);
  CK(hipFuncSetAttribute((const void*)eigmin_lds2<T, true, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)eigmin_mx<T>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - EIGMX_STATIC_LDS));
  const float t2 = timeit([&] { eigmin_lds2<T, true, 0><<<nb, 512, l2>>>(dd_, dE); });
  unsigned zero = 0, fb = 0;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_eigmx_fallbacks), &zero, sizeof(zero)));
  eigmin_mx<T><<<nb, 576, lm>>>(dd_, dE + nb, redo);
  eigmin_lds2<T, true, 0><<<nb, 512, l2>>>(dd_, dE + nb, redo);
  CK(hipDeviceSynchronize());
  CK(hipMemcpyFromSymbol(&fb, HIP_SYMBOL(g_eigmx_fallbacks), sizeof(fb)));
  const float tm = timeit([&] {
    eigmin_mx<T><<<nb, 576, lm>>>(dd_, dE + nb, redo);
    eigmin_lds2<T, true, 0><<<nb, 512, l2>>>(dd_, dE + nb, redo);
  });
  CK(hipFuncSetAttribute((const void*)eigmin_mx<T, 0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const float tl = timeit([&] {
    eigmin_mx<T, 0, 0><<<nb, 512, lm>>>(dd_, dE + nb, redo);
    eigmin_lds2<T, true, 0><<<nb, 512, l2>>>(dd_, dE + nb, redo);
  });
  // diagnostics of the DBG instance: phase stamps (s_memtime ticks) averaged over the
  // blocks, and eta / lambda / lambda_2 / rho / Temple width of the first rejected blocks
  CK(hipFuncSetAttribute((const void*)eigmin_mx<T, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - EIGMX_STATIC_LDS));
  std::vector<double> dz(256 * 24, 0.0);
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_eigmx_dbg), dz.data(), dz.size() * sizeof(double)));
  eigmin_mx<T, 1><<<nb, 576, lm>>>(dd_, dE + nb, redo);
  eigmin_lds2<T, true, 0><<<nb, 512, l2>>>(dd_, dE + nb, redo);
  CK(hipDeviceSynchronize());
  CK(hipMemcpyFromSymbol(dz.data(), HIP_SYMBOL(g_eigmx_dbg), dz.size() * sizeof(double)));
  {
    double avg[16] = {0};
    for (int b = 0; b < nb; ++b)
      for (int q = 0; q < 16; ++q) avg[q] += dz[b * 24 + q] / nb;
    printf("  stamps (k s_memtime ticks): load %.1f tridiag %.1f multisection+gap %.1f lu+invit %.1f backtransform %.1f | refine",
           avg[0] / 1e3, avg[1] / 1e3, avg[2] / 1e3, avg[3] / 1e3, avg[4] / 1e3);
    for (int q = 5; q < 16; ++q) printf(" %.1f", avg[q] / 1e3);
    printf("\n");
    int shown = 0;
    for (int b = 0; b < nb && shown < 4; ++b) {
      const double* z = &dz[b * 24];
      if (z[23] > 0.0 && z[23] <= 0x1p-3 * Num<T>::eps()) continue;
      ++shown;
      printf("  rejected block %d: eta %.3e %.3e %.3e lam %.17g lam2 %.17g rho %.17g temple %.3e\n", b,
             z[16], z[17], z[18], z[20], z[21], z[22], z[23]);
    }
  }
  std::vector<T> ev(2 * nb);
  CK(hipMemcpy(ev.data(), dE, 2 * nb * sizeof(T), hipMemcpyDeviceToHost));
  double md = 0.0;
  for (int b = 0; b < nb; ++b) {
    const T df = ev[b] - ev[nb + b];
    md = fmax(md, fabs(Num<T>::hi(df)));
  }
  printf("%s n=%d batch=%d family=%d gap=2^-%d: eigmin_lds2 %.1f us, eigmin_mx %.1f us (LDS tridiagonalisation %.1f us), "
         "max |diff| %.2e, fallbacks %u/%d, lambda_min[0] %.17g\n",
         name, n, nb, family, gexp, t2, tm, tl, md, fb, nb, Num<T>::hi(ev[nb]));
  CK(hipFree(dA));
  CK(hipFree(dE));
  CK(hipFree(dd_));
  CK(hipFree(redo));
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 64, nb = argc > 2 ? atoi(argv[2]) : 32;
  run<dd>("dd", n, nb, 0, 0);
  run<dd>("dd", n, nb, 1, 10);
  run<dd>("dd", n, nb, 1, 30);
  run<dd>("dd", n, nb, 1, 45);
  run<dd>("dd", n, nb, 2, 0);
  run<qd>("qd", 48, nb, 0, 0);
  run<qd>("qd", 48, nb, 1, 20);
  run<qd>("qd", 18, 22, 0, 0);
  return 0;
}
