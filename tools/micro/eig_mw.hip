// Multi-word eigmin_lds: Newton refinement (eigmin_lds<T, true>) against the multisection
// (eigmin_lds<T, false>) on a batch of random symmetric n x n matrices: time per launch and the
// largest difference of the two lambda_min.  Build with -DCLRSDP_EIG_STAMPS for the split
// between the Householder reduction and the eigenvalue phase.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DCLRSDP_EIG_STAMPS] eig_mw.hip -o eig_mw
//   ./eig_mw n batch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
using mw::dd;
using mw::qd;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

template <class T>
void run(const char* name, int n, int nb, const std::vector<double>& h) {
  std::vector<T> ht(h.size());
  for (size_t i = 0; i < h.size(); ++i) ht[i] = T(h[i]);
  T *dA, *dE;
  CK(hipMalloc(&dA, ht.size() * sizeof(T)));
  CK(hipMalloc(&dE, 2 * nb * sizeof(T)));
  CK(hipMemcpy(dA, ht.data(), ht.size() * sizeof(T), hipMemcpyHostToDevice));
  std::vector<MatDesc<T>> din(nb);
  for (int b = 0; b < nb; ++b) din[b] = {dA + (size_t)b * n * n, n, n};
  MatDesc<T>* ddin;
  CK(hipMalloc(&ddin, nb * sizeof(MatDesc<T>)));
  CK(hipMemcpy(ddin, din.data(), nb * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  const size_t lds = sizeof(T) * ((size_t)n * n + (n <= 64 ? 14 : 10) * n + 40);  // eig_lds_bytes
  CK(hipFuncSetAttribute((const void*)eigmin_lds<T, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)eigmin_lds<T, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int nw = 0; nw < 2; ++nw) {
#ifdef CLRSDP_EIG_STAMPS
    unsigned long long z[8] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_eig_stamps), z, sizeof(z)));
#endif
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      float ms;
      CK(hipEventRecord(e0));
      if (nw) eigmin_lds<T, true><<<nb, 512, lds>>>(ddin, dE + nb);
      else eigmin_lds<T, false><<<nb, 512, lds>>>(ddin, dE);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = fminf(best, ms);
    }
    printf("%s eigmin_lds<%s> n=%d batch=%d: %.1f us\n", name, nw ? "newton" : "multisection", n, nb,
           best * 1e3);
#ifdef CLRSDP_EIG_STAMPS
    unsigned long long st[8];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_eig_stamps), sizeof(st)));
    double hh = 0;
    for (int q = 0; q < 6; ++q) hh += st[q];
    printf("  cycles per matrix: householder %.0f  eigenvalue phase %.0f (fp64 bracket %.0f, multi-word %.0f)\n",
           hh / (3.0 * nb), (st[6] + st[7]) / (3.0 * nb), st[7] / (3.0 * nb), st[6] / (3.0 * nb));
    printf("  householder: reflector %.0f, A'v %.0f, reduce+barrier %.0f, w %.0f, update %.0f\n",
           st[0] / (3.0 * nb), st[1] / (3.0 * nb), st[2] / (3.0 * nb), st[3] / (3.0 * nb), st[4] / (3.0 * nb));
#endif
  }
  std::vector<T> ev(2 * nb);
  CK(hipMemcpy(ev.data(), dE, 2 * nb * sizeof(T), hipMemcpyDeviceToHost));
  double dmax = 0, rel = 0;
  for (int b = 0; b < nb; ++b) {
    const T df = ev[b] - ev[nb + b];
    const double a = fabs(mw::Num<T>::hi(df));
    dmax = fmax(dmax, a);
    rel = fmax(rel, a / fabs(mw::Num<T>::hi(ev[b])));
  }
  printf("  max |newton - multisection| = %.3e (relative %.3e), lambda_min[0] = %.17g\n", dmax, rel,
         mw::Num<T>::hi(ev[0]));
  CK(hipFree(dA));
  CK(hipFree(dE));
  CK(hipFree(ddin));
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 18, nb = argc > 2 ? atoi(argv[2]) : 22;
  std::vector<double> h((size_t)nb * n * n);
  srand(7);
  for (int b = 0; b < nb; ++b)
    for (int j = 0; j < n; ++j)
      for (int i = 0; i <= j; ++i) {
        const double v = rand() / (double)RAND_MAX - 0.5;
        h[(size_t)b * n * n + i + (size_t)j * n] = v;
        h[(size_t)b * n * n + j + (size_t)i * n] = v;
      }
  // a block with a double eigenvalue at the bottom (diag(-1, -1, 1, 2, ...)): the Newton path
  // converges linearly there and must still agree, through the fallback if need be
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i + (size_t)j * n] = (i == j) ? (i < 2 ? -1.0 : 1.0 + i) : 0.0;
  run<dd>("dd", n, nb, h);
  run<qd>("qd", n, nb, h);
  return 0;
}
