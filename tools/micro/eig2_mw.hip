// Multi-word eigenvalue kernels on a batch of random symmetric n x n matrices: eigmin_lds (four
// barriers per column) against eigmin_lds2 (two), the tridiagonalisation alone (eigmin_lds2 DBG
// = 1), and the largest difference of the two lambda_min.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 eig2_mw.hip -o bin/eig2_mw && bin/eig2_mw n batch
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

template <class T>
void run(const char* name, int n, int nb) {
  std::vector<T> ht((size_t)n * n * nb);
  srand(7);
  for (int b = 0; b < nb; ++b)
    for (int j = 0; j < n; ++j)
      for (int i = 0; i <= j; ++i) {
        const double v = (double)rand() / RAND_MAX - 0.5 + (i == j ? 0.1 * (j % 7) : 0.0);
        ht[(size_t)b * n * n + i + (size_t)j * n] = T(v);
        ht[(size_t)b * n * n + j + (size_t)i * n] = T(v);
      }
  T *dA, *dE;
  CK(hipMalloc(&dA, ht.size() * sizeof(T)));
  CK(hipMalloc(&dE, 3 * nb * sizeof(T)));
  CK(hipMemcpy(dA, ht.data(), ht.size() * sizeof(T), hipMemcpyHostToDevice));
  std::vector<MatDesc<T>> din(nb);
  for (int b = 0; b < nb; ++b) din[b] = {dA + (size_t)b * n * n, n, n};
  MatDesc<T>* dd_;
  CK(hipMalloc(&dd_, nb * sizeof(MatDesc<T>)));
  CK(hipMemcpy(dd_, din.data(), nb * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  const size_t l1 = sizeof(T) * ((size_t)n * n + (n <= 64 ? 14 : 10) * n + 40);
  const size_t l2 = eig2_lds_bytes<T>(n);
  CK(hipFuncSetAttribute((const void*)eigmin_lds<T, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)eigmin_lds2<T, true, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)eigmin_lds2<T, true, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const float t1 = timeit([&] { eigmin_lds<T, true><<<nb, 512, l1>>>(dd_, dE); });
  const float t2 = timeit([&] { eigmin_lds2<T, true, 0><<<nb, 512, l2>>>(dd_, dE + nb); });
  const float t3 = timeit([&] { eigmin_lds2<T, true, 1><<<nb, 512, l2>>>(dd_, dE + 2 * nb); });
  std::vector<T> ev(2 * nb);
  CK(hipMemcpy(ev.data(), dE, 2 * nb * sizeof(T), hipMemcpyDeviceToHost));
  double md = 0.0;
  for (int b = 0; b < nb; ++b) {
    const T df = ev[b] - ev[nb + b];
    md = fmax(md, fabs(Num<T>::hi(df)) / fmax(1e-300, fabs(Num<T>::hi(ev[b]))));
  }
  printf("%s n=%d batch=%d: eigmin_lds %.1f us, eigmin_lds2 %.1f us (tridiagonalisation %.1f us), "
         "max rel diff %.2e\n", name, n, nb, t1, t2, t3, md);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 64, nb = argc > 2 ? atoi(argv[2]) : 32;
  run<dd>("dd", n, nb);
  if (n <= 64) run<qd>("qd", n, nb);
  return 0;
}
