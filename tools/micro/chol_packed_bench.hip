// Multi-word Cholesky (+ L^-1) of a batch of random SPD n x n blocks: chol_inv_reg (fixed tile
// grid, 1024 threads) against chol_packed (liveness-packed slots) at 1024, 512 and 256 threads,
// which must agree bitwise (same operations per element), and the square-root-free chol_packed
// LDL (1024 threads; max relative difference of L and L^-1 entries to chol_inv_reg's).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 chol_packed_bench.hip -o bin/chol_packed_bench
//   bin/chol_packed_bench n batch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
using mw::dd;
using mw::qd;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

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

template <class T, bool INV>
void run(const char* name, int n, int nb) {
  const size_t nn = (size_t)n * n;
  std::vector<T> h(nn * nb);
  srand(11);
  for (int b = 0; b < nb; ++b) {  // A = B B^T / n + I
    std::vector<double> B(nn);
    for (auto& v : B) v = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        T s = T(i == j ? 1.0 : 0.0);
        for (int k = 0; k < n; ++k) s = s + T(B[i + k * n] * B[j + k * n] / n);
        h[b * nn + i + (size_t)j * n] = s;
      }
  }
  T *dA, *dO[5];
  CK(hipMalloc(&dA, h.size() * sizeof(T)));
  CK(hipMemcpy(dA, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  for (auto& p : dO) CK(hipMalloc(&p, 2 * h.size() * sizeof(T)));
  std::vector<MatDesc<T>> din(nb), dout[5][2];
  for (int b = 0; b < nb; ++b) din[b] = {dA + b * nn, n, n};
  MatDesc<T>*ddin, *ddout[5][2];
  CK(hipMalloc(&ddin, nb * sizeof(MatDesc<T>)));
  CK(hipMemcpy(ddin, din.data(), nb * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  for (int q = 0; q < 5; ++q)
    for (int o = 0; o < 2; ++o) {
      dout[q][o].resize(nb);
      for (int b = 0; b < nb; ++b) dout[q][o][b] = {dO[q] + (o * nb + b) * nn, n, n};
      CK(hipMalloc(&ddout[q][o], nb * sizeof(MatDesc<T>)));
      CK(hipMemcpy(ddout[q][o], dout[q][o].data(), nb * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
    }
  int* info;
  CK(hipMalloc(&info, 5 * nb * sizeof(int)));
  const float t0 = timeit([&] { chol_inv_reg<T, 1, 4, 64, 16, INV><<<nb, 1024>>>(ddin, ddout[0][0], ddout[0][1], info); });
  const float t1 = timeit([&] { chol_packed<T, 1024, INV><<<nb, 1024>>>(ddin, ddout[1][0], ddout[1][1], info + nb); });
  const float t2 = timeit([&] { chol_packed<T, 512, INV><<<nb, 512>>>(ddin, ddout[2][0], ddout[2][1], info + 2 * nb); });
  const float t3 = timeit([&] { chol_packed<T, 256, INV><<<nb, 256>>>(ddin, ddout[3][0], ddout[3][1], info + 3 * nb); });
  const float t4 = timeit([&] { chol_packed<T, 1024, INV, true><<<nb, 1024>>>(ddin, ddout[4][0], ddout[4][1], info + 4 * nb); });
  CK(hipDeviceSynchronize());
  std::vector<T> o0(2 * h.size()), o1(2 * h.size());
  std::vector<int> hi(5 * nb);
  CK(hipMemcpy(hi.data(), info, 5 * nb * sizeof(int), hipMemcpyDeviceToHost));
  CK(hipMemcpy(o0.data(), dO[0], o0.size() * sizeof(T), hipMemcpyDeviceToHost));
  bool same = true;
  for (int q = 1; q < 4; ++q) {
    CK(hipMemcpy(o1.data(), dO[q], o1.size() * sizeof(T), hipMemcpyDeviceToHost));
    // L (second half) always; L^-1 (first half) with INV
    const size_t from = INV ? 0 : h.size();
    same = same && std::memcmp(o0.data() + from, o1.data() + from, (o0.size() - from) * sizeof(T)) == 0;
  }
  CK(hipMemcpy(o1.data(), dO[4], o1.size() * sizeof(T), hipMemcpyDeviceToHost));
  double rel = 0.0;
  for (size_t i = INV ? 0 : h.size(); i < o0.size(); ++i) {
    const double a = Num<T>::hi(o0[i]);
    if (a != 0.0) rel = fmax(rel, fabs(Num<T>::hi(o1[i] - o0[i])) / fabs(a));
    else if (Num<T>::hi(o1[i]) != 0.0) rel = 1.0;
  }
  int bad = 0;
  for (int v : hi) bad += v != 0;
  printf("%s n=%d batch=%d INV=%d: chol_inv_reg %.1f us | chol_packed 1024 %.1f us, 512 %.1f us, 256 %.1f us | bitwise %s | LDL %.1f us, max rel diff %.1e | info!=0: %d\n",
         name, n, nb, (int)INV, t0, t1, t2, t3, same ? "same" : "DIFFERENT", t4, rel, bad);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 51, nb = argc > 2 ? atoi(argv[2]) : 7;
  run<qd, false>("qd", n, nb);
  run<qd, true>("qd", n, nb);
  run<dd, false>("dd", n, nb);
  run<dd, true>("dd", n, nb);
  return 0;
}
