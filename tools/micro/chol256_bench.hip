// chol_inv_tiles<256> (one workgroup per matrix, 768 threads) on a batch of SPD matrices of
// n = 255 (the S_j of C3), and n = 129, 200: time per launch (best of 5) and the largest
// |L^-1 A L^-T - I| over the first few matrices, in place and out of place; the same batch
// split as the 2x2-blocked path factors it is not timed here (that is the body's A/B).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form chol256_bench.hip \
//     -o ../../microbin/chol256_bench && ../../microbin/chol256_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static int run(int n, int nb, bool inplace) {
  std::vector<double> h((size_t)nb * n * n);
  srand(3 + n);
  for (int b = 0; b < nb; ++b) {  // A = I + G G^T / n
    std::vector<double> G((size_t)n * n);
    for (auto& g : G) g = rand() / (double)RAND_MAX - 0.5;
    double* A = h.data() + (size_t)b * n * n;
    for (int j = 0; j < n; ++j)
      for (int i = j; i < n; ++i) {
        double s = i == j ? 1.0 : 0.0;
        for (int k = 0; k < n; ++k) s += G[i + (size_t)k * n] * G[j + (size_t)k * n] / n;
        A[i + (size_t)j * n] = A[j + (size_t)i * n] = s;
      }
  }
  double *dA, *dO;
  int* info;
  CK(hipMalloc(&dA, h.size() * 8));
  CK(hipMalloc(&dO, h.size() * 8));
  CK(hipMalloc(&info, nb * 4));
  std::vector<MatDesc<double>> din(nb), dout(nb);
  for (int b = 0; b < nb; ++b) {
    din[b] = {dA + (size_t)b * n * n, n, n};
    dout[b] = {(inplace ? dA : dO) + (size_t)b * n * n, n, n};
  }
  MatDesc<double>*ddin, *ddout;
  CK(hipMalloc(&ddin, nb * sizeof(MatDesc<double>)));
  CK(hipMalloc(&ddout, nb * sizeof(MatDesc<double>)));
  CK(hipMemcpy(ddin, din.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
  CK(hipMemcpy(ddout, dout.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)chol_inv_tiles<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                         (int)chol_inv_tiles_lds<256>()));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    CK(hipMemcpy(dA, h.data(), h.size() * 8, hipMemcpyHostToDevice));  // (in place: fresh input)
    CK(hipEventRecord(e0));
    chol_inv_tiles<256><<<nb, CholTiles<256>::NTH, chol_inv_tiles_lds<256>()>>>(ddin, ddout, info, 1);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) best = fminf(best, ms * 1e3f);
  }
  std::vector<int> hinfo(nb);
  CK(hipMemcpy(hinfo.data(), info, nb * 4, hipMemcpyDeviceToHost));
  int bad_info = 0;
  for (int v : hinfo) bad_info += v != 0;
  std::vector<double> Li((size_t)n * n);
  double err = 0;
  for (int b = 0; b < 3 && b < nb; ++b) {
    CK(hipMemcpy(Li.data(), (inplace ? dA : dO) + (size_t)b * n * n, (size_t)n * n * 8, hipMemcpyDeviceToHost));
    const double* A = h.data() + (size_t)b * n * n;
    std::vector<double> T((size_t)n * n, 0.0);  // T = Li A
    for (int j = 0; j < n; ++j)
      for (int k = 0; k < n; ++k) {
        const double a = A[k + (size_t)j * n];
        for (int i = 0; i < n; ++i) T[i + (size_t)j * n] += Li[i + (size_t)k * n] * a;
      }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += T[i + (size_t)k * n] * Li[j + (size_t)k * n];
        err = fmax(err, fabs(s - (i == j ? 1.0 : 0.0)));
      }
    for (int j = 0; j < n; ++j)  // zero above the diagonal
      for (int i = 0; i < j; ++i) err = fmax(err, fabs(Li[i + (size_t)j * n]));
  }
  printf("chol_inv_tiles<256> n=%3d batch=%3d %s: %7.1f us  max|L^-1 A L^-T - I| %.2e  failed pivots %d%s\n",
         n, nb, inplace ? "in place " : "separate ", best, err, bad_info,
         (err > 1e-10 || bad_info) ? "  MISMATCH" : "");
  CK(hipFree(dA));
  CK(hipFree(dO));
  CK(hipFree(info));
  CK(hipFree(ddin));
  CK(hipFree(ddout));
  return err > 1e-10 || bad_info;
}

int main() {
  int bad = 0;
  bad += run(255, 64, true);
  bad += run(255, 64, false);
  bad += run(255, 8, true);
  bad += run(129, 64, true);
  bad += run(200, 16, false);
  bad += run(256, 8, false);
  printf("%s\n", bad ? "FAILED" : "all match");
  return bad;
}
