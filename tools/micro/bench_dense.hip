// Standalone timing of the on-chip dense kernels (chol_inv_reg, eigmin_lds) on a batch of SPD
// matrices, with a correctness spot check (||L^-1 A L^-T - I||, lambda_min vs power iteration).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 128, nb = argc > 2 ? atoi(argv[2]) : 64;
  std::vector<double> h((size_t)nb * n * n);
  srand(1);
  for (int b = 0; b < nb; ++b) {
    std::vector<double> G((size_t)n * n);
    for (auto& g : G) g = (rand() / (double)RAND_MAX - 0.5);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double s = (i == j) ? 1.0 : 0.0;
        for (int k = 0; k < n; ++k) s += G[i + k * n] * G[j + k * n] / n;
        h[(size_t)b * n * n + i + j * n] = s;
      }
  }
  double *dA, *dO, *dE;
  CK(hipMalloc(&dA, h.size() * 8)); CK(hipMalloc(&dO, h.size() * 8)); CK(hipMalloc(&dE, 2 * nb * 8));
  CK(hipMemcpy(dA, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  std::vector<MatDesc<double>> din(nb), dout(nb);
  for (int b = 0; b < nb; ++b) { din[b] = {dA + (size_t)b * n * n, n, n}; dout[b] = {dO + (size_t)b * n * n, n, n}; }
  MatDesc<double> *ddin, *ddout; int* info;
  CK(hipMalloc(&ddin, nb * sizeof(MatDesc<double>))); CK(hipMalloc(&ddout, nb * sizeof(MatDesc<double>)));
  CK(hipMalloc(&info, nb * 4));
  CK(hipMemcpy(ddin, din.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
  CK(hipMemcpy(ddout, dout.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    chol_inv_reg<double, 4, 8, 32, 16><<<nb, 512>>>(ddin, ddout, nullptr, info);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("chol_inv_reg n=%d batch=%d: %.1f us\n", n, nb, ms * 1e3);
  }
  {
    int NPv = n <= 32 ? 32 : n <= 64 ? 64 : 128;
    size_t lds = NPv == 32 ? chol_inv_tiles_lds<32>() : NPv == 64 ? chol_inv_tiles_lds<64>() : chol_inv_tiles_lds<128>();
    CK(hipFuncSetAttribute((const void*)chol_inv_tiles<128>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      if (NPv == 128) chol_inv_tiles<128><<<nb, 512, lds>>>(ddin, ddout, info);
      else if (NPv == 64) chol_inv_tiles<64><<<nb, 512, lds>>>(ddin, ddout, info);
      else chol_inv_tiles<32><<<nb, 512, lds>>>(ddin, ddout, info);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      printf("chol_inv_tiles<%d> n=%d batch=%d: %.1f us\n", NPv, n, nb, ms * 1e3);
    }
  }
  // check L^-1 A L^-T = I for matrix 0
  std::vector<double> Li((size_t)n * n);
  CK(hipMemcpy(Li.data(), dO, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0;
  for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) {
    double s = 0;
    for (int k = 0; k < n; ++k) for (int l = 0; l < n; ++l) s += Li[i + k * n] * h[k + l * n] * Li[j + l * n];
    err = fmax(err, fabs(s - (i == j)));
  }
  printf("  ||L^-1 A L^-T - I||_max = %.2e\n", err);
  size_t lds = sizeof(double) * ((size_t)n * n + 10 * n + 40);
  CK(hipFuncSetAttribute((const void*)eigmin_lds<double>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    eigmin_lds<double><<<nb, 512, lds>>>(ddin, dE);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("eigmin_lds n=%d batch=%d: %.1f us\n", n, nb, ms * 1e3);
  }
  double ev; CK(hipMemcpy(&ev, dE, 8, hipMemcpyDeviceToHost));
  std::vector<double> evl(nb), evr(nb);
  CK(hipMemcpy(evl.data(), dE, nb * 8, hipMemcpyDeviceToHost));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    eigmin_reg<0, 4><<<nb, 256>>>(ddin, dE);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("eigmin_reg<4 waves> n=%d batch=%d: %.1f us\n", n, nb, ms * 1e3);
  }
  {
    std::vector<double> ev4(nb);
    CK(hipMemcpy(ev4.data(), dE, nb * 8, hipMemcpyDeviceToHost));
    double dm = 0;
    for (int b = 0; b < nb; ++b) dm = fmax(dm, fabs(ev4[b] - evl[b]));
    printf("  max |eigmin_lds - eigmin_reg<4 waves>| = %.3e\n", dm);
  }
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    eigmin_reg<<<nb, 512>>>(ddin, dE);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("eigmin_reg n=%d batch=%d: %.1f us\n", n, nb, ms * 1e3);
  }
  {  // workgroup placement: the same launch with 100 KB of unused dynamic LDS (one per CU)
    const int pad = 100 * 1024;
    CK(hipFuncSetAttribute((const void*)eigmin_reg<0, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, pad + 16384));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      eigmin_reg<0, 8><<<nb, 512, pad>>>(ddin, dE);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      printf("eigmin_reg n=%d batch=%d, one workgroup per CU (LDS pad): %.1f us\n", n, nb, ms * 1e3);
    }
  }
  CK(hipMemcpy(evr.data(), dE, nb * 8, hipMemcpyDeviceToHost));
#ifdef CLRSDP_EIGREG_STAMPS
  {
    unsigned long long st[8];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_eigreg_stamps), sizeof(st)));
    const char* names[] = {"init", "matvec", "p sums+write", "barrier", "reads,Kc,x", "reflector+upd", "publish", "sturm"};
    for (int q = 0; q < 8; ++q) printf("  eigreg stamp %-12s %10.0f cycles per matrix\n", names[q], st[q] / (3.0 * nb));
  }
#endif
  for (int dbg : {1, 2, 3}) {
    CK(hipEventRecord(e0));
    for (int r = 0; r < 3; ++r) {
      if (dbg == 1) eigmin_reg<1, 4><<<nb, 256>>>(ddin, dE + nb);
      if (dbg == 2) eigmin_reg<2, 4><<<nb, 256>>>(ddin, dE + nb);
      if (dbg == 3) eigmin_reg<3, 4><<<nb, 256>>>(ddin, dE + nb);
    }
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("eigmin_reg<dbg %d (1 no update, 2 no matvec)>: %.1f us\n", dbg, ms * 1e3 / 3);
  }
  double dmax = 0;
  for (int b = 0; b < nb; ++b) dmax = fmax(dmax, fabs(evl[b] - evr[b]));
  printf("  max |eigmin_lds - eigmin_reg| over the batch = %.3e (lambda_min[0] = %.15f)\n", dmax, evr[0]);
#ifdef CLRSDP_EIG_STAMPS
  {
    unsigned long long st[8];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_eig_stamps), sizeof(st)));
    const char* names[] = {"A:reflector", "B:symv", "B:reduce", "C:w", "D:update", "tail", "sturm"};
    for (int i = 0; i < 7; ++i) printf("  stamp %-12s %10.0f cycles per matrix (all reps)\n", names[i], st[i] / (3.0 * nb));
  }
#endif
  // lambda_min by shifted power iteration on matrix 0
  std::vector<double> v(n, 1.0), w(n);
  double shift = 10.0, lam = 0;
  for (int it = 0; it < 20000; ++it) {
    double nv = 0;
    for (int i = 0; i < n; ++i) { double s = shift * v[i]; for (int k = 0; k < n; ++k) s -= h[i + k * n] * v[k]; w[i] = s; nv += s * s; }
    nv = sqrt(nv); lam = 0;
    for (int i = 0; i < n; ++i) { lam += w[i] * v[i]; v[i] = w[i] / nv; }
  }
  printf("  eigmin %.15f vs power-iteration %.15f\n", ev, shift - lam);
  return 0;
}
