// Per-wave timeline of chol_inv_tiles (s_memtime stamps, -DCLRSDP_CHOL_TRACE): where the panel
// loop spends its cycles, and L^-1 A L^-T = I per matrix.  Usage: chol_trace [n] [batch]
// (n <= 64: NP = 64, n <= 128: NP = 128, else NP = 256)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -DCLRSDP_CHOL_TRACE \
//     chol_trace.hip -o ../../microbin/chol_trace && ../../microbin/chol_trace 255 64
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

template <int NP>
void launch(unsigned nb, const MatDesc<double>* in, const MatDesc<double>* out, int* info) {
  CK(hipFuncSetAttribute((const void*)chol_inv_tiles<NP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                         (int)chol_inv_tiles_lds<NP>()));
  chol_inv_tiles<NP><<<nb, CholTiles<NP>::NTH, chol_inv_tiles_lds<NP>()>>>(in, out, info, 1);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 128, nb = argc > 2 ? atoi(argv[2]) : 128;
  const int NTH = n <= 128 ? 512 : CholTiles<256>::NTH, NW = NTH / 64;
  std::vector<double> h((size_t)nb * n * n);
  srand(1);
  for (int b = 0; b < nb; ++b) {
    std::vector<double> G((size_t)n * n);
    for (auto& g : G) g = (rand() / (double)RAND_MAX - 0.5);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = (i == j) ? 1.0 : 0.0;
        for (int k = 0; k < n; ++k) s += G[i + k * n] * G[j + k * n] / n;
        h[(size_t)b * n * n + i + j * n] = s;
        h[(size_t)b * n * n + j + i * n] = s;
      }
  }
  double *dA, *dO;
  CK(hipMalloc(&dA, h.size() * 8)); CK(hipMalloc(&dO, h.size() * 8));
  CK(hipMemcpy(dA, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  std::vector<MatDesc<double>> din(nb), dout(nb);
  for (int b = 0; b < nb; ++b) { din[b] = {dA + (size_t)b * n * n, n, n}; dout[b] = {dO + (size_t)b * n * n, n, n}; }
  MatDesc<double> *ddin, *ddout; int* info;
  CK(hipMalloc(&ddin, nb * sizeof(MatDesc<double>))); CK(hipMalloc(&ddout, nb * sizeof(MatDesc<double>)));
  CK(hipMalloc(&info, nb * 4));
  CK(hipMemcpy(ddin, din.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
  CK(hipMemcpy(ddout, dout.data(), nb * sizeof(MatDesc<double>), hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    if (n <= 64) launch<64>(nb, ddin, ddout, info);
    else if (n <= 128) launch<128>(nb, ddin, ddout, info);
    else launch<256>(nb, ddin, ddout, info);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("chol_inv_tiles n=%d batch=%d threads=%d: %.1f us\n", n, nb, NTH, ms * 1e3);
  }
  {
    std::vector<double> o2(h.size());
    CK(hipMemcpy(o2.data(), dO, h.size() * 8, hipMemcpyDeviceToHost));
    for (int b = 0; b < nb && b < 2; ++b) {
      double err = 0;
      const double* L = o2.data() + (size_t)b * n * n;
      const double* H = h.data() + (size_t)b * n * n;
      std::vector<double> T1((size_t)n * n, 0.0);
      for (int i = 0; i < n; ++i) for (int l = 0; l < n; ++l) { double s = 0; for (int k = 0; k < n; ++k) s += L[i + k * n] * H[k + l * n]; T1[i + l * n] = s; }
      for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) { double s = 0; for (int l = 0; l < n; ++l) s += T1[i + l * n] * L[j + l * n]; err = fmax(err, fabs(s - (i == j))); }
      printf("matrix %d: ||L^-1 A L^-T - I||_max = %.2e\n", b, err);
    }
  }
#ifdef CLRSDP_CHOL_TRACE
  std::vector<unsigned long long> tr(256 * 16 * 128);
  CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_chol2_trace), tr.size() * 8));
  // average over blocks of (stamp - block start of wave 0), per wave and point (memtime ticks)
  for (int w = 0; w < NW; ++w) {
    printf("wave %2d:", w);
    int np = 0;
    for (int p = 0; p < 128; ++p) if (tr[(0 * 16 + w) * 128 + p]) np = p + 1;
    for (int p = 0; p < np; ++p) {
      double s = 0;
      for (int b = 0; b < nb; ++b) s += (double)(tr[(b * 16 + w) * 128 + p] - tr[(b * 16 + 0) * 128 + 0]);
      printf(" %.0f", s / nb);
    }
    printf("\n");
  }
#endif
  std::vector<int> hi(nb);
  CK(hipMemcpy(hi.data(), info, nb * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int b = 0; b < nb; ++b) bad += hi[b] != 0;
  printf("failed pivots: %d\n", bad);
  return 0;
}
