// Cycles of one wave's 16x16 Cholesky + inverse (chol_diag16_bc, the chol_inv_tiles diagonal
// step) on a column-major 16 x 18 LDS tile.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;

template <int V>
__global__ __launch_bounds__(64) void probe(const double* __restrict__ S, double* __restrict__ out,
                                            unsigned long long* cyc, int reps) {
  __shared__ __attribute__((aligned(16))) double A[16 * 18];
  __shared__ __attribute__((aligned(16))) double Dinv[256];
  __shared__ int flag[4];
  const int lane = threadIdx.x;
  unsigned long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    for (int e = lane; e < 256; e += 64) A[(e >> 4) * 18 + (e & 15)] = S[e];
    if (lane == 0) flag[0] = 0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    chol_diag16_bc(A, [](int i, int j) { return j * 18 + i; }, 0, Dinv, flag, lane);
    __syncthreads();
    tot += __builtin_amdgcn_s_memtime() - t0;
  }
  for (int e = lane; e < 256; e += 64) {
    out[e] = A[(e >> 4) * 18 + (e & 15)];
    out[256 + e] = Dinv[e];
  }
  if (lane == 0) { cyc[0] = tot; cyc[1] = flag[0]; }
}

int main() {
  std::vector<double> S(256);
  srand(3);
  std::vector<double> G(256);
  for (auto& g : G) g = rand() / (double)RAND_MAX - 0.5;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = (i == j) ? 1.0 : 0.0;
      for (int k = 0; k < 16; ++k) s += G[i + 16 * k] * G[j + 16 * k];
      S[i + 16 * j] = s;
    }
  double *dS, *dO;
  unsigned long long* dc;
  hipMalloc(&dS, 256 * 8); hipMalloc(&dO, 512 * 8); hipMalloc(&dc, 16);
  hipMemcpy(dS, S.data(), 256 * 8, hipMemcpyHostToDevice);
  const int reps = 200;
  for (int v = 1; v < 2; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      probe<1><<<1, 64>>>(dS, dO, dc, reps);
      hipDeviceSynchronize();
    }
    unsigned long long c[2];
    std::vector<double> o(512);
    hipMemcpy(c, dc, 16, hipMemcpyDeviceToHost);
    hipMemcpy(o.data(), dO, 512 * 8, hipMemcpyDeviceToHost);
    // check Dinv * L = I and L L^T = S (lower triangles)
    double e1 = 0, e2 = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0, t = 0;
        for (int k = 0; k < 16; ++k) {
          const double Lik = k <= i ? o[i + 16 * k] : 0.0, Ljk = k <= j ? o[j + 16 * k] : 0.0;
          s += o[256 + i + 16 * k] * (j <= k ? o[k + 16 * j] : 0.0);
          t += Lik * Ljk;
        }
        e1 = fmax(e1, fabs(s - (i == j)));
        e2 = fmax(e2, fabs(t - S[i + 16 * j]));
      }
    printf("variant %d: %.0f cycles per 16x16 factor+inverse, |Dinv L - I| %.2e, |L L^T - S| %.2e, flag %llu\n",
           v, (double)c[0] / reps, e1, e2, c[1]);
  }
  return 0;
}
