// Two-stage eigen reduction, stage 1's serial chain (round 6): the panel
// QR factorisations of dense -> band (b = 16) for a batch of symmetric fp64 blocks of n = 128,
// the part of the blocked Householder reduction that cannot go to MFMA.  One wave per block
// holds the current panel (rows (k+1) b .. n-1 of columns k b .. k b + 15; lane l has rows l and
// l + 64) in registers and runs the 16 reflectors of each of the 7 panels with no barrier: per
// column a DPP wave sum for the norm, the pivot's square root and reciprocal, the 15 dot
// products v^T P[:, j] (DPP wave sums, independent) and the rank-1 update.  The trailing
// two-sided updates (MFMA) and stage 2 (band -> tridiagonal) would come on top.
// Prints the cycles per reflector (shader clock) and the time per batch, against the current
// one-stage eigmin_split (~0.8 us per column, 137 us per batch of 128 blocks of 128).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 eig_band_bench.hip -o ../../microbin/eig_band_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

constexpr int N = 128, B = 16;

__global__ __launch_bounds__(64) void band_panels(const double* A, double* out, unsigned long long* cyc) {
  const int blk = blockIdx.x, l = threadIdx.x;
  const double* a = A + (size_t)blk * N * N;
  unsigned long long t_all = 0;
  double keep = 0.0;
  for (int k = 0; k + 1 < N / B; ++k) {
    const int r0 = (k + 1) * B, m = N - r0, c0 = k * B;
    double p[2][B];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const int r = l + 64 * h;
        p[h][j] = r < m ? a[(r0 + r) + (size_t)(c0 + j) * N] : 0.0;
      }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int c = 0; c < B; ++c) {
      // x = column c, rows >= c of the panel
      double x0 = l >= c ? p[0][c] : 0.0, x1 = p[1][c];
      const double nrm2 = wave_sum_dpp(x0 * x0 + x1 * x1);
      const double xc = __shfl(p[0][c], c);
      const double nrm = sqrt(nrm2);
      const double alpha = xc >= 0.0 ? -nrm : nrm;
      const double denom = xc - alpha;
      const double rd = denom != 0.0 ? 1.0 / denom : 0.0;
      const double tau = nrm != 0.0 ? (alpha - xc) / alpha : 0.0;
      double v0 = l > c ? x0 * rd : (l == c ? 1.0 : 0.0), v1 = x1 * rd;
      // w_j = v^T P[:, j], j > c (independent DPP sums), then P[:, j] -= tau v w_j
      double w[B];
#pragma unroll
      for (int j = c + 1; j < B; ++j) w[j] = wave_sum_dpp(v0 * p[0][j] + v1 * p[1][j]);
#pragma unroll
      for (int j = c + 1; j < B; ++j) {
        p[0][j] -= tau * v0 * w[j];
        p[1][j] -= tau * v1 * w[j];
      }
      p[0][c] = l == c ? alpha : (l > c ? v0 : p[0][c]);
      p[1][c] = v1;
    }
    t_all += __builtin_amdgcn_s_memtime() - t0;
#pragma unroll
    for (int j = 0; j < B; ++j) keep += p[0][j] + p[1][j];
  }
  out[blk * 64 + l] = keep;
  if (l == 0) cyc[blk] = t_all;
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 16;
  std::vector<double> h((size_t)nb * N * N);
  srand(5);
  for (int b = 0; b < nb; ++b)
    for (int i = 0; i < N; ++i)
      for (int j = 0; j <= i; ++j) {
        const double v = (double)rand() / RAND_MAX - 0.5;
        h[(size_t)b * N * N + i + (size_t)j * N] = h[(size_t)b * N * N + j + (size_t)i * N] = v;
      }
  double *dA, *dO;
  unsigned long long* dc;
  CK(hipMalloc(&dA, h.size() * 8));
  CK(hipMalloc(&dO, (size_t)nb * 64 * 8));
  CK(hipMalloc(&dc, nb * 8));
  CK(hipMemcpy(dA, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  band_panels<<<nb, 64>>>(dA, dO, dc);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    float ms;
    CK(hipEventRecord(e0));
    band_panels<<<nb, 64>>>(dA, dO, dc);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = fminf(best, ms * 1e3f);
  }
  std::vector<unsigned long long> c(nb);
  CK(hipMemcpy(c.data(), dc, nb * 8, hipMemcpyDeviceToHost));
  double avg = 0;
  for (auto v : c) avg += (double)v;
  avg /= nb;
  const int refl = (N / B - 1) * B;
  printf("stage-1 panel chain, %d blocks of %d, b = %d: %d reflectors per block, %.0f cycles per reflector, %.1f us per batch (panel QRs only; no trailing update, no stage 2)\n",
         nb, N, B, refl, avg / refl, best);
  return 0;
}
