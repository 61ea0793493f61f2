// The 16x16 diagonal-tile Cholesky + inverse of chol_inv_tiles (chol_diag16_bc) in isolation:
// cycles per tile on one wave, alone or next to MFMA-busy waves (the workers of the real
// kernel), and the software-pipelined variant chol_diag16_pipe (the bulk updates of column j-1
// issued inside column j's pivot chain; inverse rows split over the four DPP rows), which must
// agree bit for bit.  Usage: diag16_bench [busy_mask] [mode] [blocks] [prio]
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form \
//     diag16_bench.hip -o ../../microbin/diag16_bench && ../../microbin/diag16_bench 254 0 128
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

constexpr int LDD = 18, REP = 64;

template <int V>
__global__ __launch_bounds__(512) void diag_bench(const double* __restrict__ Ain, double* __restrict__ Lout,
                                                  double* __restrict__ Xout, unsigned long long* cyc,
                                                  int busy, int mode, int prio) {
  __shared__ double T[16 * LDD], Di[256];
  __shared__ int flag[2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const double* a = Ain + blockIdx.x * 256;
  if (tid == 0) flag[0] = flag[1] = 0;
  __syncthreads();
  if (prio && w == 0) __builtin_amdgcn_s_setprio(3);
  if (w == 0) {
    unsigned long long tot = 0;
    for (int rep = 0; rep < REP; ++rep) {
      for (int e = lane; e < 256; e += 64) T[(e >> 4) * LDD + (e & 15)] = a[e];  // column-major
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      if constexpr (V == 0) chol_diag16_bc(T, [](int i, int j) { return j * LDD + i; }, 0, Di, flag, lane);
      else chol_diag16_pipe(T, [](int i, int j) { return j * LDD + i; }, 0, Di, flag, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      tot += t1 - t0;
    }
    if (lane == 0) {
      cyc[blockIdx.x] = tot;
      __hip_atomic_store(flag + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    for (int e = lane; e < 256; e += 64) {
      const int r = e & 15, c = e >> 4;
      Lout[blockIdx.x * 256 + e] = r >= c ? T[c * LDD + r] : 0.0;
      Xout[blockIdx.x * 256 + e] = Di[e];
    }
  } else if ((busy >> w) & 1) {
    d4 acc = {0.0, 0.0, 0.0, 0.0}, acc2 = acc;
    double f = 1e-3 * lane, v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = q;
    while (__hip_atomic_load(flag + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
      if (mode == 0) {  // dependent f64 MFMA chain
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = mfma64(f, f, acc);
      } else if (mode == 1) {  // two independent f64 MFMA chains
#pragma unroll
        for (int q = 0; q < 4; ++q) { acc = mfma64(f, f, acc); acc2 = mfma64(f, f, acc2); }
      } else {  // f64 VALU FMAs
#pragma unroll
        for (int q = 0; q < 8; ++q) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(v[q]) : "v"(f), "v"(f));
      }
    }
    if (acc[0] + acc2[0] + v[0] + v[7] == 12345.0) Xout[0] = acc[1];
  }
}

int main(int argc, char** argv) {
  // busy: bit mask of the waves (1-7) that load the CU next to the chain wave; mode 0: a
  // dependent f64 MFMA chain, 1: two MFMA chains, 2: f64 VALU FMAs
  const int busy = argc > 1 ? atoi(argv[1]) : 0, mode = argc > 2 ? atoi(argv[2]) : 0,
            nb = argc > 3 ? atoi(argv[3]) : 128, prio = argc > 4 ? atoi(argv[4]) : 0;
  std::vector<double> h((size_t)nb * 256);
  srand(3);
  for (int b = 0; b < nb; ++b) {
    double G[256];
    for (auto& g : G) g = rand() / (double)RAND_MAX - 0.5;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = i == j ? 0.5 : 0.0;
        for (int k = 0; k < 16; ++k) s += G[i + 16 * k] * G[j + 16 * k];
        h[(size_t)b * 256 + i + 16 * j] = s;
      }
  }
  double *dA, *L0, *X0, *L1, *X1;
  unsigned long long* cyc;
  CK(hipMalloc(&dA, h.size() * 8));
  CK(hipMalloc(&L0, h.size() * 8)); CK(hipMalloc(&X0, h.size() * 8));
  CK(hipMalloc(&L1, h.size() * 8)); CK(hipMalloc(&X1, h.size() * 8));
  CK(hipMalloc(&cyc, nb * 8));
  CK(hipMemcpy(dA, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  std::vector<double> hl[2], hx[2];
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      if (v == 0) diag_bench<0><<<nb, 512>>>(dA, L0, X0, cyc, busy, mode, prio);
      else diag_bench<1><<<nb, 512>>>(dA, L1, X1, cyc, busy, mode, prio);
      CK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> c(nb);
    CK(hipMemcpy(c.data(), cyc, nb * 8, hipMemcpyDeviceToHost));
    double s = 0;
    for (auto x : c) s += x;
    printf("%-18s busy mask 0x%02x mode %d prio %d: %.0f memtime ticks per tile\n",
           v == 0 ? "chol_diag16_bc" : "chol_diag16_pipe", busy, mode, prio, s / nb / REP);
    hl[v].resize(h.size()); hx[v].resize(h.size());
    CK(hipMemcpy(hl[v].data(), v ? L1 : L0, h.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hx[v].data(), v ? X1 : X0, h.size() * 8, hipMemcpyDeviceToHost));
  }
  // L L^T = A and X L = I for the reference variant; the pipelined one bit for bit
  double e1 = 0, e2 = 0;
  for (int b = 0; b < nb; ++b) {
    const double* L = hl[0].data() + b * 256, *X = hx[0].data() + b * 256, *A = h.data() + b * 256;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0, t = 0;
        for (int k = 0; k < 16; ++k) { s += L[i + 16 * k] * L[j + 16 * k]; t += X[i + 16 * k] * L[k + 16 * j]; }
        e1 = fmax(e1, fabs(s - A[i + 16 * j]));
        e2 = fmax(e2, fabs(t - (i == j)));
      }
  }
  const bool same = !memcmp(hl[0].data(), hl[1].data(), h.size() * 8) && !memcmp(hx[0].data(), hx[1].data(), h.size() * 8);
  double dmax = 0;
  for (size_t e = 0; e < h.size(); ++e) dmax = fmax(dmax, fmax(fabs(hl[0][e] - hl[1][e]), fabs(hx[0][e] - hx[1][e])));
  printf("max|LL^T - A| %.2e  max|XL - I| %.2e  pipe %s (max diff %.2e)\n", e1, e2,
         same ? "bitwise equal" : "DIFFERS", dmax);
  return 0;
}
