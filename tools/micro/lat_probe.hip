// Latency probe for the building blocks of the per-column loops of the on-chip factorisation
// and eigen kernels: workgroup barrier, LDS round trip, DPP wave sum, fp64 sqrt/div chains.
// Prints cycles (s_memtime) per loop iteration, averaged over the workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); return 1;} }while(0)

template <int MODE>
__global__ void probe(double* out, unsigned long long* cyc, int iters) {
  __shared__ double buf[1024];
  const int tid = threadIdx.x;
  double x = tid * 1e-3 + 1.0;
  buf[tid & 1023] = x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {          // barrier only
      __syncthreads();
    } else if (MODE == 1) {   // LDS write -> barrier -> LDS read (dependent)
      buf[tid & 1023] = x;
      __syncthreads();
      x = buf[(tid + 64) & 1023] * 0.5 + 0.5;
    } else if (MODE == 2) {   // DPP wave sum (dependent chain)
      x = wave_sum_dpp(x) * 1e-3;
    } else if (MODE == 3) {   // shfl wave sum
      x = wave_sum(x) * 1e-3;
    } else if (MODE == 4) {   // sqrt + div chain
      x = 2.0 / (sqrt(x) + 1.0) + 0.5;
    } else if (MODE == 5) {   // dependent fp64 fma chain of 16
#pragma unroll
      for (int q = 0; q < 16; ++q) x = fma(x, 0.999, 1e-3);
    } else if (MODE == 6) {   // LDS read dependent chain (no barrier)
      x = buf[((int)x + tid) & 1023];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + tid] = x;
  if (tid == 0) atomicAdd(cyc, t1 - t0);
}

template <int MODE>
int run(const char* name, int threads, int blocks) {
  double* o; unsigned long long* c;
  CK(hipMalloc(&o, 1024 * 1024 * 8)); CK(hipMalloc(&c, 8));
  CK(hipMemset(c, 0, 8));
  const int iters = 2000;
  probe<MODE><<<blocks, threads>>>(o, c, iters);
  CK(hipDeviceSynchronize());
  CK(hipMemset(c, 0, 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  probe<MODE><<<blocks, threads>>>(o, c, iters);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h; CK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
  printf("%-28s threads %4d blocks %4d: %8.1f cycles/iter  %8.2f ns/iter (event)\n", name, threads, blocks, (double)h / blocks / iters, ms * 1e6 / iters);
  CK(hipFree(o)); CK(hipFree(c));
  return 0;
}


// the 16x16 Cholesky + inverse of chol_inv_mfma's diagonal phase, one wave, in a loop
template <int VAR>
__global__ void diag16(double* out, unsigned long long* cyc, int iters) {
  const int lane = threadIdx.x & 63, i = lane & 15, grp = lane >> 4;
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) v[c] = grp == 0 ? (c < i ? 0.01 * (c + 1) : (c == i ? 4.0 : 0.0)) : (c == i ? 1.0 : 0.0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double djj = VAR == 1 ? 4.0 + v[j] * 1e-30 : readlane_d(v[j], j);
      double r;
      if (VAR == 2) r = 0.5 + djj * 1e-30;
      else { r = __builtin_amdgcn_rsq(djj); r = r * (1.5 - 0.5 * djj * r * r); }
      const double lij = (i == j) ? djj * r : v[j] * r;
      const double lsw = VAR == 3 ? lij : swap16_d(lij);
      double xj[16];
#pragma unroll
      for (int c = 0; c <= j; ++c) xj[c] = VAR == 4 ? v[c] : readlane_d(v[c], 16 + j);
      double lk[16];
#pragma unroll
      for (int t = j + 1; t < 16; ++t) lk[t] = VAR == 4 ? lij : readlane_d(lij, t);
      const bool g0 = grp == 0, below = i > j;
      const double m = lsw * r;
      v[j] = (g0 && i >= j) ? lij : v[j];
#pragma unroll
      for (int t = j + 1; t < 16; ++t) {
        const double u = v[t] - lij * lk[t];
        v[t] = (g0 && below && t <= i) ? u : v[t];
      }
#pragma unroll
      for (int c = 0; c <= j; ++c) {
        const double ux = (i == j) ? v[c] * r : v[c] - m * xj[c];
        v[c] = (!g0 && i >= j) ? ux : v[c];
      }
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = v[c] * 1e-3 + (c == i ? 4.0 : 0.0);  // keep it finite
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double acc = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) acc += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
}
template <int VAR>
int run_diag(const char* name) {
  double* o; unsigned long long* c;
  CK(hipMalloc(&o, 1024 * 1024 * 8)); CK(hipMalloc(&c, 8));
  CK(hipMemset(c, 0, 8));
  const int iters = 200;
  diag16<VAR><<<128, 64>>>(o, c, iters);
  CK(hipDeviceSynchronize());
  unsigned long long h; CK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
  printf("diag16 %-28s %8.1f cycles per 16-column factorisation\n", name, (double)h / 128 / iters);
  CK(hipFree(o)); CK(hipFree(c));
  return 0;
}

// launch cost of a 512-thread workgroup with a large dynamic LDS allocation
__global__ __launch_bounds__(512) void big_lds_kernel(double* out) {
  extern __shared__ double dyn[];
  dyn[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = dyn[5];
}
int run_biglds(size_t lds, int blocks) {
  double* o; CK(hipMalloc(&o, 4096 * 8));
  CK(hipFuncSetAttribute((const void*)big_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  big_lds_kernel<<<blocks, 512, lds>>>(o);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < 20; ++r) big_lds_kernel<<<blocks, 512, lds>>>(o);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("512-thread kernel, %6zu B dynamic LDS, %4d blocks: %.2f us per launch\n", lds, blocks, ms * 1e3 / 20);
  CK(hipFree(o));
  return 0;
}

int main() {
  for (int th : {64, 256, 512, 1024}) {
    run<0>("barrier", th, 128);
    run<1>("lds write+barrier+read", th, 128);
  }
  run<2>("dpp wave sum (6 steps)", 512, 128);
  run<3>("shfl wave sum (6 steps)", 512, 128);
  run<4>("sqrt+div", 512, 128);
  run<5>("16 dependent fp64 fma", 512, 128);
  run<5>("16 dependent fp64 fma", 64, 128);
  run<6>("dependent LDS read", 512, 128);
  run<6>("dependent LDS read", 64, 128);
  run_biglds(1024, 128);
  run_biglds(150 * 1024, 128);
  run_biglds(150 * 1024, 1);
  run_diag<0>("full");
  run_diag<1>("no pivot readlane");
  run_diag<2>("no rsq");
  run_diag<3>("no permlane swap");
  run_diag<4>("no row/col readlanes");
  return 0;
}
