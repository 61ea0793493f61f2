// Issue rate of v_fmac_f64_dpp (row_newbcast) against v_fmac_f64: 8 waves per workgroup, 32
// independent accumulators per lane, timed with s_memtime inside the kernel (cycles per
// instruction per SIMD = elapsed / (instructions per wave * waves per SIMD)).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;

template <int MODE>
__global__ __launch_bounds__(512) void probe(double* out, unsigned long long* cyc, int iters) {
  double acc[32];
  const double src = threadIdx.x * 1e-3, mul = 1.0 + threadIdx.x * 1e-9;
#pragma unroll
  for (int q = 0; q < 32; ++q) acc[q] = q;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int q = 0; q < 32; ++q) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(acc[q]) : "v"(src), "v"(mul));
    } else {
      static_for<0, 32>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        fmac_bcast<q & 15, false>(acc[q], src, mul);
      });
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int q = 0; q < 32; ++q) s += acc[q];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 256 * 512 * 8);
  (void)hipMalloc(&cyc, 256 * 8);
  const int iters = 1000;
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      if (mode == 0) probe<0><<<128, 512>>>(out, cyc, iters);
      else probe<1><<<128, 512>>>(out, cyc, iters);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c;
      (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      const double instr = 32.0 * iters;  // per wave
      printf("%s: %.1f us, memtime %llu ticks, %.2f ns per instruction per wave (2 waves per SIMD)\n",
             mode == 0 ? "v_fmac_f64       " : "v_fmac_f64_dpp bc", ms * 1e3, c,
             ms * 1e6 / instr);
    }
  }
  return 0;
}
