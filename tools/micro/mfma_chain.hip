// fp64 MFMA issue rate against the number of independent accumulator chains per wave and the
// number of waves per SIMD (256-thread workgroups, one wave per SIMD per workgroup; the grid is
// 256 x waves-per-SIMD workgroups).  Answers: how many chains does 16x16x4f64 need to reach peak?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

template <int CH>
__global__ __launch_bounds__(256) void chain(double* out, int iters, double s) {
  double a = threadIdx.x * 1e-3 + s, b = 1.0 - threadIdx.x * 1e-4;
  d4 c[CH];
#pragma unroll
  for (int q = 0; q < CH; ++q) c[q] = d4{0, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int q = 0; q < CH; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[q], 0, 0, 0);
  }
  double t = 0;
#pragma unroll
  for (int q = 0; q < CH; ++q) t += c[q][q & 3];
  if (t == 12345.678) out[threadIdx.x] = t;
}

template <int CH>
void run(double* dout, int wps) {
  const int nblk = 256 * wps, iters = 8192 / CH;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    chain<CH><<<nblk, 256>>>(dout, iters, 0.5);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double flops = (double)nblk * 4 * iters * CH * 2048.0;
  printf("chains/wave %d, waves/SIMD %d: %.2f TFLOP/s\n", CH, wps, flops / best / 1e9);
}

int main() {
  double* dout;
  CK(hipMalloc(&dout, 1 << 20));
  for (int wps : {1, 2, 4}) {
    run<1>(dout, wps);
    run<2>(dout, wps);
    run<4>(dout, wps);
    run<8>(dout, wps);
  }
  return 0;
}
