// Latency of one wave's dependent fp64 + LDS round-trip chain (the chol_inv_mfma diagonal step).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_lds(double* out, unsigned long long* cyc, int iters) {
  __shared__ double buf[128];
  int lane = threadIdx.x;
  buf[lane] = 1.0 + lane * 1e-3;
  __syncthreads();
  double x = buf[lane];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    double p = buf[(it & 15)];          // broadcast read
    double r = __builtin_amdgcn_rsq(p);
    r = r * (1.5 - 0.5 * p * r * r);
    x = x * r + 1e-9;
    buf[64 + (lane & 15)] = x;          // write
    __builtin_amdgcn_wave_barrier();
    x += buf[64 + ((lane + 1) & 15)] * 1e-9;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = x;
  if (lane == 0) *cyc = t1 - t0;
}
__global__ void k_fma(double* out, unsigned long long* cyc, int iters) {
  double x = threadIdx.x * 1e-3, y = 1.0000001;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) x = fma(x, y, 1e-9);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k_realtime(unsigned long long* o) {
  unsigned long long a = __builtin_amdgcn_s_memtime(), b = __builtin_amdgcn_s_memrealtime();
  for (volatile int i = 0; i < 200000; ++i) {}
  unsigned long long c = __builtin_amdgcn_s_memtime(), d = __builtin_amdgcn_s_memrealtime();
  o[0] = c - a; o[1] = d - b;
}
int main() {
  double* out; unsigned long long* cyc;
  hipMalloc(&out, 1024); hipMalloc(&cyc, 64);
  unsigned long long h[2];
  k_realtime<<<1, 1>>>(cyc); hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
  printf("memtime ticks per 100MHz realtime tick: %.2f (=> memtime clock %.2f GHz)\n", (double)h[0] / h[1], (double)h[0] / h[1] / 10.0);
  int iters = 10000;
  k_fma<<<1, 64>>>(out, cyc, iters); hipDeviceSynchronize();
  k_fma<<<1, 64>>>(out, cyc, iters); hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
  printf("dependent v_fma_f64 chain: %.1f ticks/op\n", (double)h[0] / iters);
  k_lds<<<1, 64>>>(out, cyc, iters); hipDeviceSynchronize();
  k_lds<<<1, 64>>>(out, cyc, iters); hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
  printf("LDS read -> rsq/newton -> write -> read chain: %.1f ticks/iter\n", (double)h[0] / iters);
  return 0;
}
