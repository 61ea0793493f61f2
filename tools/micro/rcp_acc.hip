// Accuracy of v_rcp_f64 / v_rsq_f64 (in ulps) and latency of independent vs dependent fp64 chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__global__ void k(const double* x, double* r, double* q, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { r[i] = __builtin_amdgcn_rcp(x[i]); q[i] = __builtin_amdgcn_rsq(x[i]); }
}
__global__ void k_ilp(double* out, unsigned long long* cyc, int iters) {
  double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 1.0000001;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) { x0 = fma(x0, y, 1e-9); x1 = fma(x1, y, 1e-9); x2 = fma(x2, y, 1e-9); x3 = fma(x3, y, 1e-9); }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x0 + x1 + x2 + x3;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k_f32(float* out, unsigned long long* cyc, int iters) {
  float x = threadIdx.x * 1e-3f, y = 1.0000001f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) x = fmaf(x, y, 1e-9f);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  const int n = 1 << 20;
  double *x, *r, *q; hipMalloc(&x, n * 8); hipMalloc(&r, n * 8); hipMalloc(&q, n * 8);
  double* h = new double[n]; double* hr = new double[n]; double* hq = new double[n];
  for (int i = 0; i < n; ++i) h[i] = exp(((double)rand() / RAND_MAX - 0.5) * 40.0);
  hipMemcpy(x, h, n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(x, r, q, n);
  hipMemcpy(hr, r, n * 8, hipMemcpyDeviceToHost); hipMemcpy(hq, q, n * 8, hipMemcpyDeviceToHost);
  double mr = 0, mq = 0;
  for (int i = 0; i < n; ++i) {
    double er = fabs(hr[i] - 1.0 / h[i]) / (fabs(1.0 / h[i]) * 2.220446049250313e-16);
    double eq = fabs(hq[i] - 1.0 / sqrt(h[i])) / (fabs(1.0 / sqrt(h[i])) * 2.220446049250313e-16);
    mr = fmax(mr, er); mq = fmax(mq, eq);
  }
  printf("v_rcp_f64 max err %.3g ulp, v_rsq_f64 max err %.3g ulp\n", mr, mq);
  unsigned long long* cyc; hipMalloc(&cyc, 8); unsigned long long c;
  int it = 10000;
  k_ilp<<<1, 64>>>(r, cyc, it); k_ilp<<<1, 64>>>(r, cyc, it); hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("4 independent fp64 fma chains: %.1f ticks per iteration (4 fmas)\n", (double)c / it);
  k_f32<<<1, 64>>>((float*)r, cyc, it); k_f32<<<1, 64>>>((float*)r, cyc, it); hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("dependent fp32 fma chain: %.1f ticks/op\n", (double)c / it);
  return 0;
}
