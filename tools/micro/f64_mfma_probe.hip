// Microbenchmark + layout probe for fp64 matrix cores on gfx950.
// (1) checks the lane->element map of v_mfma_f64_16x16x4_f64 with exact integer data;
// (2) measures back-to-back MFMA f64 throughput and v_fma_f64 VALU throughput chip-wide.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

__global__ void layout_probe(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];   // A[i][k], i=l&15, k=l>>4 (row-major 16x4)
  double b = B[(l >> 4) * 16 + (l & 15)];  // B[k][j], k=l>>4, j=l&15 (row-major 4x16)
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

__global__ __launch_bounds__(256) void mfma_tput(double* out, int iters, double s) {
  double a = threadIdx.x * 1e-3 + s, b = 1.0 - threadIdx.x * 1e-4;
  d4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  double t = c0[0] + c1[1] + c2[2] + c3[3];
  if (t == 12345.678) out[threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void valu_tput(double* out, int iters, double s) {
  double x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3 + k + s;
  double m = 0.999999, a = 1e-7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = fma(x[k], m, a);
  }
  double t = 0; for (int k = 0; k < 8; ++k) t += x[k];
  if (t == 12345.678) out[threadIdx.x] = t;
}

int main(int argc, char** argv) {
  // layout
  std::vector<double> A(64), B(64), D(256);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i * 4 + k] = i * 7 + k * 3 + 1;
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = (k + 1) * (j + 2) - 3 * j + k;
  double *dA, *dB, *dD; CK(hipMalloc(&dA, 512)); CK(hipMalloc(&dB, 512)); CK(hipMalloc(&dD, 2048));
  CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
  layout_probe<<<1, 64>>>(dA, dB, dD); CK(hipDeviceSynchronize());
  CK(hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost));
  double ref[16][16];
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { double s = 0; for (int k = 0; k < 4; ++k) s += A[i*4+k]*B[k*16+j]; ref[i][j] = s; }
  // test candidate maps
  int okA = 1, okB = 1;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int col = l & 15;
    int rowA = (l >> 4) + 4 * r;      // guide's f64 map
    int rowB = (l >> 4) * 4 + r;      // f32 map
    if (D[l*4+r] != ref[rowA][col]) okA = 0;
    if (D[l*4+r] != ref[rowB][col]) okB = 0;
  }
  printf("layout: map row=(l>>4)+4r : %s ; map row=(l>>4)*4+r : %s\n", okA ? "OK" : "no", okB ? "OK" : "no");
  // throughput
  double* dout; CK(hipMalloc(&dout, 1 << 20));
  int nblk = argc > 1 ? atoi(argv[1]) : 256 * 8, iters = 4096;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(e0)); mfma_tput<<<nblk, 256>>>(dout, iters, 0.5); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nblk * 4 /*waves*/ * iters * 4 * 2048.0;
    printf("mfma_f64_16x16x4: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
    CK(hipEventRecord(e0)); valu_tput<<<nblk, 256>>>(dout, iters, 0.5); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    flops = (double)nblk * 256 * iters * 8 * 2.0;
    printf("v_fma_f64: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  return 0;
}
