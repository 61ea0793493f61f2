// Measured ceiling of the multi-word arithmetic the dd / qd kernels run on: multiply-adds
// acc += a * b (the inner operation of gemm_valu and of the Schur pairing at w > 1) with 4
// independent accumulators per thread, 1024 workgroups x 256 threads, no memory traffic in the
// loop.  Reported as multi-word multiply-adds per second and as fp64 VALU instructions per
// multiply-add (from the fp64 FMA peak measured the same way).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/mwfloat.h"
using namespace mw;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)
constexpr int ITERS = 256;
template <class T>
__global__ __launch_bounds__(256) void mad_loop(double* out, double seed) {
  T a(seed + threadIdx.x * 1e-7), b(1.0 - seed * 1e-3);
  T acc[4] = {T(0.1), T(0.2), T(0.3), T(0.4)};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = acc[k] + a * b;
    a = a * b;
  }
  T s = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (Num<T>::hi(s) == 12345.0) out[0] = Num<T>::hi(s);
}
template <>
__global__ __launch_bounds__(256) void mad_loop<double>(double* out, double seed) {
  double a = seed + threadIdx.x * 1e-7, b = 1.0 - seed * 1e-3;
  double acc[8] = {0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8};
  for (int i = 0; i < ITERS * 4; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = fma(a, b, acc[k]);
    a = fma(a, b, 1e-9);
  }
  double s = 0;
  for (int k = 0; k < 8; ++k) s += acc[k];
  if (s == 12345.0) out[0] = s;
}
template <class T>
double rate(int madd_per_iter) {
  double* out; CK(hipMalloc(&out, 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int G = 1024 * 8;
  mad_loop<T><<<G, 256>>>(out, 0.5); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) mad_loop<T><<<G, 256>>>(out, 0.5);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = 5.0 * G * 256.0 * (double)madd_per_iter;
  return ops / (ms * 1e-3);
}
struct Num_d {};
int main() {
  const double f64 = rate<double>(ITERS * 4 * 9);        // fma per second (8 acc + 1 chain)
  const double dd_r = rate<dd>(ITERS * 5);                // 4 acc + 1 chain multiply
  const double qd_r = rate<qd>(ITERS * 5);
  printf("fp64 FMA            : %8.3f T/s  (%.1f TFLOP/s)\n", f64 / 1e12, 2 * f64 / 1e12);
  printf("dd multiply-add     : %8.3f T/s  = %5.1f fp64 FMA-slots each\n", dd_r / 1e12, f64 / dd_r);
  printf("qd multiply-add     : %8.3f T/s  = %5.1f fp64 FMA-slots each\n", qd_r / 1e12, f64 / qd_r);
  return 0;
}
