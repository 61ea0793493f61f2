// Accuracy and latency of pivot_sqrt<qd> (s = sqrt(d), r = 1/sqrt(d)): max |s^2 - d| / d and
// max |s r - 1| over random quad-double d, and the clock of a dependent chain of pivots on one
// lane.  Build twice to compare with the three full quad-double Newton steps:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 qd_pivot.hip -o qd_pivot.bin
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCLRSDP_QD_PIVOT_FULL qd_pivot.hip -o qd_pivot_full.bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
using mw::qd;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

__global__ void resid(const qd* d, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  qd s, r;
  pivot_sqrt(d[i], s, r);
  const qd e1 = (s * s - d[i]) / d[i];
  const qd e2 = s * r - qd(1.0);
  out[2 * i] = fabs(e1.x[0]);
  out[2 * i + 1] = fabs(e2.x[0]);
}
__global__ void chain(const qd* d, qd* out, long long* clk, int reps) {
  qd x = d[threadIdx.x];
  const long long t0 = clock64();
  for (int k = 0; k < reps; ++k) {
    qd s, r;
    pivot_sqrt(x, s, r);
    x = s + r;  // keeps the value near [2, 3) and the steps dependent
  }
  const long long t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}

int main() {
  const int n = 1 << 16;
  std::vector<qd> h(n);
  srand(5);
  for (auto& v : h) {
    const double a = ldexp(1.0 + rand() / (double)RAND_MAX, rand() % 200 - 100);
    v = qd(a, a * 1e-17 * (rand() / (double)RAND_MAX - 0.5), a * 1e-34 * (rand() / (double)RAND_MAX - 0.5),
           a * 1e-51 * (rand() / (double)RAND_MAX - 0.5));
    v = v + qd(0.0);  // renormalise
  }
  qd *dd_, *dout;
  double* de;
  long long* clk;
  CK(hipMalloc(&dd_, n * sizeof(qd)));
  CK(hipMalloc(&dout, 64 * sizeof(qd)));
  CK(hipMalloc(&de, 2 * n * sizeof(double)));
  CK(hipMalloc(&clk, sizeof(long long)));
  CK(hipMemcpy(dd_, h.data(), n * sizeof(qd), hipMemcpyHostToDevice));
  resid<<<n / 256, 256>>>(dd_, de, n);
  std::vector<double> e(2 * n);
  CK(hipMemcpy(e.data(), de, e.size() * sizeof(double), hipMemcpyDeviceToHost));
  double m1 = 0, m2 = 0;
  for (int i = 0; i < n; ++i) { m1 = fmax(m1, e[2 * i]); m2 = fmax(m2, e[2 * i + 1]); }
  const int reps = 64;
  chain<<<1, 1>>>(dd_, dout, clk, reps);
  long long c;
  CK(hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost));
  printf("pivot_sqrt<qd>%s: max |s^2-d|/d %.2e, max |s r - 1| %.2e, %.0f cycles per dependent pivot\n",
#ifdef CLRSDP_QD_PIVOT_FULL
         " (three qd steps)",
#else
         "",
#endif
         m1, m2, (double)c / reps);
  return 0;
}
