// Batched fp64 GEMM, nb x (M x N x K) NN, alpha = 1, beta = 0: the descriptor kernel
// gemm_f64_lds against the uniform-batch kernel gemm_f64_uni (batch in the kernel arguments),
// single- and double-buffered, BK 32 and 64.  Back-to-back launches, averaged.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form bench_gemm_uni.hip -o bin/bench_gemm_uni
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

template <class K>
float timeit(K k, int reps = 50) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const int M = 128, N = 128, K = 128;
  for (int nb : {64, 8}) {
    const size_t sa = (size_t)M * K, sb = (size_t)K * N, sc = (size_t)M * N;
    double *A, *B, *C;
    CK(hipMalloc(&A, sa * nb * 8)); CK(hipMalloc(&B, sb * nb * 8)); CK(hipMalloc(&C, sc * nb * 8));
    std::vector<double> h(sa * nb);
    for (auto& x : h) x = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(A, h.data(), sa * nb * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data(), sb * nb * 8, hipMemcpyHostToDevice));
    const double flops = 2.0 * M * N * K * nb;
    std::vector<GemmDesc<double>> d;
    std::vector<TileRef> t2d;
    for (int b = 0; b < nb; ++b) {
      GemmDesc<double> g{};
      g.A = A + sa * b; g.B = B + sb * b; g.Cin = nullptr; g.C = C + sc * b;
      g.M = M; g.N = N; g.K = K; g.lda = M; g.ldb = K; g.ldcin = M; g.ldc = M; g.tn = 2;
      d.push_back(g);
    }
    for (int t = 0; t < 4; ++t)
      for (int b = 0; b < nb; ++b) t2d.push_back(TileRef{b, t});
    GemmDesc<double>* dd; TileRef* dt;
    CK(hipMalloc(&dd, d.size() * sizeof(d[0]))); CK(hipMalloc(&dt, t2d.size() * sizeof(TileRef)));
    CK(hipMemcpy(dd, d.data(), d.size() * sizeof(d[0]), hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, t2d.data(), t2d.size() * sizeof(TileRef), hipMemcpyHostToDevice));
    UniGemm u{};
    u.A = A; u.B = B; u.C = C; u.sA = sa; u.sB = sb; u.sC = sc;
    u.M = M; u.N = N; u.K = K; u.lda = M; u.ldb = K; u.ldc = M; u.ldcin = M; u.tn = 2; u.P = nb; u.tsym = 3;
    const unsigned grid = 4 * nb;
    const float t0 = timeit([&] { gemm_f64_lds<false, false><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    const float t1 = timeit([&] { gemm_f64_uni<false, false, 0, 32, 8, false, false, false><<<grid, 512>>>(u, 1.0, 0.0); });
    const float t2 = timeit([&] { gemm_f64_uni<false, false, 0, 32, 8, false, false, true><<<grid, 512>>>(u, 1.0, 0.0); });
    const float t3 = timeit([&] { gemm_f64_uni<false, false, 0, 64, 8, false, false, true><<<grid, 512>>>(u, 1.0, 0.0); });
    printf("batch %d x 128^3 NN: lds %.2f us (%.1f TF) | uni %.2f us (%.1f TF) | uni+DB %.2f us (%.1f TF) | uni+DB BK64 %.2f us (%.1f TF)\n",
           nb, t0, flops / t0 / 1e6, t1, flops / t1 / 1e6, t2, flops / t2 / 1e6, t3, flops / t3 / 1e6);
  }
  return 0;
}
