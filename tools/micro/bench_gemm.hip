// Batched fp64 GEMM timing for the solver's shapes: gemm_f64_lds (NN/TN/NT, BK 32 and 16) on
// nb x (M x N x K), alpha=1, beta=0; workgroups tile-major as in the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

template <class K>
float timeit(K k, int reps = 20) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

__global__ void empty_kernel(const GemmDesc<double>* d, const int* t) {
  if (threadIdx.x == 999) ((double*)d)[0] = t[0];
}

int main(int argc, char** argv) {
  int M = argc > 1 ? atoi(argv[1]) : 128, N = argc > 2 ? atoi(argv[2]) : 128, K = argc > 3 ? atoi(argv[3]) : 128;
  int nb = argc > 4 ? atoi(argv[4]) : 64;
  size_t sa = (size_t)M * K, sb = (size_t)K * N, sc = (size_t)M * N;
  double *A, *B, *C;
  CK(hipMalloc(&A, sa * nb * 8)); CK(hipMalloc(&B, sb * nb * 8)); CK(hipMalloc(&C, sc * nb * 8));
  std::vector<double> h(std::max(sa, sb) * nb);
  for (auto& x : h) x = rand() / (double)RAND_MAX - 0.5;
  CK(hipMemcpy(A, h.data(), sa * nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), sb * nb * 8, hipMemcpyHostToDevice));
  double flops = 2.0 * M * N * K * nb;
  {
    float us = timeit([&] { empty_kernel<<<1024, 256>>>(nullptr, nullptr); });
    printf("empty kernel 1024x256: %.2f us\n", us);
  }
  for (int variant : {5, 7, 8, 10, 11, 12, 13, 14}) {
    const int TILE = 64;
    std::vector<GemmDesc<double>> d;
    std::vector<TileRef> t2d;
    for (int b = 0; b < nb; ++b) {
      // lda/ldb as each variant reads them: TA -> A is K x M (ld K), TB -> B is N x K (ld N)
      const bool ta = variant == 3 || variant == 6 || variant == 9, tb = variant == 4 || variant == 7 || variant == 10 || variant == 12 || variant == 14;
      GemmDesc<double> g{A + sa * b, B + sb * b, nullptr, C + sc * b, M, N, K, ta ? K : M, tb ? N : K, M, M, (N + TILE - 1) / TILE, 0, 0};
      d.push_back(g);
    }
    const int nt = ((M + TILE - 1) / TILE) * d[0].tn;
    for (int t = 0; t < nt; ++t)
      for (int b = 0; b < nb; ++b) t2d.push_back(TileRef{b, t});
    GemmDesc<double>* dd; TileRef* dt;
    CK(hipMalloc(&dd, d.size() * sizeof(d[0]))); CK(hipMalloc(&dt, t2d.size() * sizeof(TileRef)));
    CK(hipMemcpy(dd, d.data(), d.size() * sizeof(d[0]), hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, t2d.data(), t2d.size() * sizeof(TileRef), hipMemcpyHostToDevice));
    unsigned grid = t2d.size();
    float us;
    if (variant == 2) us = timeit([&] { gemm_f64_lds<false, false><<<grid, 256>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 3) us = timeit([&] { gemm_f64_lds<true, false><<<grid, 256>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 4) us = timeit([&] { gemm_f64_lds<false, true><<<grid, 256>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 5) us = timeit([&] { gemm_f64_lds<false, false, 0, 16><<<grid, 256>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 6) us = timeit([&] { gemm_f64_lds<true, false, 0, 16><<<grid, 256>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 7) us = timeit([&] { gemm_f64_lds<false, true, 0, 16><<<grid, 256>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 8) us = timeit([&] { gemm_f64_lds<false, false, 0, 16, 8><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 9) us = timeit([&] { gemm_f64_lds<true, false, 0, 16, 8><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 10) us = timeit([&] { gemm_f64_lds<false, true, 0, 16, 8><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 11) us = timeit([&] { gemm_f64_lds<false, false, 0, 32, 8><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 12) us = timeit([&] { gemm_f64_lds<false, true, 0, 32, 8><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    else if (variant == 13) us = timeit([&] { gemm_f64_lds<false, false, 0, 64, 8><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    else us = timeit([&] { gemm_f64_lds<false, true, 0, 64, 8><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
    const char* nm[] = {"", "", "lds NN       ", "lds TN       ", "lds NT       ", "lds16 NN     ", "lds16 TN     ", "lds16 NT     ", "lds16w8 NN   ", "lds16w8 TN   ", "lds16w8 NT   ", "lds32w8 NN   ", "lds32w8 NT   ", "lds64w8 NN   ", "lds64w8 NT   "};
    printf("%s  batch %d x (%d x %d x %d): %.1f us  %.1f TFLOP/s  (grid %u)\n", nm[variant], nb, M, N, K, us, flops / us / 1e6, grid);
  }
  return 0;
}
