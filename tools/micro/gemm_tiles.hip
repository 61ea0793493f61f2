// Batched fp64 NN GEMM (nb x 128^3): output-tile shape against per-CU latency.  Each wave computes
// 32 x 16 with two v_mfma_f64_16x16x4f64 accumulators; a workgroup is WM x WN waves, so its tile is
// (32 WM) x (16 WN).  64 x 64 (2 x 4 waves) is the production shape: at a batch of 64 it is one
// workgroup per CU and nothing hides its load latency.  Smaller tiles put several workgroups on a
// CU at the cost of more operand traffic.  Reported per shape: average kernel time (events over
// back-to-back launches), and the max |C - C_ref| against the 64 x 64 kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form gemm_tiles.hip -o bin/gemm_tiles
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

// C (M x N, ldc) = A (M x K, lda) B (K x N, ldb), problem p at fixed strides; workgroup b takes
// tile b / P of problem b % P.  Slabs of BK k-columns, double-buffered in LDS: A as [k][TM+pad]
// (rows contiguous), B as [n][BK+2] (k contiguous, as B is column-major K x N).
template <int WM, int WN, int BK>
__global__ __launch_bounds__(64 * WM * WN) void gemm_t(const double* __restrict__ A, const double* __restrict__ B,
                                                    double* __restrict__ C, int M, int N, int K, int lda,
                                                    int ldb, int ldc, long long sA, long long sB, long long sC,
                                                    int P, int tn) {
  constexpr int TM = 32 * WM, TN = 16 * WN, NTH = 64 * WM * WN;
  constexpr int LA = TM + 4, LB = BK + 2;
  constexpr int SA = BK * LA, SB = TN * LB;
  constexpr int PA = TM * BK / NTH, PB = TN * BK / NTH;
  static_assert(PA * NTH == TM * BK && PB * NTH == TN * BK, "slab split");
  __shared__ double sm[2 * (SA + SB)];
  const int p = blockIdx.x % P, t = blockIdx.x / P;
  const double* Ap = A + p * sA;
  const double* Bp = B + p * sB;
  double* Cp = C + p * sC;
  const int m0 = (t / tn) * TM, n0 = (t % tn) * TN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN, lr = lane & 15, lk = lane >> 4;
  double ra[PA], rb[PB];
  // A slab element q of this thread: row i = tid % TM (contiguous in memory), k = tid / TM + ...
  auto loadA = [&](int k0) {
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int e = tid + NTH * q, i = e % TM, k = e / TM;
      const int gi = min(m0 + i, M - 1), gk = min(k0 + k, K - 1);
      ra[q] = gload(Ap + gi + (size_t)gk * lda);
    }
  };
  auto storeA = [&](double* S, int k0) {
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int e = tid + NTH * q, i = e % TM, k = e / TM;
      S[k * LA + i] = k0 + k < K ? ra[q] : 0.0;
    }
  };
  // B slab: column n (contiguous along k): k = e % BK, n = e / BK
  auto loadB = [&](int k0) {
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int e = tid + NTH * q, k = e % BK, n = e / BK;
      const int gn = min(n0 + n, N - 1), gk = min(k0 + k, K - 1);
      rb[q] = gload(Bp + gk + (size_t)gn * ldb);
    }
  };
  auto storeB = [&](double* S, int k0) {
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int e = tid + NTH * q, k = e % BK, n = e / BK;
      S[n * LB + k] = k0 + k < K ? rb[q] : 0.0;
    }
  };
  d4 acc[2] = {d4{0, 0, 0, 0}, d4{0, 0, 0, 0}};
  loadA(0);
  loadB(0);
  storeA(sm, 0);
  storeB(sm + SA, 0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) {
      loadA(k0 + BK);
      loadB(k0 + BK);
    }
    const double* As = sm + cur * (SA + SB);
    const double* Bs = As + SA;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const double a0 = As[(kk + lk) * LA + wm * 32 + lr];
      const double a1 = As[(kk + lk) * LA + wm * 32 + 16 + lr];
      const double b0 = Bs[(wn * 16 + lr) * LB + kk + lk];
      acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1], 0, 0, 0);
    }
    if (!more) break;
    cur ^= 1;
    storeA(sm + cur * (SA + SB), k0 + BK);
    storeB(sm + cur * (SA + SB) + SA, k0 + BK);
    __syncthreads();
  }
  // accumulator (mi, r) of lane: row wm*32 + 16 mi + lk + 4 r, column wn*16 + lr: store direct
  // (16 lanes on 16 columns; rows lk + 4r); each column gets 4 rows x 2 per wave
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 32 + 16 * mi + lk + 4 * r, col = n0 + wn * 16 + lr;
      if (row < M && col < N) Cp[row + (size_t)col * ldc] = acc[mi][r];
    }
}

template <class K>
float timeit(K k, int reps = 100) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main() {
  const int M = 128, N = 128, K = 128;
  for (int nb : {64, 16, 8}) {
    const size_t sa = (size_t)M * K, sb = (size_t)K * N, sc = (size_t)M * N;
    double *A, *B, *C, *C0;
    CK(hipMalloc(&A, sa * nb * 8)); CK(hipMalloc(&B, sb * nb * 8));
    CK(hipMalloc(&C, sc * nb * 8)); CK(hipMalloc(&C0, sc * nb * 8));
    std::vector<double> h(sa * nb);
    for (auto& x : h) x = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(A, h.data(), sa * nb * 8, hipMemcpyHostToDevice));
    for (auto& x : h) x = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(B, h.data(), sb * nb * 8, hipMemcpyHostToDevice));
    UniGemm u{};
    u.A = A; u.B = B; u.C = C0; u.sA = sa; u.sB = sb; u.sC = sc;
    u.M = M; u.N = N; u.K = K; u.lda = M; u.ldb = K; u.ldc = M; u.ldcin = M; u.tn = 2; u.P = nb;
    const float tp = timeit([&] { gemm_f64_uni<false, false, 0, 32, 8, false, false, true><<<4 * nb, 512>>>(u, 1.0, 0.0); });
    std::vector<double> ref(sc * nb), got(sc * nb);
    CK(hipMemcpy(ref.data(), C0, sc * nb * 8, hipMemcpyDeviceToHost));
    const double flops = 2.0 * M * N * K * nb;
    printf("batch %2d: production 64x64 %.2f us (%.1f TF)\n", nb, tp, flops / tp / 1e6);
    auto run = [&](const char* name, auto kern, int WMv, int WNv) {
      const int TM = 32 * WMv, TN = 16 * WNv, tm = (M + TM - 1) / TM, tnn = (N + TN - 1) / TN;
      const unsigned grid = nb * tm * tnn, thr = 64 * WMv * WNv;
      CK(hipMemset(C, 0, sc * nb * 8));
      const float t = timeit([&] {
        kern<<<grid, thr>>>(A, B, C, M, N, K, M, K, M, (long long)sa, (long long)sb, (long long)sc, nb, tnn);
      });
      CK(hipMemcpy(got.data(), C, sc * nb * 8, hipMemcpyDeviceToHost));
      double e = 0;
      for (size_t i = 0; i < got.size(); ++i) e = fmax(e, fabs(got[i] - ref[i]));
      printf("  %-22s %4u wg  %.2f us (%.1f TF)  max|dC| %.1e\n", name, grid, t, flops / t / 1e6, e);
    };
    run("64x64 2x4 BK32", gemm_t<2, 4, 32>, 2, 4);
    run("64x64 2x4 BK64", gemm_t<2, 4, 64>, 2, 4);
    run("32x64 1x4 BK32", gemm_t<1, 4, 32>, 1, 4);
    run("32x64 1x4 BK64", gemm_t<1, 4, 64>, 1, 4);
    run("64x32 2x2 BK32", gemm_t<2, 2, 32>, 2, 2);
    run("32x32 1x2 BK32", gemm_t<1, 2, 32>, 1, 2);
    run("32x32 1x2 BK64", gemm_t<1, 2, 64>, 1, 2);
    run("32x16 1x1 BK32", gemm_t<1, 1, 32>, 1, 1);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(C0));
  }
  return 0;
}
