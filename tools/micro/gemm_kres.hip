// Round-2 experiment, kept for the record (DESIGN.md §6 "GEMM anatomy"): a K-resident fp64 GEMM
// tile (K <= 128) against the library's gemm_f64_lds on nb x (M x N x K).
//   * every global load of the tile's 64 x K slabs issued up front, stored chunk by chunk (32 k)
//     into its own LDS region, one barrier per chunk (or, DBG = 2, one barrier for all chunks);
//   * k-contiguous LDS images at pitch 132 read as k PAIRS by ds_read_b128 (the MFMA k order is
//     permuted so one 16-B read feeds two MFMA steps; 16-lane groups hit 16 distinct 4-bank slots);
//   * the tile computed transposed so accumulators store coalesced straight from registers.
// Measured (64 x 128^3): 10.4 us vs 11.4 us isolated, but no gain inside the replayed loop body
// (1120-1131 vs 1125-1130 it/s): the 135 KB LDS footprint blocks co-residency with side-stream
// kernels.  Per-workgroup phases (DBG = 1): ~2.2 us descriptor + first loads, 1.3 us per 32-k
// chunk (MFMA issue at two waves per SIMD with a barrier per chunk), 0.8 us epilogue; one barrier
// (DBG = 2) runs the MFMA phase in 4.1 us, 94 % of the fp64 matrix rate at the measured clock.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

namespace kres {
constexpr int KMAX = 128, KC = 32, NCH = KMAX / KC, KP = KMAX + 4;
constexpr int SMEM = 2 * 64 * KP * 8;
template <bool kcontig>
__device__ inline void pq(int tid, int q, int& i, int& pk) {
  if (kcontig) { pk = tid & 15; i = (tid >> 4) + 32 * q; }
  else { i = tid & 63; pk = (tid >> 6) + 8 * q; }
}
typedef double d2 __attribute__((ext_vector_type(2)));
}  // namespace kres

template <bool TA, bool TB, int DBG>
__global__ __launch_bounds__(512) void gemm_kres(const GemmDesc<double>* __restrict__ descs,
                                                 const TileRef* __restrict__ t2d, unsigned long long* stamp) {
  using namespace kres;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  unsigned long long* dbg = stamp + 8 * blockIdx.x;
  if (DBG && threadIdx.x == 0) dbg[0] = __builtin_amdgcn_s_memrealtime();
  const TileRef tr = t2d[blockIdx.x];
  const GemmDesc<double> d = descs[tr.p];
  double* As = reinterpret_cast<double*>(smem_raw);
  double* Bs = As + 64 * KP;
  const int t = tr.t, m0 = (t / d.tn) * 64, n0 = (t % d.tn) * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3, lr = lane & 15, lk = lane >> 4;
  const int M = d.M, N = d.N, K = d.K;
  constexpr bool AK = TA, BKc = !TB;
  auto ga = [&](int i, int k) {
    const int gi = min(m0 + i, M - 1), gk = min(k, K - 1);
    return gload(d.A + (AK ? gk + (size_t)gi * d.lda : gi + (size_t)gk * d.lda));
  };
  auto gb = [&](int j, int k) {
    const int gj = min(n0 + j, N - 1), gk = min(k, K - 1);
    return gload(d.B + (BKc ? gk + (size_t)gj * d.ldb : gj + (size_t)gk * d.ldb));
  };
  double ra[NCH][2][2], rb[NCH][2][2];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int i, pk;
      pq<AK>(tid, q, i, pk);
      ra[c][q][0] = ga(i, c * KC + 2 * pk);
      ra[c][q][1] = ga(i, c * KC + 2 * pk + 1);
      pq<BKc>(tid, q, i, pk);
      rb[c][q][0] = gb(i, c * KC + 2 * pk);
      rb[c][q][1] = gb(i, c * KC + 2 * pk + 1);
    }
  d4 acc[2] = {d4{0.0, 0.0, 0.0, 0.0}, d4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c * KC >= K) break;
    if (DBG == 2 && c > 0) continue;
#pragma unroll
    for (int cc = 0; cc < (DBG == 2 ? NCH : 1); ++cc)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int cs = DBG == 2 ? cc : c;
        if (cs * KC >= K) break;
        int i, pk;
        pq<AK>(tid, q, i, pk);
        const int k = cs * KC + 2 * pk;
        *reinterpret_cast<d2*>(As + i * KP + k) = d2{k < K ? ra[cs][q][0] : 0.0, k + 1 < K ? ra[cs][q][1] : 0.0};
        pq<BKc>(tid, q, i, pk);
        const int kb = cs * KC + 2 * pk;
        *reinterpret_cast<d2*>(Bs + i * KP + kb) = d2{kb < K ? rb[cs][q][0] : 0.0, kb + 1 < K ? rb[cs][q][1] : 0.0};
      }
    __syncthreads();
    if (DBG && tid == 0) dbg[1 + c] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k8 = 0; k8 < (DBG == 2 ? KMAX : KC); k8 += 8) {
      const int kc = c * KC + k8 + 2 * lk;
      const d2 bf = *reinterpret_cast<const d2*>(Bs + (wn * 16 + lr) * KP + kc);
      const d2 a0 = *reinterpret_cast<const d2*>(As + (wm * 32 + lr) * KP + kc);
      const d2 a1 = *reinterpret_cast<const d2*>(As + (wm * 32 + 16 + lr) * KP + kc);
      acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(bf.x, a0.x, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(bf.x, a1.x, acc[1], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(bf.y, a0.y, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(bf.y, a1.y, acc[1], 0, 0, 0);
    }
  }
  if (DBG) {
    __syncthreads();
    if (tid == 0) dbg[5] = __builtin_amdgcn_s_memrealtime();
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int row = m0 + wm * 32 + mi * 16 + lr;
    if (row >= M) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = n0 + wn * 16 + lk + 4 * r;
      if (col < N) d.C[row + (size_t)col * d.ldc] = acc[mi][r];
    }
  }
  if (DBG) {
    __syncthreads();
    if (tid == 0) dbg[6] = __builtin_amdgcn_s_memrealtime();
  }
}

template <class F>
float timeit(F f, int reps = 20) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 128, N = argc > 2 ? atoi(argv[2]) : 128;
  const int K = argc > 3 ? atoi(argv[3]) : 128, nb = argc > 4 ? atoi(argv[4]) : 64;
  if (K < 1 || K > kres::KMAX) { printf("K must be in [1, %d]\n", kres::KMAX); return 1; }
  const size_t sa = (size_t)M * K, sb = (size_t)K * N, sc = (size_t)M * N;
  double *A, *B, *C;
  CK(hipMalloc(&A, sa * nb * 8));
  CK(hipMalloc(&B, sb * nb * 8));
  CK(hipMalloc(&C, sc * nb * 8));
  std::vector<double> h(std::max(sa, sb) * nb);
  for (auto& x : h) x = rand() / (double)RAND_MAX - 0.5;
  CK(hipMemcpy(A, h.data(), sa * nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), sb * nb * 8, hipMemcpyHostToDevice));
  std::vector<GemmDesc<double>> d;
  std::vector<TileRef> t2d;
  for (int b = 0; b < nb; ++b) {
    GemmDesc<double> g{};
    g.A = A + sa * b; g.B = B + sb * b; g.C = C + sc * b;
    g.M = M; g.N = N; g.K = K; g.lda = M; g.ldb = K; g.ldcin = M; g.ldc = M;
    g.tn = (N + 63) / 64;
    d.push_back(g);
  }
  const int nt = ((M + 63) / 64) * d[0].tn;
  for (int t = 0; t < nt; ++t)
    for (int b = 0; b < nb; ++b) t2d.push_back(TileRef{b, t});
  GemmDesc<double>* dd;
  TileRef* dt;
  unsigned long long* st;
  CK(hipMalloc(&dd, d.size() * sizeof(d[0])));
  CK(hipMalloc(&dt, t2d.size() * sizeof(TileRef)));
  CK(hipMemcpy(dd, d.data(), d.size() * sizeof(d[0]), hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, t2d.data(), t2d.size() * sizeof(TileRef), hipMemcpyHostToDevice));
  const unsigned grid = (unsigned)t2d.size();
  CK(hipMalloc(&st, grid * 64));
  const double flops = 2.0 * M * N * K * nb;
  const float us_lds = timeit([&] { gemm_f64_lds<false, false><<<grid, 512>>>(dd, dt, 1.0, 0.0); });
  std::vector<double> ref(sc * nb), out(sc * nb);
  CK(hipMemcpy(ref.data(), C, sc * nb * 8, hipMemcpyDeviceToHost));
  printf("gemm_f64_lds NN  %d x (%d x %d x %d): %.1f us  %.1f TFLOP/s\n", nb, M, N, K, us_lds, flops / us_lds / 1e6);
  auto run = [&](auto dbgc) {
    constexpr int DB = decltype(dbgc)::value;
    CK(hipFuncSetAttribute((const void*)gemm_kres<false, false, DB>, hipFuncAttributeMaxDynamicSharedMemorySize, kres::SMEM));
    const float us = timeit([&] { gemm_kres<false, false, DB><<<grid, 512, kres::SMEM>>>(dd, dt, st); });
    CK(hipMemcpy(out.data(), C, sc * nb * 8, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t q = 0; q < out.size(); ++q) md = std::max(md, std::fabs(out[q] - ref[q]));
    printf("gemm_kres DBG %d: %.1f us  %.1f TFLOP/s  max |kres - lds| %.2e\n", DB, us, flops / us / 1e6, md);
    if (DB == 0) return;
    std::vector<unsigned long long> hs(grid * 8);
    CK(hipMemcpy(hs.data(), st, grid * 64, hipMemcpyDeviceToHost));
    double load = 0, mfma = 0, epi = 0;
    for (unsigned g = 0; g < grid; ++g) {
      load += (double)(hs[8 * g + 1] - hs[8 * g]) / grid;
      mfma += (double)(hs[8 * g + 5] - hs[8 * g + 1]) / grid;
      epi += (double)(hs[8 * g + 6] - hs[8 * g + 5]) / grid;
    }
    printf("   per workgroup (us): start -> first barrier %.2f, MFMA phase %.2f, epilogue %.2f\n",
           load * 1e-2, mfma * 1e-2, epi * 1e-2);
  };
  run(std::integral_constant<int, 0>{});
  run(std::integral_constant<int, 1>{});
  run(std::integral_constant<int, 2>{});
  return 0;
}
