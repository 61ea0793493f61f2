// Ozaki-scheme prototype (round 6): a batched double-double GEMM
// C = A B on the int8 matrix cores against the VALU double-double GEMM of the solver
// (gemm_valu_ks<dd>), at the shape of config 4's Schur products (A 64 x 64, B 64 x 128, 16
// problems; K = 64).
//
// Scheme (Ozaki et al. 2012, with integer slices as in Ootomo/Ozaki/Yokota 2024): every row i
// of A is scaled by 2^-E_i (|a_ik| 2^-E_i < 1/2) and written as S base-2^7 digits,
//     a_ik = 2^E_i sum_{p<S} d_ikp 2^-7(p+1),   d_ikp in [-64, 64]  (int8),
// each digit the rounded leading part of the exact double-double remainder; every column j of B
// likewise with 2^F_j.  Then
//     (A B)_ij = 2^(E_i+F_j) sum_L 2^-7(L+2) sum_{p+q=L} (D_p G_q)_ij ,
// each level-L sum of int8 products accumulates exactly in int32 (|.| <= 16 K 64^2 < 2^31) on
// v_mfma_i32_16x16x64_i8, converts exactly to fp64, and the S levels are summed in double-double.
// Levels L >= S are dropped: the truncation is ~2^-7S relative to 2^(E_i+F_j) K -- a normwise
// (row / column) bound, where the VALU GEMM's is componentwise.  S = 16: 136 int8 products per
// 16 x 16 tile against 64 double-double FMAs per output on the VALU.
//
// Prints: the lane-layout self-test of the int8 MFMA (exact integers), the largest error of
// each GEMM against a host double-double reference relative to 2^(E_i+F_j) K (normwise) and to
// |C_ij| (entrywise), and the time per batch (best of 7): split A, split B, the int8 GEMM, and
// gemm_valu_ks.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 ozaki_dd_bench.hip -o ../../microbin/ozaki_dd_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
using mw::dd;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int S = 16;  // digits per entry

template <class K>
float timeit(K k) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  k();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 7; ++rep) {
    float ms;
    CK(hipEventRecord(e0));
    k();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = fminf(best, ms * 1e3f);
  }
  return best;
}

// ---- int8 MFMA lane layout self-test: A 16 x 64, B 64 x 16 (row-major A, column-major B)
// LAYOUT 0: lane l holds A[l & 15][16 (l >> 4) + j] and B[16 (l >> 4) + j][l & 15], byte j
// LAYOUT 1: k = 8 (j >> 3) * 4 ... (alternative: k = 4 (l >> 4) + (j & 3) + 16 (j >> 2))
__device__ __forceinline__ int kmap(int layout, int l, int j) {
  return layout == 0 ? 16 * (l >> 4) + j : 4 * (l >> 4) + (j & 3) + 16 * (j >> 2);
}
__global__ void mfma_i8_selftest(const signed char* A, const signed char* B, int* C, int layout) {
  const int l = threadIdx.x;
  v4i a, b;
  signed char* pa = reinterpret_cast<signed char*>(&a);
  signed char* pb = reinterpret_cast<signed char*>(&b);
  for (int j = 0; j < 16; ++j) {
    const int k = kmap(layout, l, j);
    pa[j] = A[(l & 15) * 64 + k];
    pb[j] = B[(l & 15) * 64 + k];
  }
  v4i acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];  // C[row][col]
}

// ---- digit split.  Rows of A (M x K, column-major, ld M): one wave per (problem, row), lane =
// k (K = 64).  Out: D[prob][p][row][k] int8, E[prob][row].  Columns of B (K x N, column-major,
// ld K): one wave per (problem, column), lane = k.  Out: G[prob][q][col][k], F[prob][col].
__device__ __forceinline__ int wave_max_int(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ void digits(dd x, int E, signed char* out, size_t stride) {
  // x 2^-E: |.| < 1/2; digit p = rint(r 2^7), r <- r 2^7 - digit (exact in double-double)
  x = dd(ldexp(x.hi, -E), ldexp(x.lo, -E));
#pragma unroll
  for (int p = 0; p < S; ++p) {
    x = dd(x.hi * 128.0, x.lo * 128.0);
    const double dg = rint(x.hi);
    double e;
    const double h = mw::two_sum(x.hi - dg, x.lo, e);  // (x.hi - dg exact)
    x = dd(h, e);
    out[p * stride] = (signed char)(int)dg;
  }
}
__global__ void split_rows(const dd* A, int M, int K, signed char* D, int* E) {
  const int wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int prob = wv / M, row = wv % M;
  const dd a = A[(size_t)prob * M * K + row + (size_t)lane * M];
  int ex = a.hi != 0.0 ? ilogb(a.hi) : -1100;
  ex = wave_max_int(ex);
  const int Ei = ex + 2;  // |a| < 2^(ex+1) <= 2^Ei / 2
  digits(a, Ei, D + ((size_t)prob * S * M + row) * K + lane, (size_t)M * K);
  if (lane == 0) E[prob * M + row] = Ei;
}
__global__ void split_cols(const dd* B, int K, int N, signed char* G, int* F) {
  const int wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int prob = wv / N, col = wv % N;
  const dd b = B[(size_t)prob * K * N + lane + (size_t)col * K];
  int ex = b.hi != 0.0 ? ilogb(b.hi) : -1100;
  ex = wave_max_int(ex);
  const int Fj = ex + 2;
  digits(b, Fj, G + ((size_t)prob * S * N + col) * K + lane, (size_t)N * K);
  if (lane == 0) F[prob * N + col] = Fj;
}

// ---- the int8 GEMM: one wave per 16 x 16 output tile, 4 waves per workgroup; all S digit
// fragments of its 16 rows and 16 columns in registers (K = 64: one MFMA per digit pair)
__global__ __launch_bounds__(256) void ozaki_gemm(const signed char* D, const int* E, const signed char* G,
                                                  const int* F, dd* C, int M, int N, int P) {
  const int K = 64;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  const int tm = M / 16, tn = N / 16;
  const int prob = wv / (tm * tn), t = wv % (tm * tn);
  if (prob >= P) return;
  const int r0 = 16 * (t / tn), c0 = 16 * (t % tn);
  v4i a[S], b[S];
#pragma unroll
  for (int p = 0; p < S; ++p) {
    a[p] = *reinterpret_cast<const v4i*>(D + (((size_t)prob * S + p) * M + r0 + (l & 15)) * K + 16 * (l >> 4));
    b[p] = *reinterpret_cast<const v4i*>(G + (((size_t)prob * S + p) * N + c0 + (l & 15)) * K + 16 * (l >> 4));
  }
  dd acc[4] = {dd(0.0), dd(0.0), dd(0.0), dd(0.0)};
#pragma unroll
  for (int L = S - 1; L >= 0; --L) {  // smallest level first
    v4i c = {0, 0, 0, 0};
#pragma unroll
    for (int p = 0; p <= L; ++p) c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[p], b[L - p], c, 0, 0, 0);
    const double w = ldexp(1.0, -7 * (L + 2));
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // (exact: |c| < 2^31, w a power of two)
      double e;
      const double s = mw::two_sum(acc[r].hi, (double)c[r] * w, e);
      acc[r] = mw::dd(s, e + acc[r].lo);
      double e2;
      const double s2 = mw::quick_two_sum(acc[r].hi, acc[r].lo, e2);
      acc[r] = dd(s2, e2);
    }
  }
  const int col = c0 + (l & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = r0 + (l >> 4) * 4 + r;
    const int sc = E[prob * M + row] + F[prob * N + col];
    C[(size_t)prob * M * N + row + (size_t)col * M] = dd(ldexp(acc[r].hi, sc), ldexp(acc[r].lo, sc));
  }
}

int main(int argc, char** argv) {
  // lane-layout self-test
  {
    std::vector<signed char> A(16 * 64), B(16 * 64);
    srand(3);
    for (auto& v : A) v = (signed char)(rand() % 129 - 64);
    for (auto& v : B) v = (signed char)(rand() % 129 - 64);
    std::vector<int> ref(256, 0);
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j)
        for (int k = 0; k < 64; ++k) ref[i * 16 + j] += A[i * 64 + k] * B[j * 64 + k];
    signed char *dA, *dB;
    int* dC;
    CK(hipMalloc(&dA, 1024));
    CK(hipMalloc(&dB, 1024));
    CK(hipMalloc(&dC, 1024));
    CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    for (int layout = 0; layout < 2; ++layout) {
      mfma_i8_selftest<<<1, 64>>>(dA, dB, dC, layout);
      std::vector<int> got(256);
      CK(hipMemcpy(got.data(), dC, 1024, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int e = 0; e < 256; ++e) bad += got[e] != ref[e];
      printf("int8 MFMA 16x16x64 lane layout %d: %d of 256 outputs differ\n", layout, bad);
    }
  }
  const int P = argc > 1 ? atoi(argv[1]) : 16, M = 64, N = 128, K = 64;
  const size_t na = (size_t)P * M * K, nb = (size_t)P * K * N, nc = (size_t)P * M * N;
  std::vector<dd> hA(na), hB(nb);
  srand(11);
  auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
  for (size_t e = 0; e < na; ++e) {  // rows of varied scale, full double-double entries
    const int row = (int)(e % M);
    const double hi = ldexp(rnd(), (row % 7) - 3);
    hA[e] = dd(hi, hi * rnd() * 0x1p-53);
  }
  for (size_t e = 0; e < nb; ++e) {
    const double hi = rnd();
    hB[e] = dd(hi, hi * rnd() * 0x1p-53);
  }
  // host double-double reference
  std::vector<dd> ref(nc);
  for (int q = 0; q < P; ++q)
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < M; ++i) {
        dd s(0.0);
        for (int k = 0; k < K; ++k)
          s = s + hA[(size_t)q * M * K + i + (size_t)k * M] * hB[(size_t)q * K * N + k + (size_t)j * K];
        ref[(size_t)q * M * N + i + (size_t)j * M] = s;
      }
  dd *dA, *dB, *dC1, *dC2;
  CK(hipMalloc(&dA, na * sizeof(dd)));
  CK(hipMalloc(&dB, nb * sizeof(dd)));
  CK(hipMalloc(&dC1, nc * sizeof(dd)));
  CK(hipMalloc(&dC2, nc * sizeof(dd)));
  CK(hipMemcpy(dA, hA.data(), na * sizeof(dd), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), nb * sizeof(dd), hipMemcpyHostToDevice));
  signed char *dD, *dG;
  int *dE, *dF;
  CK(hipMalloc(&dD, na * S));
  CK(hipMalloc(&dG, nb * S));
  CK(hipMalloc(&dE, P * M * sizeof(int)));
  CK(hipMalloc(&dF, P * N * sizeof(int)));
  // the VALU double-double GEMM as the solver launches it (8 x 8 tiles, K split in the workgroup)
  std::vector<GemmDesc<dd>> gd(P);
  std::vector<TileRef> t2d;
  for (int q = 0; q < P; ++q) {
    GemmDesc<dd> g{};
    g.A = dA + (size_t)q * M * K; g.B = dB + (size_t)q * K * N; g.Cin = nullptr; g.C = dC1 + (size_t)q * M * N;
    g.M = M; g.N = N; g.K = K; g.lda = M; g.ldb = K; g.ldcin = M; g.ldc = M;
    g.tn = N / 8; g.tile0 = 0; g.flags = 0; g.alpha = g.beta = 0.0; g.sa = g.sl = nullptr;
    gd[q] = g;
  }
  for (int t = 0; t < (M / 8) * (N / 8); ++t)
    for (int q = 0; q < P; ++q) t2d.push_back(TileRef{q, t});
  GemmDesc<dd>* dgd;
  TileRef* dt;
  CK(hipMalloc(&dgd, P * sizeof(GemmDesc<dd>)));
  CK(hipMalloc(&dt, t2d.size() * sizeof(TileRef)));
  CK(hipMemcpy(dgd, gd.data(), P * sizeof(GemmDesc<dd>), hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, t2d.data(), t2d.size() * sizeof(TileRef), hipMemcpyHostToDevice));
  const unsigned tiles = (unsigned)t2d.size();
  const float tv = timeit([&] { gemm_valu_ks<dd, false, false><<<tiles, 256>>>(dgd, dt, 1.0, 0.0); });
  const float ts1 = timeit([&] { split_rows<<<P * M / 4, 256>>>(dA, M, K, dD, dE); });
  const float ts2 = timeit([&] { split_cols<<<P * N / 4, 256>>>(dB, K, N, dG, dF); });
  const unsigned owg = (unsigned)((P * (M / 16) * (N / 16) + 3) / 4);
  const float tg = timeit([&] { ozaki_gemm<<<owg, 256>>>(dD, dE, dG, dF, dC2, M, N, P); });
  const float tall = timeit([&] {
    split_rows<<<P * M / 4, 256>>>(dA, M, K, dD, dE);
    split_cols<<<P * N / 4, 256>>>(dB, K, N, dG, dF);
    ozaki_gemm<<<owg, 256>>>(dD, dE, dG, dF, dC2, M, N, P);
  });
  CK(hipDeviceSynchronize());
  std::vector<dd> c1(nc), c2(nc);
  CK(hipMemcpy(c1.data(), dC1, nc * sizeof(dd), hipMemcpyDeviceToHost));
  CK(hipMemcpy(c2.data(), dC2, nc * sizeof(dd), hipMemcpyDeviceToHost));
  std::vector<int> hE(P * M), hF(P * N);
  CK(hipMemcpy(hE.data(), dE, hE.size() * sizeof(int), hipMemcpyDeviceToHost));
  CK(hipMemcpy(hF.data(), dF, hF.size() * sizeof(int), hipMemcpyDeviceToHost));
  double nw1 = 0, nw2 = 0, en1 = 0, en2 = 0;
  for (int q = 0; q < P; ++q)
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < M; ++i) {
        const size_t e = (size_t)q * M * N + i + (size_t)j * M;
        const double scale = ldexp((double)K, hE[q * M + i] + hF[q * N + j]);
        const dd d1 = c1[e] - ref[e], d2 = c2[e] - ref[e];
        nw1 = fmax(nw1, fabs(d1.hi) / scale);
        nw2 = fmax(nw2, fabs(d2.hi) / scale);
        const double m = fabs(ref[e].hi);
        if (m > 0) {
          en1 = fmax(en1, fabs(d1.hi) / m);
          en2 = fmax(en2, fabs(d2.hi) / m);
        }
      }
  printf("dd GEMM %d x (%d x %d) @ (%d x %d): error vs host dd, normwise (2^(E+F) K) / entrywise:\n", P, M, K, K, N);
  printf("  gemm_valu_ks (VALU dd)   %.2e / %.2e   %.1f us\n", nw1, en1, tv);
  printf("  Ozaki int8, S = %d        %.2e / %.2e   split A %.1f + split B %.1f + int8 GEMM %.1f us; all three back to back %.1f us\n",
         S, nw2, en2, ts1, ts2, tg, tall);
  return 0;
}
