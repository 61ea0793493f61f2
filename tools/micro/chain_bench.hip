// chain_f64 (two dependent products per block as one strip launch) against the pair of
// gemm_f64_uni launches it replaces, on a C3-shaped batch (64 blocks of 128 x 128, and 8 blocks:
// the N = 8 shard): time per launch (best of 20) and the largest |difference| of the results.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form chain_bench.hip \
//     -o ../../microbin/chain_bench && ../../microbin/chain_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <class K>
float best_of(K k, int reps = 20) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  k();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    k();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  return best * 1e3f;
}

static UniGemm uni(const double* A, const double* B, const double* Cin, double* C, int n, int P) {
  UniGemm u{};
  u.A = A; u.B = B; u.Cin = Cin; u.C = C;
  u.sA = u.sB = u.sCin = u.sC = (long long)n * n;
  u.M = u.N = u.K = n; u.lda = u.ldb = u.ldcin = u.ldc = n;
  u.tn = (n + 63) / 64; u.P = P;
  return u;
}

int main() {
  const int n = 128;
  for (int P : {64, 8}) {
    const size_t N = (size_t)P * n * n;
    std::vector<double> h(N);
    auto fill = [&](double* d, unsigned seed, bool lower) {
      srand(seed);
      for (int p = 0; p < P; ++p)
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < n; ++i)
            h[(size_t)p * n * n + i + (size_t)j * n] =
                (lower && i < j) ? 0.0 : (rand() / (double)RAND_MAX - 0.5) + (i == j ? 2.0 : 0.0);
      CK(hipMemcpy(d, h.data(), N * 8, hipMemcpyHostToDevice));
    };
    double *Pm, *Y, *R, *Xi, *T, *Z1, *Z2, *L, *dM, *S1, *S2;
    for (double** b : {&Pm, &Y, &R, &Xi, &T, &Z1, &Z2, &L, &dM, &S1, &S2}) CK(hipMalloc(b, N * 8));
    fill(Pm, 1, false); fill(Y, 2, false); fill(R, 3, false); fill(Xi, 4, false);
    fill(L, 5, true); fill(dM, 6, false);
    {  // dM symmetric (the step length's dX / dY)
      for (int p = 0; p < P; ++p)
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < j; ++i)
            h[(size_t)p * n * n + i + (size_t)j * n] = h[(size_t)p * n * n + j + (size_t)i * n];
      CK(hipMemcpy(dM, h.data(), N * 8, hipMemcpyHostToDevice));
    }
    // ---- Z = X^-1 (P Y - R): the pair
    const unsigned tiles = P * 4;
    auto pair = [&] {
      gemm_f64_uni<false, false><<<tiles, 512>>>(uni(Pm, Y, R, T, n, P), 1.0, -1.0);
      gemm_f64_uni<false, false><<<tiles, 512>>>(uni(Xi, T, nullptr, Z1, n, P), 1.0, 0.0);
    };
    ChainGemm c{};
    c.A1[0] = Pm; c.B1[0] = Y; c.C1[0] = R; c.A2[0] = Xi; c.O[0] = Z2;
    c.sA1 = c.sB1 = c.sC1 = c.sA2 = c.sO = (long long)n * n;
    c.n = n; c.lda1 = c.ldb1 = c.ldc1 = c.lda2 = c.ldo = n;
    c.P = c.P1 = P;
    CK(hipFuncSetAttribute((const void*)chain_f64<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chain::LDS));
    CK(hipFuncSetAttribute((const void*)chain_f64<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chain::LDS));
    auto ch = [&] { chain_f64<false, false><<<P * 4, 512, chain::LDS>>>(c, 1.0, -1.0); };
    const float tp = best_of(pair), tc = best_of(ch);
    {  // where the chain's time goes: without its MFMAs, without its A loads
      CK(hipFuncSetAttribute((const void*)chain_f64<false, false, false, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chain::LDS));
      CK(hipFuncSetAttribute((const void*)chain_f64<false, false, false, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chain::LDS));
      auto c1 = [&] { chain_f64<false, false, false, 1><<<P * 4, 512, chain::LDS>>>(c, 1.0, -1.0); };
      auto c2 = [&] { chain_f64<false, false, false, 2><<<P * 4, 512, chain::LDS>>>(c, 1.0, -1.0); };
      auto c3 = [&] { chain_f64<false, false, false, 3><<<P * 4, 512, chain::LDS>>>(c, 1.0, -1.0); };
      CK(hipFuncSetAttribute((const void*)chain_f64<false, false, false, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chain::LDS));
      printf("P=%2d  Z chain breakdown: no MFMA %6.2f us, no A loads %6.2f us, neither %6.2f us\n", P,
             best_of(c1), best_of(c2), best_of(c3));
    }
    std::vector<double> a(N), b(N);
    CK(hipMemcpy(a.data(), Z1, N * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Z2, N * 8, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    for (size_t e = 0; e < N; ++e) { md = fmax(md, fabs(a[e] - b[e])); mx = fmax(mx, fabs(a[e])); }
    printf("P=%2d  Z chain: pair %6.2f us  chain %6.2f us  max|diff|/max %.2e\n", P, tp, tc, md / mx);
    // ---- L dM L^T (SYM): the pair (L dM, then (.) L^T) against the strip chain
    auto pair2 = [&] {
      gemm_f64_uni<false, false><<<tiles, 512>>>(uni(L, dM, nullptr, T, n, P), 1.0, 0.0);
      gemm_f64_uni<false, true><<<tiles, 512>>>(uni(T, L, nullptr, S1, n, P), 1.0, 0.0);
    };
    ChainGemm c2 = c;
    c2.A1[0] = dM; c2.B1[0] = L; c2.C1[0] = nullptr; c2.A2[0] = L; c2.O[0] = S2;
    auto ch2 = [&] { chain_f64<true, true><<<P * 4, 512, chain::LDS>>>(c2, 1.0, 0.0); };
    const float tp2 = best_of(pair2), tc2 = best_of(ch2);
    CK(hipMemcpy(a.data(), S1, N * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), S2, N * 8, hipMemcpyDeviceToHost));
    md = 0; mx = 0;
    double asym = 0;
    for (int p = 0; p < P; ++p)
      for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
          const size_t e = (size_t)p * n * n + i + (size_t)j * n, et = (size_t)p * n * n + j + (size_t)i * n;
          md = fmax(md, fabs(a[e] - b[e]));
          mx = fmax(mx, fabs(a[e]));
          asym = fmax(asym, fabs(b[e] - b[et]));
        }
    printf("P=%2d  step  : pair %6.2f us  chain %6.2f us  max|diff|/max %.2e  asym %.1e\n", P, tp2,
           tc2, md / mx, asym);
    // ---- U = Z V (n x K, K = 2n - 1) + the column sums (TRACE) against the GEMM alone
    {
      const int K = 2 * n - 1;
      double *V, *U, *lam, *din, *rout;
      CK(hipMalloc(&V, (size_t)P * n * K * 8));
      CK(hipMalloc(&U, (size_t)P * n * K * 8));
      CK(hipMalloc(&lam, (size_t)P * K * 8));
      CK(hipMalloc(&din, (size_t)P * K * 8));
      CK(hipMalloc(&rout, (size_t)P * K * 8));
      CK(hipMemset(V, 0, (size_t)P * n * K * 8));
      CK(hipMemset(lam, 0, (size_t)P * K * 8));
      CK(hipMemset(din, 0, (size_t)P * K * 8));
      UniGemm g{};
      g.A = Z1; g.B = V; g.C = U;
      g.sA = (long long)n * n; g.sB = (long long)n * K; g.sC = (long long)n * K;
      g.M = n; g.N = K; g.K = n; g.lda = n; g.ldb = n; g.ldc = n; g.tn = (K + 63) / 64; g.P = P;
      const unsigned t3 = P * 2 * g.tn;
      auto gm = [&] { gemm_f64_uni<false, false><<<t3, 512>>>(g, 1.0, 0.0); };
      ChainGemm c3{};
      c3.A1[0] = Z1; c3.B1[0] = V; c3.sA1 = (long long)n * n; c3.sB1 = (long long)n * K;
      c3.n = n; c3.lda1 = n; c3.ldb1 = n; c3.P = c3.P1 = P; c3.NC = K;
      c3.lam = lam; c3.din = din; c3.rout = rout; c3.sLam = K; c3.sX = K; c3.c_in = -1; c3.c_agg = -1;
      CK(hipFuncSetAttribute((const void*)chain_f64<false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chain::LDS));
      auto ch3 = [&] { chain_f64<false, false, true><<<P * ((K + 31) / 32), 512, chain::LDS_TRACE>>>(c3, 1.0, 0.0); };
      printf("P=%2d  trace : U = Z V gemm %6.2f us  chain (U on chip + column sums) %6.2f us\n", P,
             best_of(gm), best_of(ch3));
      for (double* b2 : {V, U, lam, din, rout}) CK(hipFree(b2));
    }
    for (double* b2 : {Pm, Y, R, Xi, T, Z1, Z2, L, dM, S1, S2}) CK(hipFree(b2));
  }
  return 0;
}
