// The Schur pairing at C3 (64 clusters, K = 255 samples, delta = 128): schur_fused_f64 (V^T X^-1
// on chip) against the unfused pair (uniform V^T X^-1 GEMM + schur_pairs_f64), and the fused
// kernel with its phase-2 (DBG 1) or phase-1 (DBG 2) MFMAs removed, to split its time.
// Events over back-to-back launches; max |G_fused - G_unfused| as the check.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form schur_fused_bench.hip -o bin/schur_fused_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

template <class F>
float timeit(F f, int reps = 50) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main() {
  const int J = 64, K = 255, D = 128;
  const size_t nV = (size_t)J * K * D, nX = (size_t)J * D * D, nG = (size_t)J * K * K;
  std::vector<double> h(nV);
  auto rnd = [] { return rand() / (double)RAND_MAX - 0.5; };
  double *Vt, *Xi, *TX, *TY, *lam, *G0, *G1, *AY0, *AY1;
  CK(hipMalloc(&Vt, nV * 8)); CK(hipMalloc(&TX, nV * 8)); CK(hipMalloc(&TY, nV * 8));
  CK(hipMalloc(&Xi, nX * 8)); CK(hipMalloc(&lam, (size_t)J * K * 8));
  CK(hipMalloc(&G0, nG * 8)); CK(hipMalloc(&G1, nG * 8));
  CK(hipMalloc(&AY0, (size_t)J * K * 8)); CK(hipMalloc(&AY1, (size_t)J * K * 8));
  for (auto& x : h) x = rnd();
  CK(hipMemcpy(Vt, h.data(), nV * 8, hipMemcpyHostToDevice));
  for (auto& x : h) x = rnd();
  CK(hipMemcpy(TY, h.data(), nV * 8, hipMemcpyHostToDevice));
  std::vector<double> hx(nX);
  for (int j = 0; j < J; ++j)
    for (int c = 0; c < D; ++c)
      for (int r = 0; r <= c; ++r) {
        const double v = rnd() + (r == c ? 4.0 : 0.0);
        hx[(size_t)j * D * D + r + (size_t)c * D] = hx[(size_t)j * D * D + c + (size_t)r * D] = v;
      }
  CK(hipMemcpy(Xi, hx.data(), nX * 8, hipMemcpyHostToDevice));
  std::vector<double> hl((size_t)J * K);
  for (auto& x : hl) x = 0.5 + rnd();
  CK(hipMemcpy(lam, hl.data(), hl.size() * 8, hipMemcpyHostToDevice));
  // unfused: TXt = Vt X^-1^T (uniform batch), then the pairs
  UniGemm u{};
  u.A = Vt; u.B = Xi; u.C = TX; u.sA = (long long)K * D; u.sB = (long long)D * D; u.sC = (long long)K * D;
  u.M = K; u.N = D; u.K = D; u.lda = K; u.ldb = D; u.ldc = K; u.ldcin = K; u.tn = 2; u.P = J;
  std::vector<PairTileDesc> pd;
  std::vector<FusedPairDesc> fd;
  for (int j = 0; j < J; ++j) {
    PairTileDesc t;
    t.grp = 1;
    t.pad = 0;
    t.Vt = Vt + (size_t)j * K * D; t.TXt = TX + (size_t)j * K * D; t.TYt = TY + (size_t)j * K * D;
    t.lam = lam + (size_t)j * K; t.G = G0 + (size_t)j * K * K; t.AY = AY0 + (size_t)j * K;
    t.K = K; t.del = D; t.ldG = K; t.tile0 = 0;
    pd.push_back(t);
    FusedPairDesc f;
    f.Vt = t.Vt; f.Xinv = Xi + (size_t)j * D * D; f.TYt = t.TYt; f.lam = t.lam;
    f.G = G1 + (size_t)j * K * K; f.AY = AY1 + (size_t)j * K; f.K = K; f.del = D; f.ldG = K; f.ldx = D;
    f.Y = Xi + (size_t)j * D * D; f.ldy = D;  // (any symmetric matrix: timing only)
    f.grp = 1; f.pad = 0;
    fd.push_back(f);
  }
  std::vector<TileRef> pt, ft;
  for (int t = 0; t < 10; ++t) for (int j = 0; j < J; ++j) pt.push_back(TileRef{j, t});
  for (int t = 0; t < 4; ++t) for (int j = 0; j < J; ++j) ft.push_back(TileRef{j, t});
  PairTileDesc* dpd; FusedPairDesc* dfd; TileRef *dpt, *dft;
  CK(hipMalloc(&dpd, pd.size() * sizeof(pd[0]))); CK(hipMalloc(&dfd, fd.size() * sizeof(fd[0])));
  CK(hipMalloc(&dpt, pt.size() * sizeof(TileRef))); CK(hipMalloc(&dft, ft.size() * sizeof(TileRef)));
  CK(hipMemcpy(dpd, pd.data(), pd.size() * sizeof(pd[0]), hipMemcpyHostToDevice));
  CK(hipMemcpy(dfd, fd.data(), fd.size() * sizeof(fd[0]), hipMemcpyHostToDevice));
  CK(hipMemcpy(dpt, pt.data(), pt.size() * sizeof(TileRef), hipMemcpyHostToDevice));
  CK(hipMemcpy(dft, ft.data(), ft.size() * sizeof(TileRef), hipMemcpyHostToDevice));
  for (auto k : {(const void*)schur_fused_f64<0>, (const void*)schur_fused_f64<1>, (const void*)schur_fused_f64<2>, (const void*)schur_fused_f64<0, true>})
    CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)schur_fused::LDS));
  const unsigned gg = (unsigned)(J * 4 * 2);
  const float tg = timeit([&] { gemm_f64_uni<false, true, 0, 32, 8, false, false, true><<<gg, 512>>>(u, 1.0, 0.0); });
  const float tp = timeit([&] { schur_pairs_f64<16><<<(unsigned)pt.size(), 256>>>(dpd, dpt, nullptr); });
  const float tu = timeit([&] {
    gemm_f64_uni<false, true, 0, 32, 8, false, false, true><<<gg, 512>>>(u, 1.0, 0.0);
    schur_pairs_f64<16><<<(unsigned)pt.size(), 256>>>(dpd, dpt, nullptr);
  });
  const float tf = timeit([&] { schur_fused_f64<0><<<(unsigned)ft.size(), 512, schur_fused::LDS>>>(dfd, dft, nullptr); });
  const float t1 = timeit([&] { schur_fused_f64<1><<<(unsigned)ft.size(), 512, schur_fused::LDS>>>(dfd, dft, nullptr); });
  const float t2 = timeit([&] { schur_fused_f64<2><<<(unsigned)ft.size(), 512, schur_fused::LDS>>>(dfd, dft, nullptr); });
  const float ty = timeit([&] { schur_fused_f64<0, true><<<(unsigned)ft.size(), 512, schur_fused::LDS>>>(dfd, dft, nullptr); });
  printf("fused with V^T Y on chip (YV): %.2f us\n", ty);
  // check
  CK(hipMemset(G1, 0, nG * 8));
  schur_fused_f64<0><<<(unsigned)ft.size(), 512, schur_fused::LDS>>>(dfd, dft, nullptr);
  CK(hipDeviceSynchronize());
  std::vector<double> g0(nG), g1(nG);
  CK(hipMemcpy(g0.data(), G0, nG * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(g1.data(), G1, nG * 8, hipMemcpyDeviceToHost));
  double e = 0, mx = 0;
  for (size_t i = 0; i < nG; ++i) { e = fmax(e, fabs(g0[i] - g1[i])); mx = fmax(mx, fabs(g0[i])); }
  printf("TXt GEMM %.2f us | pairs %.2f us | both %.2f us | fused %.2f us | fused w/o phase-2 MFMA %.2f | w/o phase-1 MFMA %.2f | max|dG|/max|G| %.1e\n",
         tg, tp, tu, tf, t1, t2, e / mx);
  return 0;
}
