// Timing of the fused Schur path at the C3 shape (64 blocks, delta = 128, K = 255):
// TXt/TYt = V^T X^-1 / V^T Y (gemm_f64_lds NT, one launch) and schur_pairs_f64.
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
template <class X> X* up(const std::vector<X>& v) { X* p; CK(hipMalloc(&p, v.size() * sizeof(X))); CK(hipMemcpy(p, v.data(), v.size() * sizeof(X), hipMemcpyHostToDevice)); return p; }

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 64, del = argc > 2 ? atoi(argv[2]) : 128, K = argc > 3 ? atoi(argv[3]) : 255;
  const size_t sv = (size_t)del * K, sx = (size_t)del * del;
  std::vector<double> h(std::max(sv, sx) * nb);
  for (auto& x : h) x = rand() / (double)RAND_MAX - 0.5;
  double *Vt, *X, *Y, *TX, *TY, *G, *AY, *lam;
  CK(hipMalloc(&Vt, sv * nb * 8)); CK(hipMalloc(&X, sx * nb * 8)); CK(hipMalloc(&Y, sx * nb * 8));
  CK(hipMalloc(&TX, sv * nb * 8)); CK(hipMalloc(&TY, sv * nb * 8)); CK(hipMalloc(&G, (size_t)K * K * nb * 8));
  CK(hipMalloc(&AY, (size_t)K * nb * 8)); CK(hipMalloc(&lam, (size_t)K * nb * 8));
  CK(hipMemcpy(Vt, h.data(), sv * nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(X, h.data(), sx * nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Y, h.data(), sx * nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(lam, h.data(), (size_t)K * nb * 8, hipMemcpyHostToDevice));
  // TXt/TYt GEMM
  std::vector<GemmDesc<double>> gd; std::vector<TileRef> gt;
  for (int b = 0; b < nb; ++b)
    for (int w = 0; w < 2; ++w) {
      GemmDesc<double> g{Vt + sv * b, (w ? Y : X) + sx * b, nullptr, (w ? TY : TX) + sv * b, K, del, del, K, del, 0, K, (del + 63) / 64, 0, 0};
      gd.push_back(g);
    }
  for (int t = 0; t < ((K + 63) / 64) * gd[0].tn; ++t)
    for (int p = 0; p < (int)gd.size(); ++p) gt.push_back(TileRef{p, t});
  GemmDesc<double>* dgd = up(gd); TileRef* dgt = up(gt);
  std::vector<PairTileDesc> pd; std::vector<TileRef> pt;
  const int nt = (K + 63) / 64;
  for (int b = 0; b < nb; ++b) {
    PairTileDesc t{Vt + sv * b, TX + sv * b, TY + sv * b, lam + (size_t)K * b, G + (size_t)K * K * b, AY + (size_t)K * b, K, del, K, 0};
    pd.push_back(t);
  }
  for (int u = 0; u < nt * (nt + 1) / 2; ++u)
    for (int b = 0; b < nb; ++b) pt.push_back(TileRef{b, u});
  PairTileDesc* dpd = up(pd); TileRef* dpt = up(pt);
  const double fl_txy = 2.0 * 2 * K * del * del * nb, fl_pairs = 2.0 * 2 * del * 64.0 * 64 * pt.size();
  const double alg = 4.0 * del * K * (del + K) * nb + 8.0 * K * (K + 1) / 2.0 * nb;
  printf("blocks %d delta %d K %d\n", nb, del, K);
  for (int v = 0; v < 2; ++v) {
    float t1, t2, t3;
    if (v == 0) {
      t1 = timeit([&] { gemm_f64_lds<false, true, 1, 32><<<(unsigned)gt.size(), 512>>>(dgd, dgt, 1.0, 0.0); });
      t2 = timeit([&] { schur_pairs_f64<32><<<(unsigned)pt.size(), 256>>>(dpd, dpt); });
      t3 = timeit([&] { gemm_f64_lds<false, true, 1, 32><<<(unsigned)gt.size(), 512>>>(dgd, dgt, 1.0, 0.0);
                        schur_pairs_f64<32><<<(unsigned)pt.size(), 256>>>(dpd, dpt); });
    } else {
      t1 = timeit([&] { gemm_f64_lds<false, true, 1, 16><<<(unsigned)gt.size(), 512>>>(dgd, dgt, 1.0, 0.0); });
      t2 = timeit([&] { schur_pairs_f64<16><<<(unsigned)pt.size(), 256>>>(dpd, dpt); });
      t3 = timeit([&] { gemm_f64_lds<false, true, 1, 16><<<(unsigned)gt.size(), 512>>>(dgd, dgt, 1.0, 0.0);
                        schur_pairs_f64<16><<<(unsigned)pt.size(), 256>>>(dpd, dpt); });
    }
    printf("BK %d\n", v == 0 ? 32 : 16);
    printf("  txy   gemm : %7.1f us  %5.1f TF executed (grid %zu)\n", t1, fl_txy / t1 / 1e6, gt.size());
    printf("  pairs      : %7.1f us  %5.1f TF executed (grid %zu)\n", t2, fl_pairs / t2 / 1e6, pt.size());
    printf("  stage      : %7.1f us  %5.1f TF algorithmic (%.2f GF)\n", t3, alg / t3 / 1e6, alg / 1e9);
  }
  return 0;
}
