// Blocked multi-word potrf across workgroups (potrf_blk_*, round 6) against the one-CU
// chol_lookahead on a batch of random SPD n x n blocks: time per factorisation (best of 7, the
// input copied back before every run, outside the timed events), the largest |difference| of
// the L entries relative to max |L| of the block, and the failure flags.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 potrf_blk_bench.hip -o ../../microbin/potrf_blk_bench
//   microbin/potrf_blk_bench n batch
// With -DCLRSDP_LA_TRACE (binary potrf_blk_trace): chol_lookahead's per-column timestamps
// (shader clock) of the chain wave and one bulk wave, averaged over the columns and blocks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;
using mw::dd;
using mw::qd;
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

template <class P, class K>
float timeit(P prep, K k) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  prep();
  k();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 7; ++rep) {
    float ms;
    prep();
    CK(hipEventRecord(e0));
    k();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = fminf(best, ms * 1e3f);
  }
  return best;
}

template <class T, bool LDL, int NB>
void blocked(const BlkPotrfDesc<T>* bd, int nmat, int n, int* info, hipStream_t s) {
  potrf_blk_first<T, LDL, NB><<<nmat, 256, 0, s>>>(bd, info, 2);
  for (int k0 = 0; k0 + NB < n; k0 += NB) {
    const int rows = n - k0 - NB;
    potrf_blk_trsm<T, NB><<<dim3((rows + 15) / 16, nmat), 256, 0, s>>>(bd, k0);
    const int ntr = (rows + 15) / 16, DT = NB / 16;
    int tiles = 0;  // lower tiles outside the diagonal block
    for (int I = DT; I < ntr; ++I) tiles += I + 1;
    potrf_blk_update<T, LDL, NB><<<dim3(1 + tiles, nmat), 256, 0, s>>>(bd, k0, info, 2);
  }
}

template <class T, bool LDL>
void run(const char* name, int n, int nmat) {
  const size_t nn = (size_t)n * n;
  std::vector<T> h(nn * nmat);
  srand(7);
  for (int b = 0; b < nmat; ++b) {  // A = B B^T / n + 1e-3 I (condition ~1e4..1e6)
    std::vector<double> B(nn);
    for (auto& v : B) v = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        T s = T(i == j ? 1e-3 : 0.0);
        for (int k = 0; k < n; ++k) s = s + T(B[i + k * n] * B[j + k * n] / n);
        h[b * nn + i + (size_t)j * n] = s;
      }
  }
  T *dA, *dR, *dW, *dLi;
  CK(hipMalloc(&dA, h.size() * sizeof(T)));
  CK(hipMalloc(&dR, h.size() * sizeof(T)));
  CK(hipMalloc(&dW, h.size() * sizeof(T)));
  CK(hipMalloc(&dLi, (size_t)nmat * 32 * 32 * sizeof(T)));
  CK(hipMemcpy(dA, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  std::vector<MatDesc<T>> din(nmat), dout(nmat);
  std::vector<BlkPotrfDesc<T>> bdh(nmat), bdh16(nmat);
  for (int b = 0; b < nmat; ++b) {
    din[b] = {dA + b * nn, n, n};
    dout[b] = {dR + b * nn, n, n};
    bdh[b] = {dW + b * nn, dLi + (size_t)b * 32 * 32, n, n};
    bdh16[b] = {dW + b * nn, dLi + (size_t)b * 32 * 32, n, n};
  }
  MatDesc<T>*ddin, *ddout;
  BlkPotrfDesc<T>* dbd;
  CK(hipMalloc(&ddin, nmat * sizeof(MatDesc<T>)));
  CK(hipMalloc(&ddout, nmat * sizeof(MatDesc<T>)));
  CK(hipMalloc(&dbd, nmat * sizeof(BlkPotrfDesc<T>)));
  CK(hipMemcpy(ddin, din.data(), nmat * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  CK(hipMemcpy(ddout, dout.data(), nmat * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  CK(hipMemcpy(dbd, bdh.data(), nmat * sizeof(BlkPotrfDesc<T>), hipMemcpyHostToDevice));
  int* info;
  CK(hipMalloc(&info, 3 * nmat * sizeof(int)));
  auto nop = [] {};
  float tr;
  if (n > 64)
    tr = timeit(nop, [&] { chol_lookahead<T, false, LDL, 128><<<nmat, 1024>>>(ddin, nullptr, ddout, info, 2); });
  else
    tr = timeit(nop, [&] { chol_lookahead<T, false, LDL, 64><<<nmat, 1024>>>(ddin, nullptr, ddout, info, 2); });
  auto prep = [&] { CK(hipMemcpy(dW, dA, h.size() * sizeof(T), hipMemcpyDeviceToDevice)); };
  const float t32 = timeit(prep, [&] { blocked<T, LDL, 32>(dbd, nmat, n, info + nmat, 0); });
  std::vector<T> r(h.size()), w32(h.size());
  CK(hipMemcpy(w32.data(), dW, h.size() * sizeof(T), hipMemcpyDeviceToHost));
  const float t16 = timeit(prep, [&] { blocked<T, LDL, 16>(dbd, nmat, n, info + 2 * nmat, 0); });
  std::vector<T> w16(h.size());
  CK(hipMemcpy(w16.data(), dW, h.size() * sizeof(T), hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.data(), dR, h.size() * sizeof(T), hipMemcpyDeviceToHost));
  std::vector<int> hi(3 * nmat);
  CK(hipMemcpy(hi.data(), info, hi.size() * sizeof(int), hipMemcpyDeviceToHost));
  double e32 = 0.0, e16 = 0.0;
  int upper_bad = 0;
  for (int b = 0; b < nmat; ++b) {
    double mx = 0.0;
    for (size_t i = 0; i < nn; ++i) mx = fmax(mx, fabs(Num<T>::hi(r[b * nn + i])));
    for (int c = 0; c < n; ++c)
      for (int rr = 0; rr < n; ++rr) {
        const size_t i = b * nn + rr + (size_t)c * n;
        if (rr < c) {
          upper_bad += Num<T>::hi(w32[i]) != 0.0 || Num<T>::hi(w16[i]) != 0.0;
          continue;
        }
        e32 = fmax(e32, fabs(Num<T>::hi(w32[i] - r[i])) / mx);
        e16 = fmax(e16, fabs(Num<T>::hi(w16[i] - r[i])) / mx);
      }
  }
  int bad[3] = {0, 0, 0};
  for (int q = 0; q < 3; ++q)
    for (int b = 0; b < nmat; ++b) bad[q] += hi[q * nmat + b] != 0;
  printf("%s%s n=%d batch=%d: chol_lookahead %.1f us | blocked NB=32 %.1f us (max rel diff %.1e) | NB=16 %.1f us (%.1e) | nonzero above diag %d | info!=0 %d %d %d\n",
         name, LDL ? " LDL" : "", n, nmat, tr, t32, e32, t16, e16, upper_bad, bad[0], bad[1], bad[2]);
}

#ifdef CLRSDP_LA_TRACE
template <class T, bool INV, bool LDL, int NMAX, int NW, bool SKIP0 = false>
void trace_run(const char* name, int n, int nmat) {
  const size_t nn = (size_t)n * n;
  std::vector<T> h(nn * nmat);
  srand(7);
  for (int b = 0; b < nmat; ++b) {
    std::vector<double> B(nn);
    for (auto& v : B) v = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        T s = T(i == j ? 1e-3 : 0.0);
        for (int k = 0; k < n; ++k) s = s + T(B[i + k * n] * B[j + k * n] / n);
        h[b * nn + i + (size_t)j * n] = s;
      }
  }
  T *dA, *dR, *dI;
  CK(hipMalloc(&dA, h.size() * sizeof(T)));
  CK(hipMalloc(&dR, h.size() * sizeof(T)));
  CK(hipMalloc(&dI, h.size() * sizeof(T)));
  CK(hipMemcpy(dA, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  std::vector<MatDesc<T>> din(nmat), dout(nmat), dinv(nmat);
  for (int b = 0; b < nmat; ++b) {
    din[b] = {dA + b * nn, n, n};
    dout[b] = {dR + b * nn, n, n};
    dinv[b] = {dI + b * nn, n, n};
  }
  MatDesc<T>*ddin, *ddout, *ddinv;
  CK(hipMalloc(&ddin, nmat * sizeof(MatDesc<T>)));
  CK(hipMalloc(&ddout, nmat * sizeof(MatDesc<T>)));
  CK(hipMalloc(&ddinv, nmat * sizeof(MatDesc<T>)));
  CK(hipMemcpy(ddin, din.data(), nmat * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  CK(hipMemcpy(ddout, dout.data(), nmat * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  CK(hipMemcpy(ddinv, dinv.data(), nmat * sizeof(MatDesc<T>), hipMemcpyHostToDevice));
  int* info;
  CK(hipMalloc(&info, nmat * sizeof(int)));
  const float t = timeit([] {}, [&] {
    chol_lookahead<T, INV, LDL, NMAX, NW, SKIP0><<<nmat, 64 * (NW + 1)>>>(ddin, INV ? ddinv : nullptr, ddout, info, 2);
  });
  std::vector<unsigned long long> tr(64 * 16 * 128 * 4);
  CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_la_trace), tr.size() * 8));
  double acc[2][4] = {{0}}, wk[16] = {0};
  int cnt = 0;
  const int nb = nmat < 64 ? nmat : 64;
  for (int b = 0; b < nb; ++b)
    for (int j = 0; j + 2 < n && j < 127; ++j) {
      auto T0 = [&](int w, int jj, int q) { return (double)tr[((b * 16 + w) * 128 + jj) * 4 + q]; };
      for (int w = 1; w <= NW; ++w) wk[w] += T0(w, j, 3) - T0(w, j, 0);
      acc[0][0] += T0(0, j, 1) - T0(0, j, 0);      // LDS reads + update of column j+1
      acc[0][1] += T0(0, j, 2) - T0(0, j, 1);      // pivot + scaled column out
      acc[0][2] += T0(0, j, 3) - T0(0, j, 2);      // row of L^-1
      acc[0][3] += T0(0, j + 1, 0) - T0(0, j, 3);  // barrier wait
      acc[1][0] += T0(1, j, 3) - T0(1, j, 0);      // bulk work
      acc[1][1] += T0(1, j + 1, 0) - T0(1, j, 3);  // bulk barrier wait
      acc[1][2] += T0(0, j + 1, 0) - T0(0, j, 0);  // whole column
      ++cnt;
    }
  printf("%s %s%s n=%d batch=%d NMAX=%d NW=%d: %.1f us | chain: update %.0f pivot %.0f row %.0f wait %.0f | bulk work %.0f wait %.0f | column %.0f cycles\n",
         name, INV ? "INV" : "potrf", SKIP0 ? " skip0" : "", n, nmat, NMAX, NW, t, acc[0][0] / cnt, acc[0][1] / cnt, acc[0][2] / cnt,
         acc[0][3] / cnt, acc[1][0] / cnt, acc[1][1] / cnt, acc[1][2] / cnt);
  printf("   bulk work per wave:");
  for (int w = 1; w <= NW; ++w) printf(" %.0f", wk[w] / cnt);
  printf("\n");
}
int main(int argc, char** argv) {
  trace_run<qd, false, true, 64, 15, true>("qd", 51, 7);
  trace_run<qd, true, true, 64, 15>("qd", 32, 32);
  trace_run<qd, true, true, 64, 15, true>("qd", 32, 32);
  trace_run<dd, true, false, 64, 15, true>("dd", 64, 16);
  trace_run<dd, false, false, 64, 15, true>("dd", 64, 16);
  trace_run<dd, false, false, 128, 15>("dd", 127, 16);
  trace_run<dd, false, false, 64, 15>("dd", 64, 16);
  trace_run<dd, true, false, 64, 15>("dd", 64, 16);
  trace_run<dd, true, false, 32, 3>("dd", 32, 16);
  trace_run<dd, true, false, 16, 3>("dd", 16, 16);
  trace_run<qd, false, true, 64, 15>("qd", 51, 7);
  trace_run<qd, true, true, 32, 3>("qd", 32, 16);
  return 0;
}
#else
int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 127, nmat = argc > 2 ? atoi(argv[2]) : 16;
  if (n <= 128) run<dd, false>("dd", n, nmat);
  if (n <= 64) run<qd, true>("qd", n, nmat);
  return 0;
}
#endif
