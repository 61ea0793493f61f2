// Multi-word kernel check: gemv_batched<T, TA> and gemm_valu<T> on random data against a host
// evaluation in the same word type (max relative difference printed per kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels.h"
using namespace clrsdp;
using mw::dd;
using mw::qd;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

template <class T> T rnd_t() {
  T v = T(0.0);
  double s = 1.0;
  for (int q = 0; q < Num<T>::W; ++q) { v += T(((double)rand() / RAND_MAX - 0.5) * s); s *= 1e-16; }
  return v;
}
template <class T> double relerr(const T& a, const T& b) {
  T d = a - b;
  return fabs(Num<T>::hi(d)) / fmax(1e-300, fabs(Num<T>::hi(b)));
}

template <class T, bool TA>
void test_gemv(int M, int K, bool a_double = false) {
  std::vector<T> A((size_t)M * K), x(K), y(M), yh(M);
  for (auto& v : A) v = a_double ? T((double)rand() / RAND_MAX - 0.5) : rnd_t<T>();
  for (auto& v : x) v = rnd_t<T>();
  // TA: y_j = sum_k A[k + j*K] x_k (A is K x M, lda = K); else y_i = sum_k A[i + k*M] x_k
  for (int i = 0; i < M; ++i) {
    T s = T(0.0);
    for (int k = 0; k < K; ++k) s += (TA ? A[k + (size_t)i * K] : A[i + (size_t)k * M]) * x[k];
    yh[i] = s;
  }
  T *dA, *dx, *dy;
  CK(hipMalloc(&dA, A.size() * sizeof(T))); CK(hipMalloc(&dx, K * sizeof(T))); CK(hipMalloc(&dy, M * sizeof(T)));
  CK(hipMemcpy(dA, A.data(), A.size() * sizeof(T), hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, x.data(), K * sizeof(T), hipMemcpyHostToDevice));
  GemmDesc<T> g{};
  g.A = dA; g.lda = TA ? K : M; g.B = dx; g.ldb = K; g.C = dy; g.ldc = M; g.Cin = nullptr; g.ldcin = M;
  g.M = M; g.N = 1; g.K = K;
  GemmDesc<T>* dg; CK(hipMalloc(&dg, sizeof(g))); CK(hipMemcpy(dg, &g, sizeof(g), hipMemcpyHostToDevice));
  std::vector<TileRef> t;
  for (int i = 0; i < (M + 63) / 64; ++i) t.push_back(TileRef{0, i});
  TileRef* dt; CK(hipMalloc(&dt, t.size() * sizeof(TileRef)));
  CK(hipMemcpy(dt, t.data(), t.size() * sizeof(TileRef), hipMemcpyHostToDevice));
  gemv_batched<T, TA><<<(unsigned)t.size(), 256>>>(dg, dt, 1.0, 0.0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(y.data(), dy, M * sizeof(T), hipMemcpyDeviceToHost));
  double e = 0;
  for (int i = 0; i < M; ++i) e = fmax(e, relerr(y[i], yh[i]));
  printf("gemv W=%d TA=%d M=%d K=%d a_double=%d: max rel diff %.3e\n", Num<T>::W, (int)TA, M, K, (int)a_double, e);
}

template <class T, int V>
__global__ void k_slab(const T* in, int cnt, long long stride, long long n, T* out, const T* base,
                       double cbase, double csum) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  T acc = in[e];
  int i = 1;
  if (V == 1) {
    for (; i + 7 < cnt; i += 8) {
      T v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = in[(size_t)(i + u) * stride + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
  }
  for (; i < cnt; ++i) acc += in[(size_t)i * stride + e];
  if (V == 2) { out[e] = acc; return; }
  if (base) acc = base[e] * T(cbase) + acc * T(csum);
  out[e] = acc;
}
template <class T>
void test_slab(int cnt, int n) {
  std::vector<T> in((size_t)cnt * n), base(n), out(n);
  for (auto& v : in) v = rnd_t<T>();
  for (auto& v : base) v = rnd_t<T>();
  T *din, *dbase, *dout;
  CK(hipMalloc(&din, in.size() * sizeof(T))); CK(hipMalloc(&dbase, n * sizeof(T))); CK(hipMalloc(&dout, n * sizeof(T)));
  CK(hipMemcpy(din, in.data(), in.size() * sizeof(T), hipMemcpyHostToDevice));
  CK(hipMemcpy(dbase, base.data(), n * sizeof(T), hipMemcpyHostToDevice));
  for (int var = 0; var < 4; ++var) {
  if (var == 0) slab_sum<T><<<(n + 255) / 256, 256>>>(din, cnt, n, n, dout, dbase, 1.0, -1.0);
  if (var == 1) k_slab<T, 0><<<(n + 255) / 256, 256>>>(din, cnt, n, n, dout, dbase, 1.0, -1.0);
  if (var == 2) k_slab<T, 1><<<(n + 255) / 256, 256>>>(din, cnt, n, n, dout, dbase, 1.0, -1.0);
  if (var == 3) k_slab<T, 2><<<(n + 255) / 256, 256>>>(din, cnt, n, n, dout, dbase, 1.0, -1.0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), dout, n * sizeof(T), hipMemcpyDeviceToHost));
  double e = 0;
  for (int i = 0; i < n; ++i) {
    T acc = in[i];
    for (int c = 1; c < cnt; ++c) acc += in[(size_t)c * n + i];
    T ref = var == 3 ? acc : base[i] * T(1.0) + acc * T(-1.0);
    e = fmax(e, relerr(out[i], ref));
  }
  printf("slab_sum var %d W=%d cnt=%d n=%d: max rel diff %.3e\n", var, Num<T>::W, cnt, n, e);
  }
}

template <class T>
__global__ void k_ops(const T* a, const T* b, T* out, int n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  out[5 * e + 0] = a[e] + b[e];
  out[5 * e + 1] = a[e] * b[e];
  out[5 * e + 2] = a[e] * T(-1.0);
  out[5 * e + 3] = b[e] * T(1.0) + a[e] * T(-1.0);
  T acc = a[e];
  acc += b[e];
  out[5 * e + 4] = acc;
}
template <class T>
void test_ops(int n) {
  std::vector<T> a(n), b(n), out(5 * n);
  for (auto& v : a) v = rnd_t<T>();
  for (auto& v : b) v = rnd_t<T>();
  T *da, *db, *dout;
  CK(hipMalloc(&da, n * sizeof(T))); CK(hipMalloc(&db, n * sizeof(T))); CK(hipMalloc(&dout, 5 * n * sizeof(T)));
  CK(hipMemcpy(da, a.data(), n * sizeof(T), hipMemcpyHostToDevice));
  CK(hipMemcpy(db, b.data(), n * sizeof(T), hipMemcpyHostToDevice));
  k_ops<T><<<(n + 255) / 256, 256>>>(da, db, dout, n);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), dout, 5 * n * sizeof(T), hipMemcpyDeviceToHost));
  double e[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    T acc = a[i]; acc += b[i];
    T ref[5] = {a[i] + b[i], a[i] * b[i], a[i] * T(-1.0), b[i] * T(1.0) + a[i] * T(-1.0), acc};
    for (int q = 0; q < 5; ++q) e[q] = fmax(e[q], relerr(out[5 * i + q], ref[q]));
  }
  printf("ops W=%d: add %.2e mul %.2e neg %.2e lin %.2e acc %.2e\n", Num<T>::W, e[0], e[1], e[2], e[3], e[4]);
}

int main() {
  srand(3);
  test_gemv<dd, true>(4, 7);
  test_gemv<dd, false>(4, 7);
  test_gemv<qd, true>(4, 7);
  test_gemv<qd, false>(4, 7);
  test_gemv<qd, true>(100, 300);
  test_gemv<qd, false>(100, 300);
  test_gemv<qd, true>(4, 7, true);
  test_gemv<qd, false>(4, 7, true);
  test_gemv<dd, true>(4, 7, true);
  test_ops<dd>(1000);
  test_ops<qd>(1000);
  test_slab<dd>(2, 4);
  test_slab<qd>(2, 4);
  test_slab<qd>(11, 300);
  return 0;
}
