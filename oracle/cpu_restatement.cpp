// cpu_restatement.cpp -- ORACLE / CPU BASELINE (test infrastructure, never the product).
//
// A C++17 + OpenMP restatement of the loop body of solverank1sdp (MPMP.jl:742-887, objectives
// 940-941), templated on the arithmetic: IEEE double, double-double and quad-double (the
// error-free-transform words of csrc/mwfloat.h, host build).  It follows oracle/mpmp_oracle.py
// function by function (each cites the MPMP.jl lines it restates) and threads over the same
// partitions as the reference: the (j,l) blocks (MPMP.jl:764, 1272, 1785), the clusters
// (1435, 1454, 1751, 1771) and the samples of each Schur block.  S_j and Q are factorised by
// partially pivoted LU as approx_lu! does (1436, 1501); X^-1 by the Cholesky inverse (spd_inv!,
// 766); the step length by Cholesky, two triangular solves and lambda_min of the symmetrised
// L^-1 dM L^-T (Householder tridiagonalisation + bisection; the reference's approx_eig_qr!
// returns the same spectrum, 1857-1870).
//
// Role: bench.py's cpu_baseline ("the reference's multithreaded CPU path timed on the GPU box's
// host cores", SURVEY.md §8d -- the Julia/Arb reference cannot run there) at the bench's own
// word type, and a fast CPU parity bridge (tests/test_cpu_restatement.py checks it against the
// Python oracle).  Built by oracle/Makefile into oracle/_build/libcpurest.so; loaded with ctypes
// by tests/ and bench.py only.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "mwfloat.h"

using mw::dd;
using mw::Num;
using mw::qd;

namespace {

template <class T>
struct Mat {
  int r = 0, c = 0;
  std::vector<T> a;
  Mat() = default;
  Mat(int r_, int c_) : r(r_), c(c_), a((size_t)r_ * c_, T(0.0)) {}
  T& operator()(int i, int j) { return a[i + (size_t)j * r]; }
  const T& operator()(int i, int j) const { return a[i + (size_t)j * r]; }
};

template <class T>
Mat<T> transpose(const Mat<T>& A) {
  Mat<T> B(A.c, A.r);
  for (int j = 0; j < A.c; ++j)
    for (int i = 0; i < A.r; ++i) B(j, i) = A(i, j);
  return B;
}

// C = A B (column-major, k-outer so the inner loop streams a column of A)
template <class T>
Mat<T> mul(const Mat<T>& A, const Mat<T>& B) {
  Mat<T> C(A.r, B.c);
  for (int j = 0; j < B.c; ++j) {
    T* cj = &C.a[(size_t)j * C.r];
    for (int k = 0; k < A.c; ++k) {
      const T bkj = B(k, j);
      const T* ak = &A.a[(size_t)k * A.r];
      for (int i = 0; i < A.r; ++i) cj[i] += ak[i] * bkj;
    }
  }
  return C;
}
// C = A^T B (dot products along contiguous columns)
template <class T>
Mat<T> mul_tn(const Mat<T>& A, const Mat<T>& B) {
  Mat<T> C(A.c, B.c);
  for (int j = 0; j < B.c; ++j)
    for (int i = 0; i < A.c; ++i) {
      T s = T(0.0);
      const T* ai = &A.a[(size_t)i * A.r];
      const T* bj = &B.a[(size_t)j * B.r];
      for (int k = 0; k < A.r; ++k) s += ai[k] * bj[k];
      C(i, j) = s;
    }
  return C;
}

template <class T>
T absv(const T& v) { return Num<T>::abs_(v); }

// ---------------------------------------------------------------- dense factorisations
// approx_lu!: A[perm] = L U, L unit lower (MPMP.jl:1436, 1501)
template <class T>
bool lu(Mat<T>& A, std::vector<int>& perm) {
  const int n = A.r;
  perm.resize(n);
  for (int i = 0; i < n; ++i) perm[i] = i;
  for (int k = 0; k < n; ++k) {
    int p = k;
    T best = absv(A(k, k));
    for (int i = k + 1; i < n; ++i)
      if (absv(A(i, k)) > best) { best = absv(A(i, k)); p = i; }
    if (!(best > T(0.0))) return false;
    if (p != k) {
      for (int j = 0; j < n; ++j) std::swap(A(k, j), A(p, j));
      std::swap(perm[k], perm[p]);
    }
    const T piv = A(k, k);
    for (int i = k + 1; i < n; ++i) A(i, k) = A(i, k) / piv;
    for (int j = k + 1; j < n; ++j) {
      const T ukj = A(k, j);
      for (int i = k + 1; i < n; ++i) A(i, j) -= A(i, k) * ukj;
    }
  }
  return true;
}
// B <- L^-1 B with L lower (unit or not): approx_solve_tril!
template <class T>
void solve_tril(const Mat<T>& L, Mat<T>& B, bool unit) {
  const int n = L.r;
  for (int j = 0; j < B.c; ++j)
    for (int i = 0; i < n; ++i) {
      T s = B(i, j);
      for (int k = 0; k < i; ++k) s -= L(i, k) * B(k, j);
      B(i, j) = unit ? s : s / L(i, i);
    }
}
// B <- U^-1 B with U upper: approx_solve_triu!
template <class T>
void solve_triu(const Mat<T>& U, Mat<T>& B) {
  const int n = U.r;
  for (int j = 0; j < B.c; ++j)
    for (int i = n - 1; i >= 0; --i) {
      T s = B(i, j);
      for (int k = i + 1; k < n; ++k) s -= U(i, k) * B(k, j);
      B(i, j) = s / U(i, i);
    }
}
// B <- U^-T B with U upper (the transposed solve of MPMP.jl:1457-1460)
template <class T>
void solve_triu_t(const Mat<T>& U, Mat<T>& B) {
  const int n = U.r;
  for (int j = 0; j < B.c; ++j)
    for (int i = 0; i < n; ++i) {
      T s = B(i, j);
      for (int k = 0; k < i; ++k) s -= U(k, i) * B(k, j);
      B(i, j) = s / U(i, i);
    }
}
template <class T>
bool cholesky(const Mat<T>& A, Mat<T>& L) {
  const int n = A.r;
  L = Mat<T>(n, n);
  for (int j = 0; j < n; ++j) {
    T s = A(j, j);
    for (int k = 0; k < j; ++k) s -= L(j, k) * L(j, k);
    if (!(s > T(0.0))) return false;
    const T d = Num<T>::sqrt_(s);
    L(j, j) = d;
    for (int i = j + 1; i < n; ++i) {
      T t = A(i, j);
      for (int k = 0; k < j; ++k) t -= L(i, k) * L(j, k);
      L(i, j) = t / d;
    }
  }
  return true;
}
// spd_inv!: X^-1 = L^-T L^-1 (MPMP.jl:766)
template <class T>
bool inv_spd(const Mat<T>& A, Mat<T>& out) {
  Mat<T> L;
  if (!cholesky(A, L)) return false;
  Mat<T> Li(A.r, A.r);
  for (int i = 0; i < A.r; ++i) Li(i, i) = T(1.0);
  solve_tril(L, Li, false);
  out = mul_tn(Li, Li);
  return true;
}

// lambda_min of a symmetric matrix: Householder tridiagonalisation, then bisection on the
// Sturm count to the word's precision
template <class T>
T eigmin_sym(Mat<T> A) {
  const int n = A.r;
  if (n == 1) return A(0, 0);
  std::vector<T> d(n), e(n, T(0.0)), v(n), p(n), w(n);
  for (int k = 0; k + 2 < n; ++k) {
    T s = T(0.0);
    for (int i = k + 1; i < n; ++i) s += A(i, k) * A(i, k);
    const T alpha0 = A(k + 1, k);
    T nrm = Num<T>::sqrt_(s);
    if (!(nrm > T(0.0))) { e[k] = T(0.0); continue; }
    const T alpha = Num<T>::hi(alpha0) > 0.0 ? -nrm : nrm;
    // v = x - alpha e1, H = I - 2 v v^T / (v^T v)
    for (int i = 0; i < n; ++i) v[i] = T(0.0);
    for (int i = k + 1; i < n; ++i) v[i] = A(i, k);
    v[k + 1] -= alpha;
    T vv = T(0.0);
    for (int i = k + 1; i < n; ++i) vv += v[i] * v[i];
    if (!(vv > T(0.0))) { e[k] = alpha; continue; }
    const T tau = T(2.0) / vv;
    // p = tau A v, K = tau/2 v^T p, w = p - K v, A -= v w^T + w v^T
    for (int i = k; i < n; ++i) {
      T t = T(0.0);
      for (int j = k + 1; j < n; ++j) t += A(i, j) * v[j];
      p[i] = tau * t;
    }
    T vp = T(0.0);
    for (int i = k + 1; i < n; ++i) vp += v[i] * p[i];
    const T K = tau * vp * T(0.5);
    for (int i = k; i < n; ++i) w[i] = p[i] - K * v[i];
    for (int j = k; j < n; ++j)
      for (int i = k; i < n; ++i) A(i, j) -= v[i] * w[j] + w[i] * v[j];
    e[k] = alpha;
  }
  for (int i = 0; i < n; ++i) d[i] = A(i, i);
  e[n - 2] = A(n - 1, n - 2);
  // Gershgorin bracket, then bisection: count(sigma) = #eigenvalues < sigma
  T lo = d[0], hi = d[0];
  for (int i = 0; i < n; ++i) {
    const T r = (i > 0 ? absv(e[i - 1]) : T(0.0)) + (i + 1 < n ? absv(e[i]) : T(0.0));
    if (d[i] - r < lo) lo = d[i] - r;
    if (d[i] + r > hi) hi = d[i] + r;
  }
  auto below = [&](const T& sg) {  // any eigenvalue < sg (LDL^T pivots, zero pivot -> -tiny)
    T q = d[0] - sg;
    if (Num<T>::hi(q) == 0.0) q = T(-1e-300);
    if (q < T(0.0)) return true;
    for (int i = 1; i < n; ++i) {
      q = (d[i] - sg) - e[i - 1] * e[i - 1] / q;
      if (Num<T>::hi(q) == 0.0) q = T(-1e-300);
      if (q < T(0.0)) return true;
    }
    return false;
  };
  for (int it = 0; it < Num<T>::BITS + 60; ++it) {
    const T mid = (lo + hi) * T(0.5);
    if (!(mid > lo) || !(mid < hi)) break;
    if (below(mid)) hi = mid;
    else lo = mid;
  }
  return (lo + hi) * T(0.5);
}

// ---------------------------------------------------------------- problem
template <class T>
struct Block {
  int j, l, m, N, del, n, K;
  Mat<T> V;              // delta x K (hcat of the v's, MPMP.jl:1249-1254)
  std::vector<T> lam;    // K
  std::vector<int> ks;   // sample of column rho
};
template <class T>
struct Cluster {
  int m, N, D, L, b0;    // b0: first block
  int64_t xoff;
  Mat<T> B;              // D x n_y
  std::vector<T> c;      // D
};

template <class T>
struct Problem {
  int J, n_y;
  std::vector<Block<T>> blk;
  std::vector<Cluster<T>> cl;
  std::vector<T> b;
  int64_t nx = 0;
  double dim = 0;
};

inline int tuple_index(int r, int s, int k, int N) { return k + (s + r * (r + 1) / 2) * N; }

template <class T>
T from_planes(const double* p, int64_t n, int64_t i) {
  T v;
  Num<T>::pack(p, n, i, &v);
  return v;
}
template <class T>
void to_planes(const T& v, double* p, int64_t n, int64_t i) { Num<T>::unpack(v, p, n, i); }

template <class T>
using Blocks = std::vector<Mat<T>>;

// ---------------------------------------------------------------- L2 functions
// dot(::BlockDiagonal, ::BlockDiagonal) MPMP.jl:205-220 (block order, fixed)
template <class T>
T dot_blocks(const Blocks<T>& A, const Blocks<T>& B) {
  T s = T(0.0);
  for (size_t q = 0; q < A.size(); ++q)
    for (size_t e = 0; e < A[q].a.size(); ++e) s += A[q].a[e] * B[q].a[e];
  return s;
}

// compute_S_integrated (MPMP.jl:1218-1414): S_j and A_Y[j][l][r][s] (K values)
template <class T>
void schur(const Problem<T>& P, const Blocks<T>& Xi, const Blocks<T>& Y, std::vector<Mat<T>>& S,
           std::vector<std::vector<std::vector<T>>>& AY) {
  const int nb = (int)P.blk.size();
  std::vector<std::vector<Mat<T>>> BX(nb), BY(nb);
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < nb; ++q) {  // Threads.@threads over (j,l) (MPMP.jl:1272)
    const Block<T>& b = P.blk[q];
    const int m = b.m, del = b.del, K = b.K;
    BX[q].resize(m * m);
    BY[q].resize(m * m);
    for (int s = 0; s < m; ++s) {
      Mat<T> Xs(b.n, del), Ys(b.n, del);
      for (int jj = 0; jj < del; ++jj)
        for (int i = 0; i < b.n; ++i) {
          Xs(i, jj) = Xi[q](i, s * del + jj);
          Ys(i, jj) = Y[q](i, s * del + jj);
        }
      const Mat<T> TX = mul(Xs, b.V), TY = mul(Ys, b.V);  // MPMP.jl:1291, 1294
      for (int r = 0; r < m; ++r) {
        Mat<T> tx(del, K), ty(del, K);
        for (int k = 0; k < K; ++k)
          for (int i = 0; i < del; ++i) {
            tx(i, k) = TX(r * del + i, k);
            ty(i, k) = TY(r * del + i, k);
          }
        BX[q][r + s * m] = mul_tn(b.V, tx);  // MPMP.jl:1300
        BY[q][r + s * m] = mul_tn(b.V, ty);  // MPMP.jl:1308
      }
    }
  }
  AY.assign(nb, {});
  for (int q = 0; q < nb; ++q) {
    const Block<T>& b = P.blk[q];
    for (int r = 0; r < b.m; ++r)
      for (int s = 0; s <= r; ++s) {
        std::vector<T> d(b.K);
        for (int i = 0; i < b.K; ++i) d[i] = BY[q][r + s * b.m](i, i);  // MPMP.jl:1320-1330
        AY[q].push_back(d);
      }
  }
  const int J = (int)P.cl.size();
  S.assign(J, Mat<T>());
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < J; ++j) {
    const Cluster<T>& c = P.cl[j];
    const int m = c.m, N = c.N, D = c.D;
    Mat<T> Sj(D, D);
    for (int l = 0; l < c.L; ++l) {
      const int q = c.b0 + l;
      const Block<T>& b = P.blk[q];
      const int K = b.K;
      auto bx = [&](int r, int s) -> const Mat<T>& { return BX[q][r + s * m]; };
      auto by = [&](int r, int s) -> const Mat<T>& { return BY[q][r + s * m]; };
      for (int r1 = 0; r1 < m; ++r1)
        for (int s1 = 0; s1 <= r1; ++s1)
          for (int r2 = 0; r2 < m; ++r2)
            for (int s2 = 0; s2 <= r2; ++s2) {
              const int h0 = tuple_index(r1, s1, 0, N), v0 = tuple_index(r2, s2, 0, N);
              // S[ver = (r2,s2,k2), hor = (r1,s1,k1)] += lambda lambda'/4 (4 pairings),
              // MPMP.jl:1373-1398, aggregated by sample
              for (int p2 = 0; p2 < K; ++p2)
                for (int p1 = 0; p1 < K; ++p1) {
                  const T t = bx(s1, r2)(p1, p2) * by(s2, r1)(p2, p1) + bx(r1, r2)(p1, p2) * by(s2, s1)(p2, p1) +
                              bx(s1, s2)(p1, p2) * by(r2, r1)(p2, p1) + bx(r1, s2)(p1, p2) * by(r2, s1)(p2, p1);
                  Sj(v0 + b.ks[p2], h0 + b.ks[p1]) += b.lam[p1] * b.lam[p2] * T(0.25) * t;
                }
            }
    }
    // keep the upper triangle and mirror it (Symmetric(S[j]), MPMP.jl:1409)
    for (int jj = 0; jj < D; ++jj)
      for (int i = jj + 1; i < D; ++i) Sj(i, jj) = Sj(jj, i);
    S[j] = std::move(Sj);
  }
}

// Tr(A_* Z) (MPMP.jl:1517-1584)
template <class T>
std::vector<T> trace_A(const Problem<T>& P, const Blocks<T>& Z) {
  std::vector<T> res(P.nx, T(0.0));
  const int J = (int)P.cl.size();
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < J; ++j) {
    const Cluster<T>& c = P.cl[j];
    for (int l = 0; l < c.L; ++l) {
      const Block<T>& b = P.blk[c.b0 + l];
      const int del = b.del;
      for (int r = 0; r < b.m; ++r)
        for (int s = 0; s <= r; ++s) {
          Mat<T> Zrs(del, del);
          for (int jj = 0; jj < del; ++jj)
            for (int i = 0; i < del; ++i) Zrs(i, jj) = Z[c.b0 + l](r * del + i, s * del + jj);
          const Mat<T> ZV = mul(Zrs, b.V);  // (V^T Z V)_{rho rho}: column sums of V .* (Z V)
          const int64_t off = c.xoff + (int64_t)(s + r * (r + 1) / 2) * c.N;
          for (int rho = 0; rho < b.K; ++rho) {
            T part = T(0.0);
            for (int i = 0; i < del; ++i) part += b.V(i, rho) * ZV(i, rho);
            res[off + b.ks[rho]] += b.lam[rho] * part;
          }
        }
    }
  }
  return res;
}
// Tr(A_* Y) from A_Y (MPMP.jl:1585-1618)
template <class T>
std::vector<T> trace_A_AY(const Problem<T>& P, const std::vector<std::vector<std::vector<T>>>& AY) {
  std::vector<T> res(P.nx, T(0.0));
  for (const Cluster<T>& c : P.cl)
    for (int l = 0; l < c.L; ++l) {
      const int q = c.b0 + l;
      const Block<T>& b = P.blk[q];
      int rs = 0;
      for (int r = 0; r < b.m; ++r)
        for (int s = 0; s <= r; ++s, ++rs)
          for (int rho = 0; rho < b.K; ++rho) {
            const int64_t t = c.xoff + tuple_index(r, s, b.ks[rho], c.N);
            res[t] += b.lam[rho] * AY[q][rs][rho];
          }
    }
  return res;
}
// sum_i a_i A_i (MPMP.jl:1621-1678)
template <class T>
Blocks<T> weighted_A(const Problem<T>& P, const std::vector<T>& a) {
  const int nb = (int)P.blk.size();
  Blocks<T> out(nb);
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < nb; ++q) {
    const Block<T>& b = P.blk[q];
    const Cluster<T>& c = P.cl[b.j];
    const int del = b.del;
    Mat<T> M(b.n, b.n);
    for (int r = 0; r < b.m; ++r)
      for (int s = 0; s <= r; ++s) {
        const int64_t off = c.xoff + (int64_t)(s + r * (r + 1) / 2) * c.N;
        Mat<T> Vw(del, b.K);
        for (int rho = 0; rho < b.K; ++rho) {
          const T w = a[off + b.ks[rho]] * b.lam[rho];
          for (int i = 0; i < del; ++i) Vw(i, rho) = b.V(i, rho) * w;
        }
        Mat<T> Q = mul(Vw, transpose(b.V));  // MPMP.jl:1654-1659
        for (int jj = 0; jj < del; ++jj)
          for (int i = 0; i < del; ++i)
            M(s * del + i, r * del + jj) = (r != s) ? Q(i, jj) * T(0.5) : Q(i, jj);  // 1661-1663
      }
    if (b.m != 1)  // Symmetric(.) keeps the upper triangle
      for (int jj = 0; jj < b.n; ++jj)
        for (int i = jj + 1; i < b.n; ++i) M(i, jj) = M(jj, i);
    out[q] = std::move(M);
  }
  return out;
}

template <class T>
struct Decomp {
  std::vector<Mat<T>> S;            // LU factors
  std::vector<std::vector<int>> perms;
  std::vector<Mat<T>> LinvB, BTUinvT;  // L^-1 P B and (B^T U^-1)^T = U^-T B
  Mat<T> Q;
  std::vector<int> qperm;
};

// compute_T_decomposition (MPMP.jl:1417-1514)
template <class T>
bool decompose(const Problem<T>& P, std::vector<Mat<T>> S, Decomp<T>& dc) {
  const int J = (int)P.cl.size();
  dc.perms.assign(J, {});
  dc.LinvB.assign(J, Mat<T>());
  dc.BTUinvT.assign(J, Mat<T>());
  std::vector<int> ok(J, 1);
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < J; ++j) {
    if (!lu(S[j], dc.perms[j])) { ok[j] = 0; continue; }  // approx_lu! 1436
    const Mat<T>& B = P.cl[j].B;
    Mat<T> W2 = B;
    solve_triu_t(S[j], W2);                                 // U^T W = B (1457-1460)
    Mat<T> W1(B.r, B.c);
    for (int jj = 0; jj < B.c; ++jj)
      for (int i = 0; i < B.r; ++i) W1(i, jj) = B(dc.perms[j][i], jj);
    solve_tril(S[j], W1, true);                             // L^-1 B[perm] (1463)
    dc.LinvB[j] = std::move(W1);
    dc.BTUinvT[j] = std::move(W2);
  }
  for (int j = 0; j < J; ++j)
    if (!ok[j]) return false;
  dc.S = std::move(S);
  std::vector<Mat<T>> part(J);
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < J; ++j) part[j] = mul_tn(dc.BTUinvT[j], dc.LinvB[j]);  // 1486-1494
  dc.Q = Mat<T>(P.n_y, P.n_y);
  for (int j = 0; j < J; ++j)
    for (size_t e = 0; e < dc.Q.a.size(); ++e) dc.Q.a[e] += part[j].a[e];
  return lu(dc.Q, dc.qperm);  // 1501
}

template <class T>
Blocks<T> symm(const Blocks<T>& Z) {
  Blocks<T> o(Z.size());
  for (size_t q = 0; q < Z.size(); ++q) {
    o[q] = Z[q];
    for (int j = 0; j < Z[q].c; ++j)
      for (int i = 0; i < Z[q].r; ++i) o[q](i, j) = (Z[q](i, j) + Z[q](j, i)) * T(0.5);
  }
  return o;
}

// compute_search_direction (MPMP.jl:1682-1824)
template <class T>
void direction(const Problem<T>& P, const Blocks<T>& Pm, const std::vector<T>& p,
               const std::vector<T>& d, const Blocks<T>& R, const Blocks<T>& Xi, const Blocks<T>& Y,
               const Decomp<T>& dc, std::vector<T>& dx, Blocks<T>& dX, std::vector<T>& dy,
               Blocks<T>& dY) {
  const int nb = (int)P.blk.size();
  Blocks<T> Z(nb);
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < nb; ++q) {  // Z = sym(X^-1 (P Y - R))  1698-1730
    Mat<T> t = mul(Pm[q], Y[q]);
    for (size_t e = 0; e < t.a.size(); ++e) t.a[e] -= R[q].a[e];
    Z[q] = mul(Xi[q], t);
  }
  Z = symm(Z);
  std::vector<T> tr = trace_A(P, Z);
  std::vector<T> rhs(P.nx);
  for (int64_t i = 0; i < P.nx; ++i) rhs[i] = -d[i] - tr[i];  // 1733-1739
  const int J = (int)P.cl.size();
  std::vector<Mat<T>> tx(J);
  std::vector<std::vector<T>> ty(J);
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < J; ++j) {  // 1751-1759
    const Cluster<T>& c = P.cl[j];
    Mat<T> t(c.D, 1);
    for (int i = 0; i < c.D; ++i) t(i, 0) = rhs[c.xoff + dc.perms[j][i]];
    solve_tril(dc.S[j], t, true);
    ty[j] = mul_tn(dc.BTUinvT[j], t).a;
    tx[j] = std::move(t);
  }
  std::vector<T> acc(P.n_y, T(0.0));
  for (int j = 0; j < J; ++j)
    for (int i = 0; i < P.n_y; ++i) acc[i] += ty[j][i];
  Mat<T> r(P.n_y, 1);
  for (int i = 0; i < P.n_y; ++i) r(i, 0) = p[i] - acc[i];  // 1761
  Mat<T> rp(P.n_y, 1);
  for (int i = 0; i < P.n_y; ++i) rp(i, 0) = r(dc.qperm[i], 0);
  solve_tril(dc.Q, rp, true);  // approx_solve_lu_precomp! 1764
  solve_triu(dc.Q, rp);
  dy = rp.a;
  dx.assign(P.nx, T(0.0));
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < J; ++j) {  // 1771-1773
    const Cluster<T>& c = P.cl[j];
    Mat<T> u = mul(dc.LinvB[j], rp);
    for (int i = 0; i < c.D; ++i) u(i, 0) += tx[j](i, 0);
    solve_triu(dc.S[j], u);
    for (int i = 0; i < c.D; ++i) dx[c.xoff + i] = u(i, 0);
  }
  Blocks<T> WA = weighted_A(P, dx);  // 1779-1786
  dX.assign(nb, Mat<T>());
  Blocks<T> dYr(nb);
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < nb; ++q) {
    Mat<T> dXq = WA[q];
    for (size_t e = 0; e < dXq.a.size(); ++e) dXq.a[e] += Pm[q].a[e];
    Mat<T> t = mul(dXq, Y[q]);  // dY = sym(X^-1 (R - dX Y))  1789-1821
    for (size_t e = 0; e < t.a.size(); ++e) t.a[e] = R[q].a[e] - t.a[e];
    dYr[q] = mul(Xi[q], t);
    dX[q] = std::move(dXq);
  }
  dY = symm(dYr);
}

// compute_step_length (MPMP.jl:1829-1898); false when a Cholesky fails
template <class T>
bool step_length(const Blocks<T>& M, const Blocks<T>& dM, const T& gamma, T& alpha) {
  const int nb = (int)M.size();
  std::vector<T> mins(nb);
  std::vector<int> ok(nb, 1);
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < nb; ++q) {
    Mat<T> L;
    if (!cholesky(M[q], L)) { ok[q] = 0; continue; }  // cho! 1846
    Mat<T> t = dM[q];
    solve_tril(L, t, false);        // 1853
    Mat<T> tt = transpose(t);
    solve_tril(L, tt, false);       // 1854-1856
    mins[q] = eigmin_sym(symm(Blocks<T>{tt})[0]);
  }
  T mn = T(1e300);
  for (int q = 0; q < nb; ++q) {
    if (!ok[q]) return false;
    if (mins[q] < mn) mn = mins[q];
  }
  alpha = (mn > -gamma) ? T(1.0) : -gamma / mn;  // 1893-1897
  return true;
}

template <class T>
T max_abs(const std::vector<T>& v) {
  T m = T(0.0);
  for (const T& x : v)
    if (absv(x) > m) m = absv(x);
  return m;
}
template <class T>
T max_abs(const Blocks<T>& B) {
  T m = T(0.0);
  for (const Mat<T>& b : B)
    for (const T& x : b.a)
      if (absv(x) > m) m = absv(x);
  return m;
}

// One loop body (MPMP.jl:755-887) and the objectives (940-941); log[8] =
// mu, alpha_p, alpha_d, beta_c, p_obj, d_obj, P_err, d_err.  Returns 0, or the reference's
// failure: 3 X^-1, 4 S, 6 step length.
template <class T>
int iteration(const Problem<T>& P, std::vector<T>& x, Blocks<T>& X, std::vector<T>& y, Blocks<T>& Y,
              const T& beta_inf, const T& beta_feas, const T& gamma, bool pd_feas, T* log) {
  const int nb = (int)P.blk.size();
  const T mu = dot_blocks(X, Y) / T(P.dim);                     // 755
  const T mu_p = pd_feas ? T(0.0) : beta_inf * mu;              // 756
  Blocks<T> R(nb), Xi(nb);
  std::vector<int> ok(nb, 1);
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < nb; ++q) {
    R[q] = mul(X[q], Y[q]);                                      // R = mu_p I - X Y  (1189-1201)
    for (size_t e = 0; e < R[q].a.size(); ++e) R[q].a[e] = -R[q].a[e];
    for (int i = 0; i < R[q].r; ++i) R[q](i, i) += mu_p;
    if (!inv_spd(X[q], Xi[q])) ok[q] = 0;                        // 762-801
  }
  for (int q = 0; q < nb; ++q)
    if (!ok[q]) return 3;
  std::vector<Mat<T>> S;
  std::vector<std::vector<std::vector<T>>> AY;
  schur(P, Xi, Y, S, AY);                                        // 806
  Decomp<T> dc;
  if (!decompose(P, S, dc)) return 4;
  // residuals (MPMP.jl:1107-1144): P = sum x_i A_i - X, d = c - B y - Tr(A_* Y), p = b - B^T x
  Blocks<T> Pm = weighted_A(P, x);
  for (int q = 0; q < nb; ++q)
    for (size_t e = 0; e < Pm[q].a.size(); ++e) Pm[q].a[e] -= X[q].a[e];
  std::vector<T> trY = trace_A_AY(P, AY);
  std::vector<T> d(P.nx), p(P.n_y);
  for (const Cluster<T>& c : P.cl)
    for (int i = 0; i < c.D; ++i) {
      T s = c.c[i];
      for (int k = 0; k < P.n_y; ++k) s -= c.B(i, k) * y[k];
      d[c.xoff + i] = s - trY[c.xoff + i];
    }
  for (int k = 0; k < P.n_y; ++k) p[k] = T(0.0);
  for (const Cluster<T>& c : P.cl)
    for (int k = 0; k < P.n_y; ++k) {
      T s = T(0.0);
      for (int i = 0; i < c.D; ++i) s += c.B(i, k) * x[c.xoff + i];
      p[k] = p[k] - s;
    }
  for (int k = 0; k < P.n_y; ++k) p[k] = p[k] + P.b[k];
  std::vector<T> dx, dy;
  Blocks<T> dX, dY;
  direction(P, Pm, p, d, R, Xi, Y, dc, dx, dX, dy, dY);        // predictor 818
  T xdy = T(0.0);
  for (int q = 0; q < nb; ++q)
    for (size_t e = 0; e < X[q].a.size(); ++e) xdy += (X[q].a[e] + dX[q].a[e]) * (Y[q].a[e] + dY[q].a[e]);
  const T r = xdy / (mu * T(P.dim));                             // 832
  const T beta = r < T(1.0) ? r * r : r;                         // 833
  T beta_c;
  if (pd_feas) {
    beta_c = beta_feas > beta ? beta_feas : beta;
    if (beta_c > T(1.0)) beta_c = T(1.0);
  } else {
    beta_c = beta_inf > beta ? beta_inf : beta;
  }
  const T mu_c = beta_c * mu;                                    // 837
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < nb; ++q) {                                 // R = mu_c I - XY - dX dY (1203-1215)
    Mat<T> a = mul(X[q], Y[q]), b2 = mul(dX[q], dY[q]);
    for (size_t e = 0; e < a.a.size(); ++e) R[q].a[e] = -a.a[e] - b2.a[e];
    for (int i = 0; i < R[q].r; ++i) R[q](i, i) += mu_c;
  }
  direction(P, Pm, p, d, R, Xi, Y, dc, dx, dX, dy, dY);        // corrector 846
  T ap, ad;
  if (!step_length(X, dX, gamma, ap) || !step_length(Y, dY, gamma, ad)) return 6;  // 863-866
  if (pd_feas) {
    const T mn = ad < ap ? ad : ap;
    ap = mn;
    ad = mn;
  }
  for (int64_t i = 0; i < P.nx; ++i) x[i] += ap * dx[i];      // 877-887
  for (int k = 0; k < P.n_y; ++k) y[k] += ad * dy[k];
  for (int q = 0; q < nb; ++q)
    for (size_t e = 0; e < X[q].a.size(); ++e) {
      X[q].a[e] += ap * dX[q].a[e];
      Y[q].a[e] += ad * dY[q].a[e];
    }
  T cx = T(0.0), by = T(0.0);
  for (const Cluster<T>& c : P.cl)
    for (int i = 0; i < c.D; ++i) cx += c.c[i] * x[c.xoff + i];  // 940-941 (b0 = 0, C = 0)
  for (int k = 0; k < P.n_y; ++k) by += P.b[k] * y[k];
  log[0] = mu; log[1] = ap; log[2] = ad; log[3] = beta_c; log[4] = cx; log[5] = by;
  log[6] = max_abs(Pm) > max_abs(p) ? max_abs(Pm) : max_abs(p);
  log[7] = max_abs(d);
  return 0;
}

template <class T>
int run(int64_t J, int64_t n_y, const int64_t* m, const int64_t* L, const int64_t* Ns,
        const int64_t* delta, const int64_t* ranks, const double* V, const double* lam, const double* B,
        const double* c, const double* b, double* xs, double* Xs, double* ys, double* Ys,
        const double* prm, int iterations, double* logs, double* seconds) {
  Problem<T> P;
  P.J = (int)J;
  P.n_y = (int)n_y;
  int64_t tot_V = 0, tot_K = 0, tot_B = 0, tot_x = 0, tot_blk = 0, g = 0, rk = 0;
  // totals first (the planes' lengths)
  {
    int64_t gg = 0, rr = 0;
    for (int64_t j = 0; j < J; ++j) {
      const int64_t D = m[j] * (m[j] + 1) / 2 * Ns[j];
      tot_x += D;
      tot_B += D * n_y;
      for (int64_t l = 0; l < L[j]; ++l, ++gg) {
        int64_t K = 0;
        for (int64_t k = 0; k < Ns[j]; ++k) K += ranks[rr + k];
        rr += Ns[j];
        tot_V += delta[gg] * K;
        tot_K += K;
        tot_blk += (m[j] * delta[gg]) * (m[j] * delta[gg]);
      }
    }
  }
  int64_t ov = 0, ok_ = 0, ob = 0, ox = 0, oblk = 0;
  for (int64_t j = 0; j < J; ++j) {
    Cluster<T> cl;
    cl.m = (int)m[j];
    cl.N = (int)Ns[j];
    cl.D = (int)(m[j] * (m[j] + 1) / 2 * Ns[j]);
    cl.L = (int)L[j];
    cl.b0 = (int)P.blk.size();
    cl.xoff = ox;
    cl.B = Mat<T>(cl.D, (int)n_y);
    for (int64_t e = 0; e < (int64_t)cl.D * n_y; ++e) cl.B.a[e] = from_planes<T>(B, tot_B, ob + e);
    cl.c.resize(cl.D);
    for (int i = 0; i < cl.D; ++i) cl.c[i] = from_planes<T>(c, tot_x, ox + i);
    for (int64_t l = 0; l < L[j]; ++l, ++g) {
      Block<T> bk;
      bk.j = (int)j; bk.l = (int)l; bk.m = cl.m; bk.N = cl.N; bk.del = (int)delta[g];
      bk.n = bk.m * bk.del;
      int K = 0;
      for (int k = 0; k < cl.N; ++k) {
        for (int q = 0; q < ranks[rk + k]; ++q) bk.ks.push_back(k);
        K += (int)ranks[rk + k];
      }
      rk += cl.N;
      bk.K = K;
      bk.V = Mat<T>(bk.del, K);
      for (int64_t e = 0; e < (int64_t)bk.del * K; ++e) bk.V.a[e] = from_planes<T>(V, tot_V, ov + e);
      bk.lam.resize(K);
      for (int q = 0; q < K; ++q) bk.lam[q] = from_planes<T>(lam, tot_K, ok_ + q);
      ov += (int64_t)bk.del * K;
      ok_ += K;
      P.dim += bk.n;
      P.blk.push_back(std::move(bk));
    }
    ob += (int64_t)cl.D * n_y;
    ox += cl.D;
    P.cl.push_back(std::move(cl));
  }
  P.nx = tot_x;
  P.b.resize(n_y);
  for (int k = 0; k < n_y; ++k) P.b[k] = from_planes<T>(b, n_y, k);
  // state
  std::vector<T> x(tot_x), y(n_y);
  for (int64_t i = 0; i < tot_x; ++i) x[i] = from_planes<T>(xs, tot_x, i);
  for (int k = 0; k < n_y; ++k) y[k] = from_planes<T>(ys, n_y, k);
  const int nb = (int)P.blk.size();
  Blocks<T> X(nb), Y(nb);
  for (int q = 0; q < nb; ++q) {
    const int n = P.blk[q].n;
    X[q] = Mat<T>(n, n);
    Y[q] = Mat<T>(n, n);
    for (int64_t e = 0; e < (int64_t)n * n; ++e) {
      X[q].a[e] = from_planes<T>(Xs, tot_blk, oblk + e);
      Y[q].a[e] = from_planes<T>(Ys, tot_blk, oblk + e);
    }
    oblk += (int64_t)n * n;
  }
  // beta_infeasible, beta_feasible, gamma: w planes of 3 values (exact limbs of the decimal
  // parameters, as clrsdp_params); then the two error thresholds (doubles)
  const T beta_inf = from_planes<T>(prm, 3, 0), beta_feas = from_planes<T>(prm, 3, 1),
          gamma = from_planes<T>(prm, 3, 2);
  const double* thr = prm + 3 * Num<T>::W;
  bool pd_feas = false;
  const auto t0 = std::chrono::steady_clock::now();
  int rc = 0, done = 0;
  for (int it = 0; it < iterations; ++it) {
    T lg[8];
    rc = iteration(P, x, X, y, Y, beta_inf, beta_feas, gamma, pd_feas, lg);
    if (rc) break;
    for (int q = 0; q < 8; ++q) to_planes(lg[q], logs + (size_t)it * 8 * Num<T>::W, 8, q);
    // check_pd_feasibility (MPMP.jl:949-953) with the primal / dual error thresholds prm[3..4]
    pd_feas = Num<T>::hi(lg[6]) < thr[0] && Num<T>::hi(lg[7]) < thr[1];
    ++done;
  }
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (int64_t i = 0; i < tot_x; ++i) to_planes(x[i], xs, tot_x, i);
  for (int k = 0; k < n_y; ++k) to_planes(y[k], ys, n_y, k);
  oblk = 0;
  for (int q = 0; q < nb; ++q) {
    for (size_t e = 0; e < X[q].a.size(); ++e) {
      to_planes(X[q].a[e], Xs, tot_blk, oblk + (int64_t)e);
      to_planes(Y[q].a[e], Ys, tot_blk, oblk + (int64_t)e);
    }
    oblk += (int64_t)X[q].a.size();
  }
  return rc ? -rc : done;
}

}  // namespace

extern "C" {
// Run `iterations` loop bodies from the given state (planar limbs, the layout of
// clrsdp_upload_constraints / clrsdp_set_state; the state is updated in place).  prm = w planes
// of {beta_infeasible, beta_feasible, gamma}, then {primal_error_threshold,
// dual_error_threshold} as doubles.  Returns the number of bodies completed, or
// -code of the reference's failure (3 X^-1, 4 S/Q LU, 6 step length).  Per iteration `it`,
// logs + 8 w it holds w planes of 8 values (w = words): mu, alpha_p, alpha_d, beta_c, <c,x>,
// <b,y>, max|P|,|p|, max|d|.  *seconds: wall time of the loop.  threads <= 0: OpenMP's
// default.
int cpurest_run(int words, int threads, int64_t J, int64_t n_y, const int64_t* m, const int64_t* L,
                const int64_t* N, const int64_t* delta, const int64_t* ranks, const double* V,
                const double* lam, const double* B, const double* c, const double* b, double* x,
                double* X, double* y, double* Y, const double* prm, int iterations,
                double* logs, double* seconds) {
  if (threads > 0) omp_set_num_threads(threads);
  if (words == 1)
    return run<double>(J, n_y, m, L, N, delta, ranks, V, lam, B, c, b, x, X, y, Y, prm, iterations,
                       logs, seconds);
  if (words == 2)
    return run<dd>(J, n_y, m, L, N, delta, ranks, V, lam, B, c, b, x, X, y, Y, prm, iterations,
                   logs, seconds);
  if (words == 4)
    return run<qd>(J, n_y, m, L, N, delta, ranks, V, lam, B, c, b, x, X, y, Y, prm, iterations,
                   logs, seconds);
  return -1;
}
int cpurest_max_threads(void) { return omp_get_max_threads(); }
}
