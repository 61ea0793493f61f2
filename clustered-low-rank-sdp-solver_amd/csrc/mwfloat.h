// mwfloat.h -- fixed-width multi-word floating point held in registers (host + device).
//
// Replaces the Arb midpoint arithmetic of the reference (every heavy Arb product in MPMP.jl is
// an `approx_*` midpoint product followed by `get_mid!`) with
//   double  : IEEE binary64                       (53-bit significand)
//   dd      : double-double, unevaluated sum hi+lo (~106-bit significand)
// built from error-free transformations (two-sum, and two-prod via fused multiply-add).
// The algorithms are the published double-double algorithms of Dekker (1971) and of Hida, Li &
// Bailey's QD library ("Algorithms for quad-double precision floating point arithmetic",
// ARITH-15, 2001): accurate ("IEEE") addition, FMA-based multiplication, Newton division and
// square root.  Every kernel of the solver is a template on the word type T.
#pragma once
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

#define MW_HD __host__ __device__ __forceinline__
// Error-free transformations must not be contracted into FMAs by the compiler (hipcc's default
// -ffp-contract=fast-honor-pragmas would fuse e.g. `a.hi*b.hi + p2` inside quick_two_sum and
// silently lose the low word).  Every multi-word function body starts with this pragma.
#define MW_EXACT _Pragma("clang fp contract(off)")

namespace mw {

MW_HD double two_sum(double a, double b, double& err) {
  MW_EXACT
  double s = a + b;
  double bb = s - a;
  err = (a - (s - bb)) + (b - bb);
  return s;
}
MW_HD double quick_two_sum(double a, double b, double& err) {
  MW_EXACT
  double s = a + b;
  err = b - (s - a);
  return s;
}
MW_HD double two_prod(double a, double b, double& err) {
  MW_EXACT
  double p = a * b;
  err = fma(a, b, -p);
  return p;
}

struct dd {
  double hi, lo;
  dd() = default;
  MW_HD dd(double h) : hi(h), lo(0.0) {}
  MW_HD dd(double h, double l) : hi(h), lo(l) {}
};

MW_HD dd operator+(const dd& a, const dd& b) {
  MW_EXACT
  double s2, t2;
  double s1 = two_sum(a.hi, b.hi, s2);
  double t1 = two_sum(a.lo, b.lo, t2);
  s2 += t1;
  s1 = quick_two_sum(s1, s2, s2);
  s2 += t2;
  s1 = quick_two_sum(s1, s2, s2);
  return dd(s1, s2);
}
MW_HD dd operator-(const dd& a) {
  MW_EXACT return dd(-a.hi, -a.lo); }
MW_HD dd operator-(const dd& a, const dd& b) {
  MW_EXACT return a + (-b); }
MW_HD dd operator*(const dd& a, const dd& b) {
  MW_EXACT
  double p2;
  double p1 = two_prod(a.hi, b.hi, p2);
  p2 = fma(a.hi, b.lo, p2);
  p2 = fma(a.lo, b.hi, p2);
  p1 = quick_two_sum(p1, p2, p2);
  return dd(p1, p2);
}
MW_HD dd operator*(const dd& a, double b) {
  MW_EXACT
  double p2;
  double p1 = two_prod(a.hi, b, p2);
  p2 = fma(a.lo, b, p2);
  p1 = quick_two_sum(p1, p2, p2);
  return dd(p1, p2);
}
MW_HD dd operator/(const dd& a, const dd& b) {
  MW_EXACT
  // long division: q1 = a/b, r = a - q1 b, q2 = r/b, r -= q2 b, q3 = r/b
  double q1 = a.hi / b.hi;
  dd r = a - b * q1;
  double q2 = r.hi / b.hi;
  r = r - b * q2;
  double q3 = r.hi / b.hi;
  double e;
  q1 = quick_two_sum(q1, q2, e);
  return dd(q1, e) + dd(q3);
}
MW_HD dd& operator+=(dd& a, const dd& b) {
  MW_EXACT a = a + b; return a; }
MW_HD dd& operator-=(dd& a, const dd& b) {
  MW_EXACT a = a - b; return a; }
MW_HD dd& operator*=(dd& a, const dd& b) {
  MW_EXACT a = a * b; return a; }
MW_HD dd& operator/=(dd& a, const dd& b) {
  MW_EXACT a = a / b; return a; }
MW_HD bool operator<(const dd& a, const dd& b) {
  MW_EXACT return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
MW_HD bool operator>(const dd& a, const dd& b) {
  MW_EXACT return b < a; }
MW_HD bool operator<=(const dd& a, const dd& b) {
  MW_EXACT return !(b < a); }
MW_HD bool operator>=(const dd& a, const dd& b) {
  MW_EXACT return !(a < b); }
MW_HD bool operator==(const dd& a, const dd& b) {
  MW_EXACT return a.hi == b.hi && a.lo == b.lo; }
MW_HD bool operator!=(const dd& a, const dd& b) {
  MW_EXACT return !(a == b); }

MW_HD dd sqrt_dd(const dd& a) {
  MW_EXACT
  if (!(a.hi > 0.0)) return dd(a.hi == 0.0 ? 0.0 : NAN);
  // one Newton step on x = sqrt(a.hi):  sqrt(a) ~ x + (a - x^2) / (2x)
  double x = sqrt(a.hi);
  double e;
  double p = two_prod(x, x, e);
  dd d = a - dd(p, e);
  return dd(x) + dd(d.hi / (2.0 * x));
}

// ---- word-type traits used by every kernel -------------------------------------------------
template <class T> struct Num;

template <> struct Num<double> {
  static constexpr int W = 1;
  static constexpr int BITS = 53;
  MW_HD static double hi(double v) { return v; }
  MW_HD static double from(double v) { return v; }
  MW_HD static double sqrt_(double v) { return sqrt(v); }
  MW_HD static double abs_(double v) { return fabs(v); }
  MW_HD static double eps() { return 1.1102230246251565e-16; }
  static void pack(const double* planes, int64_t n, int64_t i, double* out) { *out = planes[i]; }
  static void unpack(double v, double* planes, int64_t n, int64_t i) { planes[i] = v; }
};

template <> struct Num<dd> {
  static constexpr int W = 2;
  static constexpr int BITS = 106;
  MW_HD static double hi(const dd& v) { return v.hi; }
  MW_HD static dd from(double v) { return dd(v); }
  MW_HD static dd sqrt_(const dd& v) { return sqrt_dd(v); }
  MW_HD static dd abs_(const dd& v) { return v.hi < 0.0 ? -v : v; }
  MW_HD static double eps() { return 1.2325951644078309e-32; }
  static void pack(const double* planes, int64_t n, int64_t i, dd* out) {
    double e;
    double s = two_sum(planes[i], planes[n + i], e);
    *out = dd(s, e);
  }
  static void unpack(const dd& v, double* planes, int64_t n, int64_t i) {
    planes[i] = v.hi;
    planes[n + i] = v.lo;
  }
};

}  // namespace mw
