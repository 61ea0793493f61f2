// mwfloat.h -- fixed-width multi-word floating point held in registers (host + device).
//
// Replaces the Arb midpoint arithmetic of the reference (every heavy Arb product in MPMP.jl is
// an `approx_*` midpoint product followed by `get_mid!`) with
//   double  : IEEE binary64                       (53-bit significand)
//   dd      : double-double, unevaluated sum hi+lo (~106-bit significand)
//   qd      : quad-double, unevaluated sum of four doubles (~212-bit significand)
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
// a - b c for the trailing updates of the factorisations (round 6): the product's words are not
// renormalised and the subtraction is the QD library's "sloppy" double-double addition (one
// two-sum of the leading words, the low words added plainly): 15 operations against 27 for
// a - (b * c) with the accurate addition.  Its error is below ~2 u^2 (|a| + |b c|) (u = 2^-53)
// -- an absolute bound, not one relative to the result -- which is the componentwise bound the
// backward-error analysis of Cholesky asks of every update, so the factor stays backward stable
// at double-double precision while the bulk update (VALU-issue bound) runs ~1.8x fewer
// instructions.
MW_HD dd fms_fast(const dd& a, const dd& b, const dd& c) {
  MW_EXACT
  double p2;
  const double p1 = two_prod(b.hi, c.hi, p2);
  p2 = fma(b.hi, c.lo, p2);
  p2 = fma(b.lo, c.hi, p2);
  double e;
  double s = two_sum(a.hi, -p1, e);
  e += a.lo - p2;
  s = quick_two_sum(s, e, e);
  return dd(s, e);
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


// ---- quad-double ----------------------------------------------------------------------------
// Hida, Li & Bailey (ARITH-15, 2001): three-sum networks, the five-term renormalisation,
// "sloppy" addition (error bounded relative to |a| + |b|, like the midpoint products it
// replaces), the O(eps^3)-truncated multiplication, long division and Newton square root.
MW_HD void three_sum(double& a, double& b, double& c) {
  MW_EXACT
  double t1, t2, t3;
  t1 = two_sum(a, b, t2);
  a = two_sum(c, t1, t3);
  b = two_sum(t2, t3, c);
}
MW_HD void three_sum2(double& a, double& b, double& c) {
  MW_EXACT
  double t1, t2, t3;
  t1 = two_sum(a, b, t2);
  a = two_sum(c, t1, t3);
  b = t2 + t3;
}

struct qd {
  double x[4];
  qd() = default;
  MW_HD qd(double h) : x{h, 0.0, 0.0, 0.0} {}
  MW_HD qd(double a, double b, double c, double d) : x{a, b, c, d} {}
  MW_HD qd(const dd& v) : x{v.hi, v.lo, 0.0, 0.0} {}
};

// five components (non-increasing magnitude up to overlap) -> four non-overlapping ones.
// Branch-free: a bottom-up quick-two-sum pass (as in the published renormalisation), then a
// top-down two-sum pass that makes the words non-overlapping.  The published version skips
// zero words with data-dependent branches to keep the representation dense; here a zero word
// may stay in the middle (no information is lost, the value is the same).
MW_HD qd qd_renorm(double c0, double c1, double c2, double c3, double c4) {
  MW_EXACT
  double s0, s1, s2, s3, t;
  s0 = quick_two_sum(c3, c4, c4);
  s0 = quick_two_sum(c2, s0, c3);
  s0 = quick_two_sum(c1, s0, c2);
  c0 = quick_two_sum(c0, s0, c1);
  s1 = two_sum(c1, c2, t);
  s2 = two_sum(t, c3, t);
  s3 = t + c4;
  // one more pass so that s1..s3 do not overlap after the cascade above
  s1 = quick_two_sum(c0, s1, t);
  s0 = s1;
  s1 = two_sum(t, s2, t);
  s2 = two_sum(t, s3, s3);
  return qd(s0, s1, s2, s3);
}

MW_HD qd operator+(const qd& a, const qd& b) {
  MW_EXACT
  double s0, s1, s2, s3, t0, t1, t2, t3;
  s0 = two_sum(a.x[0], b.x[0], t0);
  s1 = two_sum(a.x[1], b.x[1], t1);
  s2 = two_sum(a.x[2], b.x[2], t2);
  s3 = two_sum(a.x[3], b.x[3], t3);
  s1 = two_sum(s1, t0, t0);
  three_sum(s2, t0, t1);
  three_sum2(s3, t0, t2);
  t0 = t0 + t1 + t3;
  return qd_renorm(s0, s1, s2, s3, t0);
}
MW_HD qd operator-(const qd& a) {
  MW_EXACT return qd(-a.x[0], -a.x[1], -a.x[2], -a.x[3]); }
MW_HD qd operator-(const qd& a, const qd& b) {
  MW_EXACT return a + (-b); }
MW_HD qd operator*(const qd& a, double b) {
  MW_EXACT
  double p0, p1, p2, p3, q0, q1, q2, s0, s1, s2, s3, s4;
  p0 = two_prod(a.x[0], b, q0);
  p1 = two_prod(a.x[1], b, q1);
  p2 = two_prod(a.x[2], b, q2);
  p3 = a.x[3] * b;
  s0 = p0;
  s1 = two_sum(q0, p1, s2);
  three_sum(s2, q1, p2);
  three_sum2(q1, q2, p3);
  s3 = q1;
  s4 = q2 + p2;
  return qd_renorm(s0, s1, s2, s3, s4);
}
MW_HD qd operator*(const qd& a, const qd& b) {
  MW_EXACT
  double p0, p1, p2, p3, p4, p5, q0, q1, q2, q3, q4, q5, t0, t1, s0, s1, s2;
  p0 = two_prod(a.x[0], b.x[0], q0);
  p1 = two_prod(a.x[0], b.x[1], q1);
  p2 = two_prod(a.x[1], b.x[0], q2);
  p3 = two_prod(a.x[0], b.x[2], q3);
  p4 = two_prod(a.x[1], b.x[1], q4);
  p5 = two_prod(a.x[2], b.x[0], q5);
  three_sum(p1, p2, q0);
  // six-three sum of p2, q1, q2, p3, p4, p5
  three_sum(p2, q1, q2);
  three_sum(p3, p4, p5);
  s0 = two_sum(p2, p3, t0);
  s1 = two_sum(q1, p4, t1);
  s2 = q2 + p5;
  s1 = two_sum(s1, t0, t0);
  s2 += (t0 + t1);
  // O(eps^3) terms
  s1 += a.x[0] * b.x[3] + a.x[1] * b.x[2] + a.x[2] * b.x[1] + a.x[3] * b.x[0] + q0 + q3 + q4 + q5;
  return qd_renorm(p0, p1, s0, s1, s2);
}
MW_HD qd operator/(const qd& a, const qd& b) {
  MW_EXACT
  // long division: q_k = r_0 / b_0, r -= b q_k
  double q0 = a.x[0] / b.x[0];
  qd r = a - b * q0;
  double q1 = r.x[0] / b.x[0];
  r = r - b * q1;
  double q2 = r.x[0] / b.x[0];
  r = r - b * q2;
  double q3 = r.x[0] / b.x[0];
  r = r - b * q3;
  double q4 = r.x[0] / b.x[0];
  return qd_renorm(q0, q1, q2, q3, q4);
}
MW_HD qd& operator+=(qd& a, const qd& b) {
  MW_EXACT a = a + b; return a; }
MW_HD qd& operator-=(qd& a, const qd& b) {
  MW_EXACT a = a - b; return a; }
MW_HD qd& operator*=(qd& a, const qd& b) {
  MW_EXACT a = a * b; return a; }
MW_HD qd& operator/=(qd& a, const qd& b) {
  MW_EXACT a = a / b; return a; }
MW_HD bool operator<(const qd& a, const qd& b) {
  MW_EXACT
  return a.x[0] < b.x[0] ||
         (a.x[0] == b.x[0] && (a.x[1] < b.x[1] ||
                               (a.x[1] == b.x[1] && (a.x[2] < b.x[2] ||
                                                     (a.x[2] == b.x[2] && a.x[3] < b.x[3])))));
}
MW_HD bool operator>(const qd& a, const qd& b) {
  MW_EXACT return b < a; }
MW_HD bool operator<=(const qd& a, const qd& b) {
  MW_EXACT return !(b < a); }
MW_HD bool operator>=(const qd& a, const qd& b) {
  MW_EXACT return !(a < b); }
MW_HD bool operator==(const qd& a, const qd& b) {
  MW_EXACT return a.x[0] == b.x[0] && a.x[1] == b.x[1] && a.x[2] == b.x[2] && a.x[3] == b.x[3]; }
MW_HD bool operator!=(const qd& a, const qd& b) {
  MW_EXACT return !(a == b); }

MW_HD qd sqrt_qd(const qd& a) {
  MW_EXACT
  if (!(a.x[0] > 0.0)) return qd(a.x[0] == 0.0 ? 0.0 : NAN);
  // Newton on r = 1/sqrt(a): r += r (1/2 - (a/2) r^2), three steps (53 -> 106 -> 212 bits)
  const qd h = a * 0.5;
  qd r(1.0 / sqrt(a.x[0]));
  for (int it = 0; it < 3; ++it) r = r + r * (qd(0.5) - h * (r * r));
  return a * r;
}

// ---- component-wise select ------------------------------------------------------------------
// c ? a : b on the limbs.  A C++ ternary on the structs is lowered to a select of the operands'
// addresses, which keeps them in memory (scratch on the device: eigmin_lds2<qd> spilled 172
// B/lane, vec_reduce<qd> 304); selecting each limb keeps everything in registers.
MW_HD double sel(bool c, double a, double b) { return c ? a : b; }
MW_HD dd sel(bool c, const dd& a, const dd& b) { return dd(c ? a.hi : b.hi, c ? a.lo : b.lo); }
MW_HD qd sel(bool c, const qd& a, const qd& b) {
  return qd(c ? a.x[0] : b.x[0], c ? a.x[1] : b.x[1], c ? a.x[2] : b.x[2], c ? a.x[3] : b.x[3]);
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
  MW_HD static dd abs_(const dd& v) { return sel(v.hi < 0.0, -v, v); }
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


template <> struct Num<qd> {
  static constexpr int W = 4;
  static constexpr int BITS = 212;
  MW_HD static double hi(const qd& v) { return v.x[0]; }
  MW_HD static qd from(double v) { return qd(v); }
  MW_HD static qd sqrt_(const qd& v) { return sqrt_qd(v); }
  MW_HD static qd abs_(const qd& v) { return sel(v.x[0] < 0.0, -v, v); }
  MW_HD static double eps() { return 1.2154326714572501e-63; }  // 2^-209
  static void pack(const double* planes, int64_t n, int64_t i, qd* out) {
    *out = qd_renorm(planes[i], planes[n + i], planes[2 * n + i], planes[3 * n + i], 0.0);
  }
  static void unpack(const qd& v, double* planes, int64_t n, int64_t i) {
    for (int q = 0; q < 4; ++q) planes[q * n + i] = v.x[q];
  }
};

}  // namespace mw
