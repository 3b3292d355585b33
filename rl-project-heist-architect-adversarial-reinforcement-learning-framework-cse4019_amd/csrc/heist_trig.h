// heist_trig.h -- bit-exact restatement of the host libm's double sin/cos.
//
// Why: the reference raycasts cameras and guards with CPython math.cos/sin
// (heist_architect/components/security.py:71-75, :172-175), i.e. glibc 2.35
// libm, then rounds col + dx*dist half-to-even (security.py:84-88).  Exact .5
// ties are common at integer headings, so a 1-ulp difference in dx/dy flips
// tiles.  glibc's sin/cos are NOT correctly rounded (~0.3% of inputs differ
// from round-to-nearest), so the GPU must evaluate glibc's own algorithm.
//
// What: glibc 2.35 sysdeps/ieee754/dbl-64/s_sin.c (IBM Accurate Mathematical
// Library: table of sin/cos at i/128 as double-double + short polynomials;
// 3-part pi/2 reduction for |x| < 105414350), as built for the x86-64 FMA
// ifunc variant that CPython dispatches to on AVX2+FMA hosts: every
// multiply feeding a single add/sub is fused.  Each fused op below mirrors
// one vfmadd/vfnmadd/vfmsub of that build.  Only |x| < 105414350 is
// supported (ray angles are < 10 rad).
//
// The header compiles for HIP device code and for plain host C++ (the CPU
// test harness checks it bit-for-bit against libm on ~10^8 inputs); it must be
// compiled with -ffp-contract=off so no extra fusion happens.
#pragma once

#if defined(__HIPCC__)
#define HEIST_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#include <cstdint>
#define HEIST_HD static inline
#endif

#include "heist_sincos_table.h"

namespace heist_trig {

// Constants of the published algorithm (usncs.h / s_sin.c).
constexpr double kBig   = 0x1.8p45;                  // 52776558133248: rounds |x| to 1/128
constexpr double kSn3   = -1.66666666666664880952546298448555E-01;
constexpr double kSn5   = 8.33333214285722277379541354343671E-03;
constexpr double kCs2   = 4.99999999999999999999950396842453E-01;
constexpr double kCs4   = -4.16666666666664434524222570944589E-02;
constexpr double kCs6   = 1.38888874007937613028114285595617E-03;
constexpr double kS1    = -0x1.5555555555555p-3;     // -0.16666666666666666
constexpr double kS2    = 0x1.1111111110ecep-7;      //  0.0083333333333323288
constexpr double kS3    = -0x1.a01a019db08b8p-13;    // -0.00019841269834414642
constexpr double kS4    = 0x1.71de27b9a7ed9p-19;     //  2.755729806860771e-06
constexpr double kS5    = -0x1.addffc2fcdf59p-26;    // -2.5022014848318398e-08
constexpr double kHp0   = 0x1.921fb54442d18p0;       // pi/2 hi
constexpr double kHp1   = 0x1.1a62633145c07p-54;     // pi/2 lo
constexpr double kMp1   = 0x1.921fb58000000p0;       // 3-part pi/2 for reduction
constexpr double kMp2   = -0x1.dde973c000000p-27;
constexpr double kPp3   = -0x1.cb3b398000000p-55;
constexpr double kPp4   = -0x1.d747f23e32ed7p-83;
constexpr double kHpInv = 0x1.45f306dc9c883p-1;      // 2/pi
constexpr double kToInt = 0x1.8p52;
constexpr double kTaylorMax = 0.126;

HEIST_HD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
HEIST_HD uint32_t hiword_abs(double x) { return (uint32_t)(bits(x) >> 32) & 0x7fffffffu; }
HEIST_HD int lo_index(double u) { return (int)(uint32_t)bits(u); }

// a + da with |a| < 0.126: odd Taylor polynomial with first-order correction.
HEIST_HD double taylor_sin(double a, double da) {
  double xx = a * a;
  double p = fma(fma(fma(fma(kS5, xx, kS4), xx, kS3), xx, kS2), xx, kS1);
  double t = fma(xx, fma(p, a, -(0.5 * da)), da);
  return a + t;
}

// sin(x + dx) for 0.126 <= |x| < 0.855 via the i/128 table.
HEIST_HD double do_sin(double x, double dx, const double* tab) {
  if (x <= 0) dx = -dx;
  double ax = fabs(x);
  double u = kBig + ax;
  const double* e = tab + 4 * lo_index(u);   // sn, ssn, cs, ccs
  double r = ax - (u - kBig);
  double xx = r * r;
  double s = r + fma(r * xx, fma(xx, kSn5, kSn3), dx);
  double c = fma(r, dx, xx * fma(xx, fma(xx, kCs6, kCs4), kCs2));
  double cor = fma(s, e[2], fma(-c, e[0], fma(s, e[3], e[1])));
  return copysign(e[0] + cor, x);
}

// cos(x + dx) for |x| < 0.855 via the i/128 table.
HEIST_HD double do_cos(double x, double dx, const double* tab) {
  if (x < 0) dx = -dx;
  double ax = fabs(x);
  double u = kBig + ax;
  const double* e = tab + 4 * lo_index(u);
  double r = (ax - (u - kBig)) + dx;
  double xx = r * r;
  double s = fma(r * xx, fma(xx, kSn5, kSn3), r);
  double c = xx * fma(xx, fma(xx, kCs6, kCs4), kCs2);
  double cor = fma(-s, e[0], fma(-c, e[2], fma(-s, e[1], e[3])));
  return e[2] + cor;
}

HEIST_HD double sin_of_reduced(double a, double da, const double* tab) {
  return fabs(a) < kTaylorMax ? taylor_sin(a, da) : do_sin(a, da, tab);
}

// x = n*pi/2 + (a + da), |a| <= pi/4; returns n & 3.
HEIST_HD int reduce(double x, double* a, double* da) {
  double t = fma(x, kHpInv, kToInt);
  double xn = t - kToInt;
  int n = (int)(bits(t) & 3u);
  double y = fma(-xn, kMp2, fma(-xn, kMp1, x));
  double t2 = fma(-xn, kPp3, y);
  double db = fma(-kPp3, xn, y - t2);
  double b = fma(-xn, kPp4, t2);
  db = db + fma(-xn, kPp4, t2 - b);
  *a = b;
  *da = db;
  return n;
}

HEIST_HD double sin(double x, const double* tab) {
  uint32_t k = hiword_abs(x);
  if (k < 0x3e500000u) return x;
  if (k < 0x3feb6000u) return fabs(x) < kTaylorMax ? taylor_sin(x, 0.0) : do_sin(x, 0.0, tab);
  if (k < 0x400368fdu) return copysign(do_cos(kHp0 - fabs(x), kHp1, tab), x);
  double a, da;
  int n = reduce(x, &a, &da);
  double r = (n & 1) ? do_cos(a, da, tab) : sin_of_reduced(a, da, tab);
  return (n & 2) ? -r : r;
}

HEIST_HD double cos(double x, const double* tab) {
  uint32_t k = hiword_abs(x);
  if (k < 0x3e400000u) return 1.0;
  if (k < 0x3feb6000u) return do_cos(x, 0.0, tab);
  if (k < 0x400368fdu) {
    double y = kHp0 - fabs(x);
    double a = y + kHp1;
    double da = (y - a) + kHp1;
    return sin_of_reduced(a, da, tab);
  }
  double a, da;
  int n = reduce(x, &a, &da) + 1;
  double r = (n & 1) ? do_cos(a, da, tab) : sin_of_reduced(a, da, tab);
  return (n & 2) ? -r : r;
}

// sin-type kernel and do_cos on the SAME argument (a, da), |a| < 0.855: one table row and
// one r0 = |a| - (u - big) serve both (do_sin / do_cos above, unchanged op for op).
HEIST_HD void sin_cos_same(double a, double da, const double* tab, double* S, double* D) {
  const double ax = fabs(a);
  const double u = kBig + ax;
  const double* e = tab + 4 * lo_index(u);
  const double r0 = ax - (u - kBig);
  {  // do_cos(a, da)
    const double dxc = a < 0 ? -da : da;
    const double r = r0 + dxc;
    const double xx = r * r;
    const double s = fma(r * xx, fma(xx, kSn5, kSn3), r);
    const double c = xx * fma(xx, fma(xx, kCs6, kCs4), kCs2);
    const double cor = fma(-s, e[0], fma(-c, e[2], fma(-s, e[1], e[3])));
    *D = e[2] + cor;
  }
  if (ax < kTaylorMax) {
    *S = taylor_sin(a, da);
  } else {  // do_sin(a, da)
    const double dxs = a <= 0 ? -da : da;
    const double r = r0;
    const double xx = r * r;
    const double s = r + fma(r * xx, fma(xx, kSn5, kSn3), dxs);
    const double c = fma(r, dxs, xx * fma(xx, fma(xx, kCs6, kCs4), kCs2));
    const double cor = fma(s, e[2], fma(-c, e[0], fma(s, e[3], e[1])));
    *S = copysign(e[0] + cor, a);
  }
}

// sin(x) and cos(x) together, bit-identical to sin() and cos() above.  In every glibc
// branch one value comes from a sin-type kernel (taylor_sin or do_sin) and the other from
// do_cos:
//   A |x| < 0.855 (k < 0x3feb6000):  sin = sin_type(x, 0)             cos = do_cos(x, 0)
//   B |x| < 2.426:   t = hp0 - |x|   sin = copysign(do_cos(t, hp1), x)  cos = sin_type(t + hp1, da)
//   C otherwise:     x = n pi/2 + a  sin = (n odd ? do_cos : sin_type)(a, da), cos uses n + 1
// plus the tiny-argument early returns (sin x = x, cos x = 1).  In A and C both kernels see
// the same argument, so they share one table lookup (sin_cos_same); the branches are real
// branches because neighbouring rays (a wavefront) almost always take the same one.
HEIST_HD void sincos(double x, const double* tab, double* s_out, double* c_out) {
  const uint32_t k = hiword_abs(x);
  double sv, cv;
  if (k < 0x3feb6000u || k >= 0x400368fdu) {
    double a = x, da = 0.0;
    int n = 0;
    if (k >= 0x400368fdu) n = reduce(x, &a, &da);
    double S, D;
    sin_cos_same(a, da, tab, &S, &D);
    if (k < 0x3feb6000u) {
      sv = S;
      cv = D;
    } else {
      const double s0 = (n & 1) ? D : S;
      const double c0 = (n & 1) ? S : D;
      sv = (n & 2) ? -s0 : s0;
      cv = ((n + 1) & 2) ? -c0 : c0;
    }
  } else {
    const double t = kHp0 - fabs(x);
    const double ab = t + kHp1;
    const double dab = (t - ab) + kHp1;
    sv = copysign(do_cos(t, kHp1, tab), x);
    cv = sin_of_reduced(ab, dab, tab);
  }
  *s_out = k < 0x3e500000u ? x : sv;
  *c_out = k < 0x3e400000u ? 1.0 : cv;
}

}  // namespace heist_trig
