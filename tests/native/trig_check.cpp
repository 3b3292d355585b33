// Host check: heist_trig::sin/cos (the GPU's restatement of glibc 2.35 dbl-64
// sin/cos) must equal the host libm bit-for-bit.  Built and run by
// tests/test_trig.py (g++ -O2 -ffp-contract=off).  argv[1] = samples per class.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include "heist_trig.h"

static const double kTab[] = HEIST_SINCOS_TAB_INIT;
static long long g_bad = 0, g_n = 0;

// Through volatile pointers: at -O2 gcc would merge ::sin(x) and ::cos(x)
// into one sincos() call, a different (non-ifunc) libm routine.  CPython
// calls sin and cos separately, so that is what the GPU must match.
static double (*volatile p_sin)(double) = ::sin;
static double (*volatile p_cos)(double) = ::cos;

static void check(double x) {
  double s0 = p_sin(x), c0 = p_cos(x);
  double s1 = heist_trig::sin(x, kTab), c1 = heist_trig::cos(x, kTab);
  double s2, c2;
  heist_trig::sincos(x, kTab, &s2, &c2);
  ++g_n;
  if (memcmp(&s0, &s1, 8) || memcmp(&c0, &c1, 8) || memcmp(&s0, &s2, 8) || memcmp(&c0, &c2, 8)) {
    if (++g_bad <= 10)
      printf("MISMATCH x=%a sin libm=%a emu=%a joint=%a cos libm=%a emu=%a joint=%a\n", x, s0, s1, s2, c0, c1, c2);
  }
}

int main(int argc, char** argv) {
  long long n = argc > 1 ? atoll(argv[1]) : 1000000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> u(-10.0, 10.0), deg(-200.0, 800.0), fov(30.0, 120.0),
      head(0.0, 360.0);
  const double d2r = 3.141592653589793 / 180.0;  // CPython degToRad
  for (long long i = 0; i < n; ++i) check(u(rng));
  for (long long i = 0; i < n; ++i) check(deg(rng) * d2r);
  // ray angles exactly as security.py:70-71 forms them
  for (long long i = 0; i < n / 64; ++i) {
    double f = (double)(float)fov(rng);
    double h = (i & 1) ? head(rng) : (double)(long long)head(rng);
    int nr = (int)(f * 2) > 30 ? (int)(f * 2) : 30;
    for (int k = 0; k <= nr; k += 4) check(((h - f / 2.0) + (f * k) / nr) * d2r);
  }
  // dense grid of quarter/thousandth degrees
  for (long long k = -200000; k <= 800000; ++k) check((k * 0.001) * d2r);
  for (long long k = -800; k <= 3200; ++k) check((k * 0.25) * d2r);
  // tiny and boundary magnitudes
  std::uniform_int_distribution<int> e(-40, 3);
  std::uniform_real_distribution<double> m(1.0, 2.0);
  for (long long i = 0; i < n / 4; ++i) check(ldexp(m(rng), e(rng)) * ((i & 1) ? 1 : -1));
  printf("checked %lld bad %lld\n", g_n, g_bad);
  return g_bad ? 1 : 0;
}
