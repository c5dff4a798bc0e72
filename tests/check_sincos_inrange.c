/* tests/check_sincos_inrange.c — exhaustive check behind device_math.hpp
 * sincosf_glibc<kInRange>: for every float y in [+0, 6.5) the in-range
 * evaluation (f32-fma quadrant, double reduction and polynomials, no tiny-
 * argument branch) equals this host's glibc sinf(y) and cosf(y) bit for bit.
 * OpenMP over the range; prints floats checked and mismatches, exit 1 on any. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static void sincos_inrange(float y, float* s, float* c) {
  const double hpi = 0x1.921FB54442D18p0;
  const double x = y;
  const int n = (int)fmaf(y, 0x1.45f306p-1f, 0.5f);
  double xr = fma(-(double)n, hpi, x);
  const double x2 = xr * xr;
  if (((unsigned)(n + 1) >> 1) & 1u) xr = -xr;
  const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
  double x3 = xr * x2, sp = fma(x2, s3, s2), x7 = x3 * x2, ss = fma(x3, s1, xr);
  const float fs = (float)fma(x7, sp, ss);
  const double c0 = 0x1p0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
               c4 = 0x1.99343027bf8c3p-16;
  double x4 = x2 * x2, cp2 = fma(x2, c4, c3), cp1 = fma(x2, c1, c0), x6 = x4 * x2, cc = fma(x4, c2, cp1);
  float fc = (float)fma(x6, cp2, cc);
  if (((unsigned)n >> 1) & 1u) fc = bitsf(fbits(fc) ^ 0x80000000u);
  *s = (n & 1) ? fc : fs;
  *c = (n & 1) ? fs : fc;
}

int main(void) {
  const uint32_t hi = fbits(6.5f);
  long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static, 1 << 20)
  for (int64_t b = 0; b < (int64_t)hi; ++b) {
    const float y = bitsf((uint32_t)b);
    float s, c;
    sincos_inrange(y, &s, &c);
    bad += fbits(s) != fbits(sinf(y)) || fbits(c) != fbits(cosf(y));
  }
  printf("%ld floats, %ld mismatches\n", (long)hi, bad);
  return bad != 0;
}
