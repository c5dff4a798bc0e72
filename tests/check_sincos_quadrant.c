/* tests/check_sincos_quadrant.c — exhaustive check behind device_math.hpp
 * sincosf_glibc<kInRange>: for every float y in [0, 6.5), glibc's reduce_fast
 * quadrant ((int)((double)y * 2^24 * 2/pi) + 2^23) >> 24 (sincosf.h,
 * !TOINT_INTRINSICS) equals (int)fmaf(y, (float)(2/pi), 0.5f).  Prints the
 * count of floats checked and of mismatches; exit status 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int main(void) {
  const double hpi_inv = 0x1.45F306DC9C883p+23;
  const float k = 0x1.45f306p-1f;
  const float top = 6.5f;
  uint32_t hi;
  memcpy(&hi, &top, 4);
  long bad = 0, n = 0;
  for (uint32_t b = 0; b < hi; ++b) {
    float y;
    memcpy(&y, &b, 4);
    const int ref = ((int)((double)y * hpi_inv) + 0x800000) >> 24;
    const int f32 = (int)fmaf(y, k, 0.5f);
    ++n;
    bad += ref != f32;
  }
  printf("%ld floats, %ld mismatches\n", n, bad);
  return bad != 0;
}
