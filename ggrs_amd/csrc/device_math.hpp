// ggrs_amd/csrc/device_math.hpp — scalar arithmetic the game handlers need,
// written so the GPU reproduces the reference's CPU results bit for bit.
//
// * sincosf_glibc: Rust's f32::sin/cos (ex_game.rs:282-288) lower to glibc's
//   sinf/cosf on x86_64 Linux.  glibc 2.28+ evaluates them in double precision
//   (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h, sincosf_data.c:
//   reduce_fast + degree-4/5 polynomials).  That algorithm is restated here in
//   double arithmetic, which the GPU executes with IEEE-exact add/mul/fma, so
//   device results equal glibc's.  Checked exhaustively against the host libm
//   for every float in [-0.1, 6.4] (tests/test_device_math.py, GPU) and on the
//   host for all 2.1e9 floats of that range when this file was written.
//   Only |x| < 120 is restated (ex_game rotations live in [0, 2*pi]); larger
//   arguments fall back to the ocml routines and are counted as unexpected.
// * fletcher16 closed form: the serial mod-255 loop of ex_game.rs:42-52 equals
//   s1 = sum(b_i) mod 255, s2 = sum((n - i) * b_i) mod 255 (s2 sums every
//   prefix s1).  Per 32-bit word that is two v_dot4_u32_u8.
// * SipHash-1-3 with keys (0,0): Rust std DefaultHasher (tests/stubs.rs:8-12).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rb {

// ----------------------------------------------------------------------------
// glibc sinf/cosf restated (double evaluation, FMA form — the variant the
// x86_64 ifunc selects on FMA-capable hosts; the non-FMA form gives identical
// float results on this range, verified).
// ----------------------------------------------------------------------------
struct SinCos {
  float s, c;
};

__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }

// sincosf.h sinf_poly(x, x2, p, n) for n even (sine polynomial); s1..s3 are the
// same in both __sincosf_table rows.
__device__ __forceinline__ double sin_poly(double x, double x2) {
  const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
  double x3 = x * x2;
  double sp = __builtin_fma(x2, s3, s2);
  double x7 = x3 * x2;
  double s = __builtin_fma(x3, s1, x);
  return __builtin_fma(x7, sp, s);
}
// sinf_poly for n odd (cosine polynomial) with __sincosf_table[0]; row [1] has
// every c_i negated, which negates the result exactly.
__device__ __forceinline__ double cos_poly(double x2) {
  const double c0 = 0x1p0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5,
               c3 = -0x1.6c087e89a359dp-10, c4 = 0x1.99343027bf8c3p-16;
  double x4 = x2 * x2;
  double cp2 = __builtin_fma(x2, c4, c3);
  double cp1 = __builtin_fma(x2, c1, c0);
  double x6 = x4 * x2;
  double c = __builtin_fma(x4, c2, cp1);
  return __builtin_fma(x6, cp2, c);
}

// |y| >= 120: not restated (ex_game never gets there); the library routines,
// out of line so they do not bloat the hot path, and counted.
__device__ __noinline__ SinCos sincosf_large(float y, uint32_t* unexpected) {
  if (unexpected) atomicAdd(unexpected, 1u);
  SinCos r;
  r.s = sinf(y);
  r.c = cosf(y);
  return r;
}

// kInRange: the caller guarantees +0 <= y < 6.5 (no out-of-line library path,
// and no tiny-argument branch: on that range this evaluation without it equals
// glibc's sinf/cosf for every float, tests/check_sincos_inrange.c).
template <bool kInRange = false>
__device__ __forceinline__ SinCos sincosf_glibc(float y, uint32_t* unexpected) {
  // |y| < pi/4 takes glibc's unreduced branch: reduce_fast yields n = 0 and
  // xr = y exactly there, so one straight-line path serves both.
  const double hpi_inv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;  // !TOINT_INTRINSICS form (x86_64)
  const double x = y;
  // reduce_fast's quadrant n = ((int)(x * 2^24 * 2/pi) + 2^23) >> 24; for 0 <= y < 6.5 it equals
  // (int)(y * (float)(2/pi) + 0.5f) with one f32 fma, for every float there
  // (tests/check_sincos_quadrant.c, run by tests/test_oracle.py)
  const int n = kInRange ? static_cast<int32_t>(__builtin_fmaf(y, 0x1.45f306p-1f, 0.5f))
                         : (static_cast<int32_t>(x * hpi_inv) + 0x800000) >> 24;
  double xr = __builtin_fma(-static_cast<double>(n), hpi, x);
  const double x2 = xr * xr;
  // sign[4] = {1,-1,-1,1}: negate when (n & 3) is 1 or 2, i.e. bit 1 of n + 1.
  // Adding 2^31 to the high word flips the sign bit (no carry out of bit 31).
  const uint32_t sflip = (static_cast<uint32_t>(n + 1) >> 1) & 1u;
  xr = __hiloint2double(static_cast<int>(static_cast<uint32_t>(__double2hiint(xr)) + (sflip << 31)), __double2loint(xr));
  const float sp = static_cast<float>(sin_poly(xr, x2));
  // __sincosf_table[1] (n & 2) negates every cosine coefficient: negate the
  // rounded result (rounding is sign-symmetric).
  const uint32_t cflip = (static_cast<uint32_t>(n) >> 1) & 1u;
  const float cp = __uint_as_float(__float_as_uint(static_cast<float>(cos_poly(x2))) + (cflip << 31));
  SinCos r;
  // sinf: n even -> sine poly, odd -> cosine poly; cosf uses n ^ 1.
  r.s = (n & 1) ? cp : sp;
  r.c = (n & 1) ? sp : cp;
  // |y| < 2^-12: glibc returns (y, 1).  Inline: ex_game's rotations sit at
  // exactly 0 for long stretches (State::new gives player 1 rot = 0).
  if constexpr (!kInRange) {
    const uint32_t top = abstop12(y);
    if (top < abstop12(0x1p-12f)) {
      r.s = y;
      r.c = 1.0f;
    }
    if (__builtin_expect(top >= abstop12(120.0f), 0)) r = sincosf_large(y, unexpected);
  }
  return r;
}

// f32::rem_euclid (r = x % rhs; r < 0 ? r + |rhs| : r).  fmod is exact; for
// |x| < 2|rhs| it is x or x -/+ rhs (Sterbenz), else the library fmodf (out of line).
__device__ __noinline__ float fmodf_slow(float x, float y) { return fmodf(x, y); }
// kInRange: the caller guarantees |x| < 2|rhs|.
template <bool kInRange = false>
__device__ __forceinline__ float rem_euclid(float x, float rhs) {
  const float ay = __builtin_fabsf(rhs), ax = __builtin_fabsf(x);
  float r = ax < ay ? x : __builtin_copysignf(ax - ay, x);
  if constexpr (!kInRange)
    if (__builtin_expect(!(ax < 2.0f * ay), 0)) r = fmodf_slow(x, rhs);
  return r < 0.0f ? r + ay : r;
}

// kNear: the caller guarantees -|rhs| < x < 2|rhs|.  There fmod(x, rhs) is x
// for x < |rhs| and x - |rhs| (exact) above, so rem_euclid is one add or
// subtract of |rhs|, the same operation rem_euclid performs on that range.
template <bool kNear = false>
__device__ __forceinline__ float rem_euclid_near(float x, float rhs) {
  if constexpr (kNear) {
    const float ay = __builtin_fabsf(rhs);
    return x < 0.0f ? x + ay : (x >= ay ? x - ay : x);
  } else {
    return rem_euclid<false>(x, rhs);
  }
}

// ----------------------------------------------------------------------------
// Correctly rounded f32 sqrt and division for operands in known ranges: the
// sequences the compiler emits under -fhip-fp32-correctly-rounded-divide-sqrt,
// minus the scaling and special-value fix-ups those ranges never need.
// ----------------------------------------------------------------------------
// sqrt(x) for x in (1, +inf]: v_sqrt_f32 (within 1 ulp), then the neighbour
// test (fma residuals of s - 1 ulp and s + 1 ulp).  The compiler's sequence adds
// a 2^32 scaling below 2^-96 and a class check for +-0/inf; for x = +inf this
// one also returns +inf (both residuals are NaN).
__device__ __forceinline__ float sqrt_rn_above_one(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
  const float t = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
  return __builtin_fmaf(-su, s, x) > 0.0f ? su : t;
}
// 1/d refined once, the reciprocal step of the division sequence.
__device__ __forceinline__ float rcp_refined(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  return __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
}
// n / d with r = rcp_refined(d): the quotient and two residual corrections of
// the compiler's sequence (v_div_scale / v_div_fmas / v_div_fixup reduce to
// exactly these fmas when nothing is scaled).  Valid, i.e. nothing would be
// scaled or fixed up, for d in (1, 256) and 2^-96 <= |n| (so |n/d| is normal
// and far from overflow).
__device__ __forceinline__ float div_rn_unscaled(float n, float d, float r) {
  float q = n * r;
  q = __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
  return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
}

// ----------------------------------------------------------------------------
// fletcher16 closed form pieces
// ----------------------------------------------------------------------------
struct Fl16 {
  uint32_t s1, s2;  // plain sums, reduced once at the end
};
// Add a 32-bit little-endian word whose first byte sits at image offset `o`
// of an n-byte image: weights n-o, n-o-1, n-o-2, n-o-3 (all < 256 for the
// images used here).
__device__ __forceinline__ void fl16_word(Fl16& a, uint32_t w, uint32_t wpack) {
  a.s1 = __builtin_amdgcn_udot4(w, 0x01010101u, a.s1, false);
  a.s2 = __builtin_amdgcn_udot4(w, wpack, a.s2, false);
}
__host__ __device__ constexpr uint32_t fl16_weights(int n, int o) {
  return static_cast<uint32_t>(n - o) | (static_cast<uint32_t>(n - o - 1) << 8) |
         (static_cast<uint32_t>(n - o - 2) << 16) | (static_cast<uint32_t>(n - o - 3) << 24);
}
// x mod 255 for x < 2^24, valid in the low 8 bits only: q = floor(x / 255)
// by a multiply-high; x - 255 q = x + 0xFF01 q (mod 2^16) is one v_mad_u32_u24.
__device__ __forceinline__ uint32_t mod255_lo8(uint32_t x) {
  const uint32_t q = __umulhi(x, 0x80808081u) >> 7;
  return __umul24(q, 0xFF01u) + x;
}
// Both sums must be < 2^24: images of n bytes with 255 * n * (n + 1) / 2 < 2^24
// (n <= 361; ex_game images are at most 116 bytes).
__device__ __forceinline__ uint16_t fl16_finish(const Fl16& a) {
  // (s2 mod 255) << 8 | (s1 mod 255): byte 0 of each, packed by one v_perm_b32
  return static_cast<uint16_t>(__builtin_amdgcn_perm(mod255_lo8(a.s2), mod255_lo8(a.s1), 0x0c0c0400u));
}

// ----------------------------------------------------------------------------
// SipHash-1-3, keys (0,0), 8-byte message le32(a) || le32(b)
// ----------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t rotl64(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }
#define RB_SIPROUND                                                      \
  do {                                                                   \
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);        \
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                             \
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                             \
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);        \
  } while (0)
__host__ __device__ __forceinline__ uint64_t siphash13_i32x2(int32_t a, int32_t b) {
  uint64_t v0 = 0x736f6d6570736575ULL, v1 = 0x646f72616e646f6dULL;
  uint64_t v2 = 0x6c7967656e657261ULL, v3 = 0x7465646279746573ULL;
  const uint64_t m = static_cast<uint64_t>(static_cast<uint32_t>(a)) |
                     (static_cast<uint64_t>(static_cast<uint32_t>(b)) << 32);
  v3 ^= m;
  RB_SIPROUND;
  v0 ^= m;
  const uint64_t t = 8ULL << 56;  // length byte, empty tail
  v3 ^= t;
  RB_SIPROUND;
  v0 ^= t;
  v2 ^= 0xff;
  RB_SIPROUND;
  RB_SIPROUND;
  RB_SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}
#undef RB_SIPROUND

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

}  // namespace rb
