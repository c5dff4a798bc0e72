// ggrs_amd/csrc/games.hpp — the compiled-in request handlers.
//
// A game plugs into the engine with (the `Config` trait of lib.rs:240-262 plus
// the user's handle_requests of ex_game.rs:76-84, as device code):
//   kLanes    lanes per session (1, 2 or 4): a session's state may be sliced
//             over a lane group that advances in lock-step; the checksum is
//             then combined across the group with DPP lane swaps
//   NWL       state words per lane stored in a snapshot slot (u32 each)
//   InRec     one session's packed inputs for one frame (P Input values)
//   CS        checksum type stored per cell (zero-extended to u128 on export)
//   init      host: State::new, words [kLanes][NWL]
//   advance   device: one AdvanceFrame on the lane's register-resident slice
//   checksum  device: the checksum the game's save_game_state stores (the
//             whole session's value, in every lane of the group)
//   image     host: canonical byte image of (frame, words [kLanes][NWL])
// The cell's frame tag is stored once per slot (batch-uniform): every game
// here asserts state.frame == cell frame on save (ex_game.rs:89,
// stubs.rs:53,93, stubs_enum.rs:59), so the per-session frame word is
// redundant and is supplied from the tag instead of being stored S times.
#pragma once

#include <cmath>
#include <cstring>
#include <type_traits>

#include "device_math.hpp"

namespace rb {

enum SaveMode : uint32_t { SAVE_NONE = 0, SAVE_RECORD = 1, SAVE_COMPARE = 2, SAVE_PLAIN = 3 };

struct U128 {
  uint64_t lo, hi;
};
__host__ __device__ inline bool operator!=(const U128& a, const U128& b) { return a.lo != b.lo || a.hi != b.hi; }

// Per-save context (only the random-checksum stub uses it).
struct CsCtx {
  uint64_t seed;
  uint32_t session;
  uint32_t nonce;  // tick * 256 + step, batch-uniform
};

template <int P>
struct InRecOf {
  using T = uint32_t;
};
template <>
struct InRecOf<1> {
  using T = uint8_t;
};
template <>
struct InRecOf<2> {
  using T = uint16_t;
};

// Sum of a u32 over the lane group of a session (groups of 1, 2 or 4
// consecutive lanes): DPP quad_perm swaps, no LDS round trip.
template <int L>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
  if constexpr (L >= 2) v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  if constexpr (L >= 4) v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  return v;
}

// ============================================================================
// examples/ex_game/ex_game.rs — one lane per player (kSplit) or per session
// ============================================================================
template <int P, bool kSplit>
struct ExGame {
  static_assert(P >= 1 && P <= 4, "ex_game supports 1..4 players (ex_game.rs:65)");
  static constexpr int kPlayers = P;
  static constexpr int kLanes = kSplit ? (P == 1 ? 1 : (P == 2 ? 2 : 4)) : 1;
  static constexpr int kPlayersPerLane = kSplit ? 1 : P;
  static constexpr int NWL = 5 * kPlayersPerLane;  // per player: x, y, vx, vy, rot
  static constexpr int kInputBytes = 1;
  static constexpr uint32_t kInputAlphabet = 16;  // the 4 input flag bits (ex_game.rs:16-19): the fan-out's candidates
  static constexpr int kImageBytes = 36 + 20 * P;  // bincode 1.3 image of State (ex_game.rs:224-231)
  static_assert(255 * kImageBytes * (kImageBytes + 1) / 2 < (1 << 24), "fl16_finish needs sums < 2^24");
  static constexpr bool kDisplay = true;           // Game::last_checksum / periodic_checksum
  using InRec = typename InRecOf<P>::T;
  using CS = uint16_t;

  // ex_game.rs:8-24
  static constexpr float kFriction = 0.98f;
  static constexpr float kMovementSpeed = 15.0f / 60.0f;
  static constexpr float kRotationSpeed = 2.5f / 60.0f;
  static constexpr float kMaxSpeed = 7.0f;
  static constexpr float kWidth = 600.0f, kHeight = 800.0f;
  static constexpr float kPi = 3.14159265358979323846f;

  // byte offsets of player i's fields in the bincode image
  __host__ __device__ static constexpr int off_x(int i) { return 20 + 8 * i; }
  __host__ __device__ static constexpr int off_vx(int i) { return 28 + 8 * P + 8 * i; }
  __host__ __device__ static constexpr int off_rot(int i) { return 36 + 16 * P + 4 * i; }

  // State::new (ex_game.rs:234-257), evaluated with the host libm like the
  // reference (glibc cosf/sinf/fmodf).  words: [kLanes][NWL].
  static void init(uint32_t* words) {
    std::memset(words, 0, sizeof(uint32_t) * kLanes * NWL);
    const float r = kWidth / 4.0f;
    for (int i = 0; i < P; ++i) {
      // volatile: keep the compiler from constant-folding libm calls with its
      // own (correctly rounded) evaluation; the reference calls glibc at run time.
      volatile float fi = static_cast<float>(i), fp = static_cast<float>(P);
      float rot = fi / fp * 2.0f * kPi;
      float x = kWidth / 2.0f + r * std::cos(rot);
      float y = kHeight / 2.0f + r * std::sin(rot);
      float ro = std::fmod(rot + kPi, 2.0f * kPi);
      uint32_t* w = words + (kSplit ? i * NWL : 0);
      const int j = kSplit ? 0 : i;
      std::memcpy(&w[5 * j + 0], &x, 4);
      std::memcpy(&w[5 * j + 1], &y, 4);
      std::memcpy(&w[5 * j + 4], &ro, 4);
    }
  }

  static void image(const uint32_t* words, int32_t frame, uint8_t* out) {
    std::memset(out, 0, kImageBytes);
    std::memcpy(out, &frame, 4);
    const uint64_t np = P;
    std::memcpy(out + 4, &np, 8);
    std::memcpy(out + 12, &np, 8);
    std::memcpy(out + 20 + 8 * P, &np, 8);
    std::memcpy(out + 28 + 16 * P, &np, 8);
    for (int i = 0; i < P; ++i) {
      const uint32_t* w = words + (kSplit ? i * NWL : 5 * i);
      std::memcpy(out + off_x(i), &w[0], 4);
      std::memcpy(out + off_x(i) + 4, &w[1], 4);
      std::memcpy(out + off_vx(i), &w[2], 4);
      std::memcpy(out + off_vx(i) + 4, &w[3], 4);
      std::memcpy(out + off_rot(i), &w[4], 4);
    }
  }
  static U128 cs128(CS c) { return U128{c, 0}; }
  // canonical word k (bincode order: positions, velocities, rotations) -> (lane, word)
  static void word_loc(int k, int* lane, int* word) {
    int i, f;
    if (k < 2 * P) { i = k / 2; f = k % 2; }
    else if (k < 4 * P) { i = (k - 2 * P) / 2; f = 2 + (k - 2 * P) % 2; }
    else { i = k - 4 * P; f = 4; }
    *lane = kSplit ? i : 0;
    *word = kSplit ? f : 5 * i + f;
  }
  static constexpr int kCanonWords = 5 * P;

  __device__ static uint32_t player_input(InRec rec, int i) { return (static_cast<uint32_t>(rec) >> (8 * i)) & 0xffu; }
  // The representative of the inputs that move a player alike (p2p.hpp InputCanon): State::advance
  // reads only up != down and up (thrust, :281-289) and left != right and left (rotation, :291-296),
  // so the 16 inputs fall into 9 classes (4 bits only: the fan-out's candidates are < 16).
  __host__ __device__ static constexpr uint32_t canon_input(uint32_t v) {
    const bool up = v & 1u, down = v & 2u, left = v & 4u, right = v & 8u;
    return (up != down ? (up ? 1u : 2u) : 0u) | (left != right ? (left ? 4u : 8u) : 0u);
  }

  // ex_game.rs:300-304: if |v| > MAX_SPEED { v = v * MAX_SPEED / |v| }.
  __device__ static void speed_clamp(float& vx, float& vy) {
    // mag > 7 <=> vx^2+vy^2 > 49: sqrt is correctly rounded and monotone,
    // sqrt(49) = 7 exactly, and the next float above 49 (49 + 2^-18) has a
    // square root that rounds above 7 (tests/test_oracle.py checks both
    // sides), NaN compares false both ways.  The sqrt is only needed for
    // the clamp, so it moves inside the branch.
    const float m2 = vx * vx + vy * vy;
    if (m2 > kMaxSpeed * kMaxSpeed) {
      const float mag = sqrt_rn_above_one(m2);
      const float nx = vx * kMaxSpeed, ny = vy * kMaxSpeed;
      if (mag < 256.0f && __builtin_fabsf(nx) >= 0x1p-96f && __builtin_fabsf(ny) >= 0x1p-96f) {
        const float r = rcp_refined(mag);  // both divisions share the denominator
        vx = div_rn_unscaled(nx, mag, r);
        vy = div_rn_unscaled(ny, mag, r);
      } else {  // zeros, tiny or huge operands: the full IEEE division
        vx = nx / mag;
        vy = ny / mag;
      }
    }
  }

  // State::advance (ex_game.rs:259-321) for one player.  Compiled with
  // -ffp-contract=off: every f32 operation rounds exactly as the reference's.
  template <bool kInRange = false>
  __device__ static void advance_player(uint32_t* w, uint32_t input, uint32_t* unexpected) {
    const float old_x = __uint_as_float(w[0]), old_y = __uint_as_float(w[1]);
    const float old_vx = __uint_as_float(w[2]), old_vy = __uint_as_float(w[3]);
    float rot = __uint_as_float(w[4]);
    float vx = old_vx * kFriction;
    float vy = old_vy * kFriction;
    const bool up = input & 1u, down = input & 2u, left = input & 4u, right = input & 8u;
    {  // thrust (:281-284) / brake (:286-289) and rotation (:291-296) as selects: some lane of
       // every wave needs each of them, so branches only add exec-mask bookkeeping
      const SinCos sc = sincosf_glibc<kInRange>(rot, unexpected);
      const float tx = kMovementSpeed * sc.c, ty = kMovementSpeed * sc.s;
      const float vx1 = up ? vx + tx : vx - tx, vy1 = up ? vy + ty : vy - ty;
      vx = up != down ? vx1 : vx;
      vy = up != down ? vy1 : vy;
      const float r1 = rem_euclid<kInRange>(left ? rot - kRotationSpeed : rot + kRotationSpeed, 2.0f * kPi);
      rot = left != right ? r1 : rot;
    }
    speed_clamp(vx, vy);
    float x = old_x + vx, y = old_y + vy;
    x = fminf(fmaxf(x, 0.0f), kWidth);
    y = fminf(fmaxf(y, 0.0f), kHeight);
    w[0] = __float_as_uint(x);
    w[1] = __float_as_uint(y);
    w[2] = __float_as_uint(vx);
    w[3] = __float_as_uint(vy);
    w[4] = __float_as_uint(rot);
  }

  template <bool kInRange = false>
  __device__ static void advance(uint32_t (&w)[NWL], InRec rec, int lane, uint32_t disconnected_mask,
                                 uint32_t* unexpected) {
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      const int i = kSplit ? lane : j;  // player index
      const uint32_t input = ((disconnected_mask >> i) & 1u) ? 4u : player_input(rec, i);  // Disconnected => 4 (:268)
      advance_player<kInRange>(&w[5 * j], input, unexpected);
    }
  }

  // ---- phase-split AdvanceFrames for the fused steady ticks (kernels.hpp
  // steady_kernel).  In State::advance (:259-321) the rotation and its
  // sine/cosine depend on nothing but the rotation and the inputs, never on
  // position or velocity.  So `prepare` runs the rotation chain of all N
  // AdvanceFrames of a tick first — N independent double-precision sincos
  // evaluations the scheduler can interleave — and `advance_prepared` then
  // runs each frame's velocity/position chain on the precomputed thrust.
  // Every f32 operation is the same one on the same operands as in
  // advance_player, so the results are bit-identical:
  //   up ? v + t : v - t          ==  v + (up ? t : -t)    (IEEE a - b = a + (-b))
  //   -(S * c)                    ==  (-S) * c             (rounding is sign-symmetric)
  //   up != down ? v + t : v      ==  v + (up != down ? t : -0.0)
  //     (v + -0 is v for every v, +-0 included; v is never a signalling NaN
  //     here: it comes out of the friction multiply, which quiets NaNs)
  //   left ? rot - r : rot + r    ==  rot + (left ? -r : r)
  static constexpr bool kHasPrep = true;
  static constexpr bool kUsesStatus = false;  // reads only Disconnected (status bit i)
  template <int N>
  struct Prep {
    float tx[kPlayersPerLane][N], ty[kPlayersPerLane][N];  // thrust added in frame k (-0 when none)
    float rot[kPlayersPerLane][N + 1];                       // rotation before frame k (rot[N]: after the last)
  };
  // One frame's input as this lane's players act on it (decoded once, when the
  // input enters the steady kernel's window): the signed thrust speed, the
  // signed rotation step, and all-ones masks for "UP xor DOWN" and "LEFT xor
  // RIGHT" (bit selects, no compare per use).
  struct Dec {
    float sp[kPlayersPerLane], rd[kPlayersPerLane];
    uint32_t thm[kPlayersPerLane], rom[kPlayersPerLane];
  };
  __device__ static Dec decode(InRec rec, int lane) {
    Dec d;
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      const uint32_t input = player_input(rec, kSplit ? lane : j);
      // Integer bit arithmetic, each value passed through an empty asm: the compiler keeps all four
      // as plain VGPR words.  Written as selects on the input bits they became per-lane booleans,
      // which the compiler holds as 64-bit lane masks in SGPRs; the window of CD+1 decoded frames
      // then spilled SGPRs into VGPR lanes and read them back (v_readlane) at every use.  Measured
      // (interleaved A/B, profiles/r05_ab_decbits.log): SyncTest 4.03 -> 3.92 us per tick, the
      // driver's call 1.242e11 -> 1.262e11, one-tick launches 9.51 -> 9.40 us.
      const uint32_t x = input ^ (input >> 1);  // bit 0: up ^ down, bit 2: left ^ right
      uint32_t sp = __float_as_uint(kMovementSpeed) | ((~input & 1u) << 31);         // up ? S : -S
      uint32_t rd = __float_as_uint(kRotationSpeed) | (((input >> 2) & 1u) << 31);   // left ? -R : R
      uint32_t thm = 0u - (x & 1u), rom = 0u - ((x >> 2) & 1u);
      asm volatile("" : "+v"(sp), "+v"(rd), "+v"(thm), "+v"(rom));
      d.sp[j] = __uint_as_float(sp);
      d.rd[j] = __uint_as_float(rd);
      d.thm[j] = thm;
      d.rom[j] = rom;
    }
    return d;
  }
  template <bool kInRange, int N>
  __device__ static void prepare(const uint32_t (&w)[NWL], const Dec (&dec)[N], Prep<N>& pr, uint32_t* unexpected) {
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      float rot = __uint_as_float(w[5 * j + 4]);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const Dec& d = dec[k];
        pr.rot[j][k] = rot;
        const SinCos sc = sincosf_glibc<kInRange>(rot, unexpected);
        const float tx = d.sp[j] * sc.c, ty = d.sp[j] * sc.s;
        // thrust ? t : -0.0 as a bit select on the mask
        pr.tx[j][k] = __uint_as_float((d.thm[j] & __float_as_uint(tx)) | (~d.thm[j] & 0x80000000u));
        pr.ty[j][k] = __uint_as_float((d.thm[j] & __float_as_uint(ty)) | (~d.thm[j] & 0x80000000u));
        const float r1 = rem_euclid_near<kInRange>(rot + d.rd[j], 2.0f * kPi);
        rot = __uint_as_float((d.rom[j] & __float_as_uint(r1)) | (~d.rom[j] & __float_as_uint(rot)));
      }
      pr.rot[j][N] = rot;
    }
  }
  // AdvanceFrame k of the prepared tick: friction, thrust, speed clamp, position.
  template <int N>
  __device__ static void advance_prepared(uint32_t (&w)[NWL], const Prep<N>& pr, int k) {
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      uint32_t* p = &w[5 * j];
      const float old_x = __uint_as_float(p[0]), old_y = __uint_as_float(p[1]);
      float vx = __uint_as_float(p[2]) * kFriction + pr.tx[j][k];
      float vy = __uint_as_float(p[3]) * kFriction + pr.ty[j][k];
      speed_clamp(vx, vy);
      float x = old_x + vx, y = old_y + vy;
      x = fminf(fmaxf(x, 0.0f), kWidth);
      y = fminf(fmaxf(y, 0.0f), kHeight);
      p[0] = __float_as_uint(x);
      p[1] = __float_as_uint(y);
      p[2] = __float_as_uint(vx);
      p[3] = __float_as_uint(vy);
      p[4] = __float_as_uint(pr.rot[j][k + 1]);
    }
  }
  // The fused steady ticks' fast form of advance_prepared: no branch at all.
  // The speed clamp's arithmetic (speed_clamp) is evaluated on every lane and
  // selected where |v| > 7; the operand ranges its short division sequence
  // does not cover (a zero or tiny component, a huge or infinite magnitude)
  // are not handled here but flagged in `special`, and the caller re-runs the
  // whole tick through the general form when any lane of the wave flagged one
  // (kernels.hpp steady_kernel).  On every lane without a flag each f32
  // operation is the one speed_clamp performs, so the bits are the same.
  static constexpr bool kHasFast = true;
  template <int N>
  __device__ static void advance_prepared_fast(uint32_t (&w)[NWL], const Prep<N>& pr, int k, uint32_t& special) {
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      uint32_t* p = &w[5 * j];
      const float old_x = __uint_as_float(p[0]), old_y = __uint_as_float(p[1]);
      float vx = __uint_as_float(p[2]) * kFriction + pr.tx[j][k];
      float vy = __uint_as_float(p[3]) * kFriction + pr.ty[j][k];
      const float m2 = vx * vx + vy * vy;
      const bool clamp = m2 > kMaxSpeed * kMaxSpeed;  // see speed_clamp
      const float mag = sqrt_rn_above_one(clamp ? m2 : 64.0f);
      const float nx = vx * kMaxSpeed, ny = vy * kMaxSpeed;
      const float r = rcp_refined(mag);
      const float qx = div_rn_unscaled(nx, mag, r), qy = div_rn_unscaled(ny, mag, r);
      const bool ok = mag < 256.0f && __builtin_fabsf(nx) >= 0x1p-96f && __builtin_fabsf(ny) >= 0x1p-96f;
      special |= (clamp && !ok) ? 1u : 0u;
      vx = clamp ? qx : vx;
      vy = clamp ? qy : vy;
      float x = old_x + vx, y = old_y + vy;
      x = fminf(fmaxf(x, 0.0f), kWidth);
      y = fminf(fmaxf(y, 0.0f), kHeight);
      p[0] = __float_as_uint(x);
      p[1] = __float_as_uint(y);
      p[2] = __float_as_uint(vx);
      p[3] = __float_as_uint(vy);
      p[4] = __float_as_uint(pr.rot[j][k + 1]);
    }
  }
  // One AdvanceFrame without any branch, for callers that redo the frame in
  // the general form (advance) when any lane of the wave flags `special`: a
  // rotation outside [+0, 6.5) (in_range) or a clamp operand outside the short
  // division sequence.  Unflagged lanes get advance's bits: the rotation step
  // and sincos are the in-range forms (exact there, see in_range), the thrust
  // and clamp the operations of advance_player / advance_prepared_fast.
  __device__ static void advance_fast(uint32_t (&w)[NWL], InRec rec, int lane, uint32_t disconnected_mask,
                                      uint32_t& special) {
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      const int i = kSplit ? lane : j;
      const uint32_t input = ((disconnected_mask >> i) & 1u) ? 4u : player_input(rec, i);  // Disconnected => 4 (:268)
      uint32_t* p = &w[5 * j];
      const float rot = __uint_as_float(p[4]);
      special |= __float_as_uint(rot) < 0x40D00000u ? 0u : 1u;  // +0 <= rot < 6.5
      const bool up = input & 1u, down = input & 2u, left = input & 4u, right = input & 8u;
      const SinCos sc = sincosf_glibc<true>(rot, nullptr);
      const float sp = up ? kMovementSpeed : -kMovementSpeed;
      const float tx = sp * sc.c, ty = sp * sc.s;  // -(S * c) == (-S) * c
      const uint32_t thm = up != down ? ~0u : 0u;
      const float txm = __uint_as_float((thm & __float_as_uint(tx)) | (~thm & 0x80000000u));
      const float tym = __uint_as_float((thm & __float_as_uint(ty)) | (~thm & 0x80000000u));
      const float r1 = rem_euclid_near<true>(rot + (left ? -kRotationSpeed : kRotationSpeed), 2.0f * kPi);
      float vx = __uint_as_float(p[2]) * kFriction + txm;
      float vy = __uint_as_float(p[3]) * kFriction + tym;
      const float m2 = vx * vx + vy * vy;
      const bool clamp = m2 > kMaxSpeed * kMaxSpeed;
      const float mag = sqrt_rn_above_one(clamp ? m2 : 64.0f);
      const float nx = vx * kMaxSpeed, ny = vy * kMaxSpeed;
      const float r = rcp_refined(mag);
      const float qx = div_rn_unscaled(nx, mag, r), qy = div_rn_unscaled(ny, mag, r);
      const bool ok = mag < 256.0f && __builtin_fabsf(nx) >= 0x1p-96f && __builtin_fabsf(ny) >= 0x1p-96f;
      special |= (clamp && !ok) ? 1u : 0u;
      vx = clamp ? qx : vx;
      vy = clamp ? qy : vy;
      float x = __uint_as_float(p[0]) + vx, y = __uint_as_float(p[1]) + vy;
      x = fminf(fmaxf(x, 0.0f), kWidth);
      y = fminf(fmaxf(y, 0.0f), kHeight);
      p[0] = __float_as_uint(x);
      p[1] = __float_as_uint(y);
      p[2] = __float_as_uint(vx);
      p[3] = __float_as_uint(vy);
      p[4] = left != right ? __float_as_uint(r1) : __float_as_uint(rot);
    }
  }
  // A rotation in [+0, 6.5) steps to rot +- 2.5/60 in (-2pi, 4pi), which
  // rem_euclid maps into [+0, 2pi] with one add or subtract (rem_euclid_near;
  // never -0); from there every later step stays in that interval.  So a state
  // whose every rotation is in [+0, 6.5) needs no out-of-line library path
  // (sincos below 120, no fmodf) for any number of AdvanceFrames, and every
  // sincos argument is in [+0, 6.5) (sincosf_glibc's in-range evaluation).
  // Tested on the bits: -0, negatives and NaN are out of range.
  static constexpr bool kHasRangePath = true;
  __device__ static bool in_range(const uint32_t (&w)[NWL]) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      const float r = __uint_as_float(w[5 * j + 4]);
      ok &= __float_as_uint(r) < 0x40D00000u;  // +0 <= r < 6.5f
    }
    return ok;
  }

  // fletcher16(bincode::serialize(&state)) (ex_game.rs:90-91) from registers:
  // closed-form weighted byte sums per lane, summed over the lane group.
  // Constant bytes of the image: num_players and the three Vec lengths (u64 =
  // P, LE) at offsets 4, 12, 20+8P, 28+16P.
  static constexpr uint32_t kCsC1 = 4u * P;
  static constexpr uint32_t kCsC2 =
      P * static_cast<uint32_t>((kImageBytes - 4) + (kImageBytes - 12) + (kImageBytes - 20 - 8 * P) + (kImageBytes - 28 - 16 * P));
  // (n-o, n-o-1, n-o-2, n-o-3): the weights of the 4 bytes of a word at image offset o
  __host__ __device__ static constexpr uint32_t wp(int o) {
    return static_cast<uint32_t>(kImageBytes - o) * 0x01010101u - 0x03020100u;
  }
  __device__ static CS checksum(const uint32_t (&w)[NWL], int32_t frame, int lane, const CsCtx&) {
    constexpr int n = kImageBytes;
    constexpr uint32_t c1 = kCsC1, c2 = kCsC2;
    const bool lead = lane == 0;
    Fl16 a{lead ? c1 : 0u, lead ? c2 : 0u};  // loop-invariant: hoisted by the compiler
#pragma unroll
    for (int j = 0; j < kPlayersPerLane; ++j) {
      const int i = kSplit ? lane : j;
      const uint32_t live = (!kSplit || i < P) ? ~0u : 0u;  // padding lanes of a 4-lane group add nothing
      fl16_word(a, w[5 * j + 0] & live, wp(off_x(i)));
      fl16_word(a, w[5 * j + 1] & live, wp(off_x(i) + 4));
      fl16_word(a, w[5 * j + 2] & live, wp(off_vx(i)));
      fl16_word(a, w[5 * j + 3] & live, wp(off_vx(i) + 4));
      fl16_word(a, w[5 * j + 4] & live, wp(off_rot(i)));
    }
    a.s1 = group_sum<kLanes>(a.s1);
    a.s2 = group_sum<kLanes>(a.s2);
    fl16_word(a, static_cast<uint32_t>(frame), fl16_weights(n, 0));  // the frame word, once per session
    return fl16_finish(a);
  }

  // ---- independent players (the in-kernel speculative fan-out, p2p.hpp
  // inlane_fan): State::advance (:259-321) moves every player from its own
  // input alone, so the branches of the speculated player are simulated on
  // that player's words alone and the other players keep the main
  // trajectory's.  The checksum of a branch cell is then assembled from
  // per-player parts: fan_partial of each player's words, summed, and fan_finish.
  static constexpr bool kIndependentPlayers = kSplit;
  __device__ static Fl16 fan_partial(const uint32_t (&w)[NWL], int i) {  // player i's words (one player per lane)
    Fl16 a{0u, 0u};
    fl16_word(a, w[0], wp(off_x(i)));
    fl16_word(a, w[1], wp(off_x(i) + 4));
    fl16_word(a, w[2], wp(off_vx(i)));
    fl16_word(a, w[3], wp(off_vx(i) + 4));
    fl16_word(a, w[4], wp(off_rot(i)));
    return a;
  }
  // The per-player fan-out's shared rotation (p2p.hpp fan_per_player, FanShare): a player's input
  // classes that turn alike (class bits 2-3) share the rotation and its sine / cosine over the
  // frames they hold, so one AdvanceFrame splits into fan_turn (once per turn group and frame) and
  // fan_move (per class).  Each is advance_player's operations on the same operands: bit-identical.
  static constexpr bool kFanShare = kSplit;
  template <bool kInRange>
  __device__ static float fan_turn(float rot, uint32_t cls) {  // the rotation after the frame (:291-296)
    const bool left = cls & 4u, right = cls & 8u;
    const float r1 = rem_euclid<kInRange>(left ? rot - kRotationSpeed : rot + kRotationSpeed, 2.0f * kPi);
    return left != right ? r1 : rot;
  }
  // friction, thrust (tx, ty = MOVEMENT_SPEED * (cos, sin)(rotation before the frame)), speed clamp
  // and position (:277-289, :298-314) of one player's words; the rotation word is the caller's
  __device__ static void fan_move(uint32_t* w, float tx, float ty, uint32_t cls) {
    const float old_x = __uint_as_float(w[0]), old_y = __uint_as_float(w[1]);
    float vx = __uint_as_float(w[2]) * kFriction;
    float vy = __uint_as_float(w[3]) * kFriction;
    const bool up = cls & 1u, down = cls & 2u;
    const float vx1 = up ? vx + tx : vx - tx, vy1 = up ? vy + ty : vy - ty;
    vx = up != down ? vx1 : vx;
    vy = up != down ? vy1 : vy;
    speed_clamp(vx, vy);
    float x = old_x + vx, y = old_y + vy;
    x = fminf(fmaxf(x, 0.0f), kWidth);
    y = fminf(fmaxf(y, 0.0f), kHeight);
    w[0] = __float_as_uint(x);
    w[1] = __float_as_uint(y);
    w[2] = __float_as_uint(vx);
    w[3] = __float_as_uint(vy);
  }
  template <bool kInRange>
  __device__ static SinCos fan_thrust(float rot, uint32_t* unexpected) {  // MOVEMENT_SPEED * (cos, sin)(rot)
    const SinCos sc = sincosf_glibc<kInRange>(rot, unexpected);
    return SinCos{kMovementSpeed * sc.s, kMovementSpeed * sc.c};
  }
  __device__ static CS fan_finish(Fl16 a, int32_t frame) {  // + the constant bytes and the frame word
    a.s1 += kCsC1;
    a.s2 += kCsC2;
    fl16_word(a, static_cast<uint32_t>(frame), fl16_weights(kImageBytes, 0));
    return fl16_finish(a);
  }
};

// G::kFanShare (ExGame::fan_turn / fan_move / fan_thrust), false for a game that does not declare it
template <class G, class = void>
struct FanShare {
  static constexpr bool value = false;
};
template <class G>
struct FanShare<G, std::void_t<decltype(G::kFanShare)>> {
  static constexpr bool value = G::kFanShare;
};

// G::kIndependentPlayers, false for a game that does not declare it
template <class G, class = void>
struct IndepPlayers {
  static constexpr bool value = false;
};
template <class G>
struct IndepPlayers<G, std::void_t<decltype(G::kIndependentPlayers)>> {
  static constexpr bool value = G::kIndependentPlayers;
};

// Sum of a u32 over the 64 lanes of a wave (butterfly over ds_swizzle/bpermute);
// every lane receives the total.
__device__ __forceinline__ uint32_t wave_sum64(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), m, 64));
  return v;
}

// ============================================================================
// BASELINE config 3: fixed-point 256-entity brawler (no reference game; the
// definition is oracle/ggrs_oracle.hpp namespace brawler, restated here).
// One wavefront per session: lane l holds entities l, 64+l, 128+l, 192+l
// (8 words each, 32 VGPRs); the players are entities 0..P-1 = lanes 0..P-1.
// ============================================================================
template <int P>
struct Brawler {
  static_assert(P >= 1 && P <= 4, "brawler supports 1..4 players");
  static constexpr int kPlayers = P;
  static constexpr int kLanes = 64;
  static constexpr int kEntities = 256, kEntPerLane = 4;
  static constexpr int NWL = 8 * kEntPerLane;
  static constexpr int kInputBytes = 1;
  static constexpr int kImageBytes = 4 + kEntities * 32;  // le32 frame || entities
  static constexpr bool kDisplay = false;
  static constexpr int kCanonWords = kEntities * 8;
  using InRec = typename InRecOf<P>::T;
  using CS = uint16_t;

  static constexpr int32_t kArena = 1 << 20;
  static constexpr int32_t kPlayerAcc = 1 << 12, kPlayerVmax = 1 << 14;
  static constexpr int32_t kAiAcc = 1 << 10, kAiVmax = 1 << 13;
  static constexpr int32_t kContact = 1 << 14;
  static constexpr int32_t kAttackCd = 8, kAiDamage = 25, kPlayerHp0 = 1000, kAiHp0 = 100;
  static constexpr uint64_t kInitKey = 0x627261776C6572ULL;
  enum { X = 0, Y, VX, VY, HP, FLAGS, RNG, COUNTER };

  // State::make (oracle brawler::State::make); words [64 lanes][32]
  static void init(uint32_t* words) {
    for (int e = 0; e < kEntities; ++e) {
      const uint64_t h = splitmix64(kInitKey ^ static_cast<uint64_t>(e));
      uint32_t* w = words + (e % 64) * NWL + (e / 64) * 8;
      w[X] = static_cast<uint32_t>(h & (kArena - 1));
      w[Y] = static_cast<uint32_t>((h >> 20) & (kArena - 1));
      w[VX] = w[VY] = 0;
      w[HP] = static_cast<uint32_t>(e < P ? kPlayerHp0 : kAiHp0);
      w[FLAGS] = static_cast<uint32_t>(e < P ? 0 : e % P);
      w[RNG] = static_cast<uint32_t>(h >> 32) | 1u;
      w[COUNTER] = 0;
    }
  }
  static void image(const uint32_t* words, int32_t frame, uint8_t* out) {
    std::memcpy(out, &frame, 4);
    for (int e = 0; e < kEntities; ++e) std::memcpy(out + 4 + 32 * e, words + (e % 64) * NWL + (e / 64) * 8, 32);
  }
  static void word_loc(int k, int* lane, int* word) {
    const int e = k / 8, f = k % 8;
    *lane = e % 64;
    *word = (e / 64) * 8 + f;
  }

  __device__ static int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }
  __device__ static int32_t sgn(int32_t v) { return (v > 0) - (v < 0); }
  __device__ static int32_t iabs(int32_t v) { return v < 0 ? -v : v; }
  template <class T>
  __device__ static T pick(const T (&a)[P], int32_t t) {  // a[t] for a per-lane t < P, no scratch
    T r = a[0];
#pragma unroll
    for (int i = 1; i < P; ++i) r = t == i ? a[i] : r;
    return r;
  }

  // State::advance (oracle brawler::State::advance): players, then AI against
  // the players' new positions, then the damage the players took.
  static constexpr bool kHasRangePath = false;
  static constexpr bool kHasPrep = false;  // plain advance in the fused steady ticks
  static constexpr bool kUsesStatus = false;
  __device__ static bool in_range(const uint32_t (&)[NWL]) { return false; }
  template <bool = false>
  __device__ static void advance(uint32_t (&w)[NWL], InRec rec, int lane, uint32_t disc, uint32_t*) {
    if (lane < P) {  // phase 1: player `lane` (entity lane, slot 0)
      const uint32_t in = ((disc >> lane) & 1u) ? 0u : (static_cast<uint32_t>(rec) >> (8 * lane)) & 0xFFu;
      const int32_t ax = static_cast<int32_t>((in >> 3) & 1u) - static_cast<int32_t>((in >> 2) & 1u);
      const int32_t ay = static_cast<int32_t>((in >> 1) & 1u) - static_cast<int32_t>(in & 1u);
      int32_t vx = static_cast<int32_t>(w[VX]), vy = static_cast<int32_t>(w[VY]);
      vx = clampi(vx - (vx >> 3) + ax * kPlayerAcc, -kPlayerVmax, kPlayerVmax);
      vy = clampi(vy - (vy >> 3) + ay * kPlayerAcc, -kPlayerVmax, kPlayerVmax);
      w[VX] = static_cast<uint32_t>(vx);
      w[VY] = static_cast<uint32_t>(vy);
      w[X] = static_cast<uint32_t>(clampi(static_cast<int32_t>(w[X]) + vx, 0, kArena - 1));
      w[Y] = static_cast<uint32_t>(clampi(static_cast<int32_t>(w[Y]) + vy, 0, kArena - 1));
      int32_t cd = static_cast<int32_t>(w[FLAGS] & 0xFFu), atk = 0;
      if ((in & 16u) && cd == 0) {
        cd = kAttackCd;
        atk = 1;
      } else {
        cd = cd > 0 ? cd - 1 : 0;
      }
      w[FLAGS] = static_cast<uint32_t>(cd | (atk << 8));
    }
    int32_t px[P], py[P], pa[P];
#pragma unroll
    for (int t = 0; t < P; ++t) {  // scalar broadcasts of the players' new state
      px[t] = __builtin_amdgcn_readlane(static_cast<int>(w[X]), t);
      py[t] = __builtin_amdgcn_readlane(static_cast<int>(w[Y]), t);
      pa[t] = (__builtin_amdgcn_readlane(static_cast<int>(w[FLAGS]), t) >> 8) & 1;
    }
    uint32_t hits = 0;  // 8-bit count per player (at most 255 AI entities)
#pragma unroll
    for (int j = 0; j < kEntPerLane; ++j) {  // phase 2: AI entities j*64 + lane
      uint32_t* q = &w[8 * j];
      const bool ai = j > 0 || lane >= P;
      if (!ai || static_cast<int32_t>(q[HP]) <= 0) continue;
      const int32_t t = static_cast<int32_t>(q[FLAGS]);
      const int32_t tx = pick(px, t), ty = pick(py, t), ta = pick(pa, t);
      uint32_t r = q[RNG];
      r ^= r << 13;
      r ^= r >> 17;
      r ^= r << 5;
      q[RNG] = r;
      const int32_t jx = static_cast<int32_t>(r & 0xFFu) - 128, jy = static_cast<int32_t>((r >> 8) & 0xFFu) - 128;
      int32_t x = static_cast<int32_t>(q[X]), y = static_cast<int32_t>(q[Y]);
      int32_t vx = static_cast<int32_t>(q[VX]), vy = static_cast<int32_t>(q[VY]);
      vx = clampi(vx - (vx >> 2) + sgn(tx - x) * kAiAcc + jx, -kAiVmax, kAiVmax);
      vy = clampi(vy - (vy >> 2) + sgn(ty - y) * kAiAcc + jy, -kAiVmax, kAiVmax);
      x = clampi(x + vx, 0, kArena - 1);
      y = clampi(y + vy, 0, kArena - 1);
      q[X] = static_cast<uint32_t>(x);
      q[Y] = static_cast<uint32_t>(y);
      q[VX] = static_cast<uint32_t>(vx);
      q[VY] = static_cast<uint32_t>(vy);
      q[COUNTER] += 1u;
      if (iabs(tx - x) + iabs(ty - y) < kContact) {
        if (ta) {
          const int32_t hp = static_cast<int32_t>(q[HP]) - kAiDamage;
          q[HP] = static_cast<uint32_t>(hp < 0 ? 0 : hp);
        } else {
          hits += 1u << (8 * t);
        }
      }
    }
    hits = wave_sum64(hits);
    if (lane < P) {  // phase 3
      const int32_t dmg = static_cast<int32_t>((hits >> (8 * lane)) & 0xFFu);
      const int32_t hp = static_cast<int32_t>(w[HP]) - dmg;
      w[HP] = static_cast<uint32_t>(hp < 0 ? 0 : hp);
      w[COUNTER] += static_cast<uint32_t>(dmg);
    }
  }

  // fletcher16 of the 8196-byte image from registers: s1 = sum(b) mod 255,
  // s2 = (n * sum(b) - sum(i * b)) mod 255.  Word f of entity e = j*64+lane sits
  // at image offset o = 4 + 32e + 4f = (4 + 2048j + 4f) + 32*lane; per word two
  // v_dot4_u32_u8 give its byte sum and sum(byte index * byte); per-lane sums are
  // reduced mod 255 and packed before one wave butterfly.
  __device__ static CS checksum(const uint32_t (&w)[NWL], int32_t frame, int lane, const CsCtx&) {
    uint32_t sb = 0, sib = 0;
#pragma unroll
    for (int j = 0; j < kEntPerLane; ++j)
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        const uint32_t v = w[8 * j + f];
        const uint32_t bs = __builtin_amdgcn_udot4(v, 0x01010101u, 0u, false);
        sb += bs;
        sib = __builtin_amdgcn_udot4(v, 0x03020100u, sib, false) + static_cast<uint32_t>(4 + 2048 * j + 4 * f) * bs;
      }
    sib += 32u * static_cast<uint32_t>(lane) * sb;
    if (lane == 0) {  // frame word at offset 0
      const uint32_t fr = static_cast<uint32_t>(frame);
      sb = __builtin_amdgcn_udot4(fr, 0x01010101u, sb, false);
      sib = __builtin_amdgcn_udot4(fr, 0x03020100u, sib, false);
    }
    const uint32_t tot = wave_sum64(((sib % 255u) << 16) | (sb % 255u));
    const uint32_t s1 = (tot & 0xFFFFu) % 255u, b = (tot >> 16) % 255u;
    constexpr uint32_t n_mod = static_cast<uint32_t>(kImageBytes) % 255u;
    const uint32_t s2 = (n_mod * s1 + 255u - b) % 255u;
    return static_cast<CS>((s2 << 8) | s1);
  }
};

// ============================================================================
// tests/stubs.rs GameStub / StateStub
// ============================================================================
struct StubGame {
  static constexpr int kPlayers = 2;  // StateStub::advance_frame reads inputs[0], inputs[1]
  static constexpr int kLanes = 1;
  static constexpr int NWL = 1;  // state (frame comes from the cell tag)
  static constexpr int kInputBytes = 4;
  static constexpr int kImageBytes = 8;
  static constexpr bool kDisplay = false;
  using InRec = uint64_t;  // two StubInput{inp:u32}
  using CS = uint64_t;     // DefaultHasher::finish() as u128

  static void init(uint32_t* w) { w[0] = 0; }
  static void image(const uint32_t* w, int32_t frame, uint8_t* out) {
    std::memcpy(out, &frame, 4);
    std::memcpy(out + 4, &w[0], 4);
  }
  static U128 cs128(CS c) { return U128{c, 0}; }
  static void word_loc(int, int* lane, int* word) { *lane = 0; *word = 0; }
  static constexpr int kCanonWords = 1;
  __device__ static uint32_t player_input(InRec rec, int p) { return static_cast<uint32_t>(rec >> (32 * p)); }
  // stubs.rs:115-125
  static constexpr bool kHasRangePath = false;
  static constexpr bool kHasPrep = false;  // plain advance in the fused steady ticks
  static constexpr bool kUsesStatus = false;
  __device__ static bool in_range(const uint32_t (&)[NWL]) { return false; }
  template <bool = false>
  __device__ static void advance(uint32_t (&w)[NWL], InRec rec, int, uint32_t, uint32_t*) {
    const uint32_t p0 = player_input(rec, 0), p1 = player_input(rec, 1);
    w[0] = ((p0 + p1) % 2u == 0u) ? w[0] + 2u : w[0] - 1u;
  }
  // calculate_hash(&StateStub{frame, state}) (stubs.rs:8-12, 54)
  __device__ static CS checksum(const uint32_t (&w)[NWL], int32_t frame, int, const CsCtx&) {
    return siphash13_i32x2(frame, static_cast<int32_t>(w[0]));
  }
};

// tests/stubs_enum.rs GameStubEnum: EnumInput #[repr(u8)] {Val1, Val2}
struct StubEnumGame {
  static constexpr int kPlayers = 2;
  static constexpr int kLanes = 1;
  static constexpr int NWL = 1;
  static constexpr int kInputBytes = 1;
  static constexpr int kImageBytes = 8;
  static constexpr bool kDisplay = false;
  using InRec = uint16_t;
  using CS = uint64_t;
  static void init(uint32_t* w) { w[0] = 0; }
  static void image(const uint32_t* w, int32_t frame, uint8_t* out) { StubGame::image(w, frame, out); }
  static U128 cs128(CS c) { return U128{c, 0}; }
  static void word_loc(int, int* lane, int* word) { *lane = 0; *word = 0; }
  static constexpr int kCanonWords = 1;
  __device__ static uint32_t player_input(InRec rec, int p) { return (static_cast<uint32_t>(rec) >> (8 * p)) & 0xffu; }
  // StateStubEnum::advance_frame (stubs_enum.rs:80-90): `p0_inputs == p1_inputs`
  // compares (EnumInput, InputStatus) tuples.  InputStatus of player i from the
  // status bits: bit i Disconnected (its input is zeroed), bit 8+i Predicted.
  static constexpr bool kHasRangePath = false;
  static constexpr bool kHasPrep = false;  // plain advance in the fused steady ticks
  static constexpr bool kUsesStatus = true;  // Predicted bits (8 + i) too
  __device__ static bool in_range(const uint32_t (&)[NWL]) { return false; }
  __device__ static uint32_t status_of(uint32_t bits, int i) {
    return ((bits >> i) & 1u) ? 2u : ((bits >> (8 + i)) & 1u);  // Disconnected 2, Predicted 1, Confirmed 0
  }
  template <bool = false>
  __device__ static void advance(uint32_t (&w)[NWL], InRec rec, int, uint32_t status_bits, uint32_t*) {
    const bool same = player_input(rec, 0) == player_input(rec, 1) && status_of(status_bits, 0) == status_of(status_bits, 1);
    w[0] = same ? w[0] + 2u : w[0] - 1u;
  }
  __device__ static CS checksum(const uint32_t (&w)[NWL], int32_t frame, int, const CsCtx&) {
    return siphash13_i32x2(frame, static_cast<int32_t>(w[0]));
  }
};

// tests/stubs.rs:67-106 RandomChecksumGameStub: a fresh random u128 on every
// save (counter-based: splitmix64 of seed/session/save nonce).
struct StubRandomCsGame : StubGame {
  using CS = U128;
  __device__ static CS checksum(const uint32_t (&)[NWL], int32_t frame, int, const CsCtx& c) {
    const uint64_t k = c.seed ^ (static_cast<uint64_t>(c.session) << 32) ^ c.nonce ^ (static_cast<uint64_t>(frame) << 48);
    return U128{splitmix64(k), splitmix64(k ^ 0x5bd1e995ULL)};
  }
  static U128 cs128(CS c) { return c; }
};

// ============================================================================
// A user's game (include/ggrs_amd_game.hpp contract) adapted to the engine's
// game interface: one lane per session, frame supplied by the cell tag, image
// = le32 frame || le32 words.  Instantiated by ggrs_amd/csrc/plugin.hip into a
// plugin library (rb_register_game_plugin).
// ============================================================================
template <int Bytes>
struct PackedInRec {
  using T = uint64_t;
};
template <>
struct PackedInRec<1> {
  using T = uint8_t;
};
template <>
struct PackedInRec<2> {
  using T = uint16_t;
};
template <>
struct PackedInRec<3> {
  using T = uint32_t;
};
template <>
struct PackedInRec<4> {
  using T = uint32_t;
};

template <class U>
struct PluginGame {
  static_assert(U::kPlayers >= 1 && U::kPlayers <= 4, "plugin games have 1..4 players");
  static_assert(U::kInputBytes == 1 || U::kInputBytes == 2 || U::kInputBytes == 4, "Input is 1, 2 or 4 bytes");
  static_assert(U::kPlayers * U::kInputBytes <= 8, "all players' inputs of a frame must pack into 8 bytes");
  static_assert(U::kStateWords >= 1 && U::kStateWords <= 64, "1..64 state words");
  static constexpr int kPlayers = U::kPlayers;
  static constexpr int kLanes = 1;
  static constexpr int NWL = U::kStateWords;
  static constexpr int kInputBytes = U::kInputBytes;
  static constexpr int kImageBytes = 4 + 4 * NWL;
  static constexpr bool kDisplay = false;
  static constexpr int kCanonWords = NWL;
  static constexpr bool kHasRangePath = false;
  static constexpr bool kHasPrep = false;
  static constexpr bool kUsesStatus = true;
  using InRec = typename PackedInRec<kPlayers * kInputBytes>::T;
  using CS = typename U::Checksum;

  static void init(uint32_t* w) { U::init(w); }
  static void image(const uint32_t* w, int32_t frame, uint8_t* out) {
    std::memcpy(out, &frame, 4);
    std::memcpy(out + 4, w, 4 * NWL);
  }
  static void word_loc(int k, int* lane, int* word) {
    *lane = 0;
    *word = k;
  }
  __device__ static bool in_range(const uint32_t (&)[NWL]) { return false; }
  template <bool = false>
  __device__ static void advance(uint32_t (&w)[NWL], InRec rec, int, uint32_t status_bits, uint32_t*) {
    uint32_t in[kPlayers];
    uint8_t st[kPlayers];
#pragma unroll
    for (int p = 0; p < kPlayers; ++p) {
      const uint64_t v = static_cast<uint64_t>(rec) >> (8 * kInputBytes * p);
      in[p] = static_cast<uint32_t>(kInputBytes == 4 ? v & 0xffffffffull : v & ((1ull << (8 * kInputBytes)) - 1));
      st[p] = static_cast<uint8_t>(((status_bits >> p) & 1u) ? 2u : ((status_bits >> (8 + p)) & 1u));
    }
    U::advance(w, in, st);
  }
  __device__ static CS checksum(const uint32_t (&w)[NWL], int32_t frame, int, const CsCtx&) {
    return U::checksum(w, frame);
  }
};

}  // namespace rb
