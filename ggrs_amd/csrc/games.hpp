// ggrs_amd/csrc/games.hpp — the compiled-in request handlers.
//
// A game plugs into the engine with (the `Config` trait of lib.rs:240-262 plus
// the user's handle_requests of ex_game.rs:76-84, as device code):
//   NW        state words per session stored in a snapshot slot (u32 each)
//   InRec     one session's packed inputs for one frame (P Input values)
//   CS        checksum type stored per cell (zero-extended to u128 on export)
//   init      host: State::new words
//   advance   device: one AdvanceFrame on the register-resident state
//   checksum  device: the checksum the game's save_game_state stores
//   image     host: canonical byte image of (frame, words) for read-back
// The cell's frame tag is stored once per slot (batch-uniform): every game
// here asserts state.frame == cell frame on save (ex_game.rs:89,
// stubs.rs:53,93, stubs_enum.rs:185), so the per-session frame word is
// redundant and is supplied from the tag instead of being stored S times.
#pragma once

#include <cmath>
#include <cstring>

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

// ============================================================================
// examples/ex_game/ex_game.rs
// ============================================================================
template <int P>
struct ExGame {
  static_assert(P >= 1 && P <= 4, "ex_game supports 1..4 players (ex_game.rs:65)");
  static constexpr int kPlayers = P;
  static constexpr int NW = 5 * P;  // bincode order: positions (x,y)*P, velocities (x,y)*P, rotations*P
  static constexpr int kInputBytes = 1;
  static constexpr int kImageBytes = 36 + 20 * P;  // bincode 1.3 image of State (ex_game.rs:224-231)
  using InRec = typename InRecOf<P>::T;
  using CS = uint16_t;

  // ex_game.rs:8-24
  static constexpr float kFriction = 0.98f;
  static constexpr float kMovementSpeed = 15.0f / 60.0f;
  static constexpr float kRotationSpeed = 2.5f / 60.0f;
  static constexpr float kMaxSpeed = 7.0f;
  static constexpr float kWidth = 600.0f, kHeight = 800.0f;
  static constexpr float kPi = 3.14159265358979323846f;

  // State::new (ex_game.rs:234-257), evaluated with the host libm like the
  // reference (glibc cosf/sinf/fmodf).
  static void init(uint32_t* w) {
    const float r = kWidth / 4.0f;
    for (int i = 0; i < P; ++i) {
      // volatile: keep the compiler from constant-folding libm calls with its
      // own (correctly rounded) evaluation; the reference calls glibc at run time.
      volatile float fi = static_cast<float>(i), fp = static_cast<float>(P);
      float rot = fi / fp * 2.0f * kPi;
      float x = kWidth / 2.0f + r * std::cos(rot);
      float y = kHeight / 2.0f + r * std::sin(rot);
      float ro = std::fmod(rot + kPi, 2.0f * kPi);
      std::memcpy(&w[2 * i], &x, 4);
      std::memcpy(&w[2 * i + 1], &y, 4);
      w[2 * P + 2 * i] = 0;
      w[2 * P + 2 * i + 1] = 0;
      std::memcpy(&w[4 * P + i], &ro, 4);
    }
  }

  __device__ static uint32_t player_input(InRec rec, int p) { return (static_cast<uint32_t>(rec) >> (8 * p)) & 0xffu; }

  // State::advance (ex_game.rs:259-321).  Compiled with -ffp-contract=off:
  // every f32 operation rounds exactly as the reference's.
  __device__ static void advance(uint32_t (&w)[NW], InRec rec, uint32_t disconnected_mask, uint32_t* unexpected) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const uint32_t input = ((disconnected_mask >> i) & 1u) ? 4u : player_input(rec, i);
      const float old_x = __uint_as_float(w[2 * i]), old_y = __uint_as_float(w[2 * i + 1]);
      const float old_vx = __uint_as_float(w[2 * P + 2 * i]), old_vy = __uint_as_float(w[2 * P + 2 * i + 1]);
      float rot = __uint_as_float(w[4 * P + i]);
      float vx = old_vx * kFriction;
      float vy = old_vy * kFriction;
      const bool up = input & 1u, down = input & 2u, left = input & 4u, right = input & 8u;
      if (up != down) {  // thrust (:281-284) or brake (:286-289): exactly one of them
        SinCos sc = sincosf_glibc(rot, unexpected);
        const float tx = kMovementSpeed * sc.c, ty = kMovementSpeed * sc.s;
        if (up) {
          vx = vx + tx;
          vy = vy + ty;
        } else {
          vx = vx - tx;
          vy = vy - ty;
        }
      }
      if (left != right) rot = rem_euclid(left ? rot - kRotationSpeed : rot + kRotationSpeed, 2.0f * kPi);
      const float mag = __builtin_sqrtf(vx * vx + vy * vy);
      if (mag > kMaxSpeed) {
        vx = (vx * kMaxSpeed) / mag;
        vy = (vy * kMaxSpeed) / mag;
      }
      float x = old_x + vx, y = old_y + vy;
      x = fminf(fmaxf(x, 0.0f), kWidth);
      y = fminf(fmaxf(y, 0.0f), kHeight);
      w[2 * i] = __float_as_uint(x);
      w[2 * i + 1] = __float_as_uint(y);
      w[2 * P + 2 * i] = __float_as_uint(vx);
      w[2 * P + 2 * i + 1] = __float_as_uint(vy);
      w[4 * P + i] = __float_as_uint(rot);
    }
  }

  // Byte offset of state word k inside the bincode image.
  __host__ __device__ static constexpr int word_offset(int k) {
    return 20 + 4 * k + (k >= 2 * P ? 8 : 0) + (k >= 4 * P ? 8 : 0);
  }

  // fletcher16(bincode::serialize(&state)) (ex_game.rs:90-91) from registers.
  __device__ static CS checksum(const uint32_t (&w)[NW], int32_t frame, const CsCtx&) {
    constexpr int n = kImageBytes;
    // constant bytes: num_players and the three Vec lengths (u64 = P, LE) at
    // offsets 4, 12, 20+8P, 28+16P
    constexpr uint32_t c1 = 4u * P;
    constexpr uint32_t c2 = P * static_cast<uint32_t>((n - 4) + (n - 12) + (n - 20 - 8 * P) + (n - 28 - 16 * P));
    Fl16 a{c1, c2};
    fl16_word(a, static_cast<uint32_t>(frame), fl16_weights(n, 0));
#pragma unroll
    for (int k = 0; k < NW; ++k) fl16_word(a, w[k], fl16_weights(n, word_offset(k)));
    return fl16_finish(a);
  }

  static void image(const uint32_t* w, int32_t frame, uint8_t* out) {
    std::memset(out, 0, kImageBytes);
    std::memcpy(out, &frame, 4);
    const uint64_t np = P;
    std::memcpy(out + 4, &np, 8);
    std::memcpy(out + 12, &np, 8);
    std::memcpy(out + 20 + 8 * P, &np, 8);
    std::memcpy(out + 28 + 16 * P, &np, 8);
    for (int k = 0; k < NW; ++k) std::memcpy(out + word_offset(k), &w[k], 4);
  }
  static U128 cs128(CS c) { return U128{c, 0}; }
};

// ============================================================================
// tests/stubs.rs GameStub / StateStub
// ============================================================================
struct StubGame {
  static constexpr int kPlayers = 2;  // StateStub::advance_frame reads inputs[0], inputs[1]
  static constexpr int NW = 1;        // state (frame comes from the cell tag)
  static constexpr int kInputBytes = 4;
  static constexpr int kImageBytes = 8;
  using InRec = uint64_t;  // two StubInput{inp:u32}
  using CS = uint64_t;     // DefaultHasher::finish() as u128

  static void init(uint32_t* w) { w[0] = 0; }
  __device__ static uint32_t player_input(InRec rec, int p) { return static_cast<uint32_t>(rec >> (32 * p)); }
  // stubs.rs:115-125
  __device__ static void advance(uint32_t (&w)[NW], InRec rec, uint32_t, uint32_t*) {
    const uint32_t p0 = player_input(rec, 0), p1 = player_input(rec, 1);
    w[0] = ((p0 + p1) % 2u == 0u) ? w[0] + 2u : w[0] - 1u;
  }
  // calculate_hash(&StateStub{frame, state}) (stubs.rs:8-12, 54)
  __device__ static CS checksum(const uint32_t (&w)[NW], int32_t frame, const CsCtx&) {
    return siphash13_i32x2(frame, static_cast<int32_t>(w[0]));
  }
  static void image(const uint32_t* w, int32_t frame, uint8_t* out) {
    std::memcpy(out, &frame, 4);
    std::memcpy(out + 4, &w[0], 4);
  }
  static U128 cs128(CS c) { return U128{c, 0}; }
};

// tests/stubs_enum.rs GameStubEnum: EnumInput #[repr(u8)] {Val1, Val2}
struct StubEnumGame {
  static constexpr int kPlayers = 2;
  static constexpr int NW = 1;
  static constexpr int kInputBytes = 1;
  static constexpr int kImageBytes = 8;
  using InRec = uint16_t;
  using CS = uint64_t;
  static void init(uint32_t* w) { w[0] = 0; }
  __device__ static uint32_t player_input(InRec rec, int p) { return (static_cast<uint32_t>(rec) >> (8 * p)) & 0xffu; }
  // stubs_enum.rs:206-216
  __device__ static void advance(uint32_t (&w)[NW], InRec rec, uint32_t, uint32_t*) {
    w[0] = (player_input(rec, 0) == player_input(rec, 1)) ? w[0] + 2u : w[0] - 1u;
  }
  __device__ static CS checksum(const uint32_t (&w)[NW], int32_t frame, const CsCtx&) {
    return siphash13_i32x2(frame, static_cast<int32_t>(w[0]));
  }
  static void image(const uint32_t* w, int32_t frame, uint8_t* out) { StubGame::image(w, frame, out); }
  static U128 cs128(CS c) { return U128{c, 0}; }
};

// tests/stubs.rs:67-106 RandomChecksumGameStub: a fresh random u128 on every
// save (counter-based: splitmix64 of seed/session/save nonce).
struct StubRandomCsGame : StubGame {
  using CS = U128;
  __device__ static CS checksum(const uint32_t (&)[NW], int32_t frame, const CsCtx& c) {
    const uint64_t k = c.seed ^ (static_cast<uint64_t>(c.session) << 32) ^ c.nonce ^ (static_cast<uint64_t>(frame) << 48);
    return U128{splitmix64(k), splitmix64(k ^ 0x5bd1e995ULL)};
  }
  static U128 cs128(CS c) { return c; }
};

}  // namespace rb
