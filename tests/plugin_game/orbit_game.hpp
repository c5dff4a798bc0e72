// tests/plugin_game/orbit_game.hpp — a game defined OUTSIDE the engine
// (include/ggrs_amd_game.hpp contract), compiled into a plugin library by
// __graft_entry__.build() and into the oracle by oracle/Makefile's plugin
// target.  It proves the handler plug-in path end to end: nothing in
// ggrs_amd/csrc knows this game.
//
// Three players steer integer ships on a 2^20 x 2^20 torus (Q8 velocities):
// inputs are 5 bits (left, right, up, down, boost); the checksum is 64-bit
// FNV-1a over the le32 image (frame || words).  The game also folds every
// player's InputStatus into a word, so Predicted / Disconnected inputs change
// its state exactly as they would in a reference handler that reads them.
#pragma once
#include "../../include/ggrs_amd_game.hpp"

struct OrbitGame {
  static constexpr int kPlayers = 3;
  static constexpr int kStateWords = 4 * kPlayers + 3;  // per player x, y, vx, vy; rng, hits, status mix
  static constexpr int kInputBytes = 1;
  using Checksum = uint64_t;
  static constexpr int32_t kArenaMask = (1 << 20) - 1;
  static constexpr int32_t kVmax = 8192, kAcc = 256, kNear = 4096;
  enum { RNG = 4 * kPlayers, HITS, MIX };

  static void init(uint32_t* w) {
    for (int p = 0; p < kPlayers; ++p) {
      w[4 * p + 0] = static_cast<uint32_t>((p * 340000 + 12345) & kArenaMask);
      w[4 * p + 1] = static_cast<uint32_t>((p * 270000 + 54321) & kArenaMask);
      w[4 * p + 2] = 0;
      w[4 * p + 3] = 0;
    }
    w[RNG] = 0x9E3779B9u;
    w[HITS] = 0;
    w[MIX] = 1;
  }

  RB_GAME_FN static int32_t clampv(int32_t v) { return v < -kVmax ? -kVmax : (v > kVmax ? kVmax : v); }
  RB_GAME_FN static int32_t iabs(int32_t v) { return v < 0 ? -v : v; }

  RB_GAME_FN static void advance(uint32_t* w, const uint32_t* inputs, const uint8_t* status) {
    uint32_t r = w[RNG];
    for (int p = 0; p < kPlayers; ++p) {
      const uint32_t in = inputs[p];
      const int32_t ax = static_cast<int32_t>((in >> 3) & 1u) - static_cast<int32_t>((in >> 2) & 1u);
      const int32_t ay = static_cast<int32_t>((in >> 1) & 1u) - static_cast<int32_t>(in & 1u);
      const int32_t acc = kAcc << ((in >> 4) & 1u);
      r ^= r << 13;
      r ^= r >> 17;
      r ^= r << 5;
      const int32_t jitter = static_cast<int32_t>(r & 63u) - 32;
      int32_t vx = static_cast<int32_t>(w[4 * p + 2]), vy = static_cast<int32_t>(w[4 * p + 3]);
      vx = clampv(vx - vx / 16 + ax * acc + jitter);
      vy = clampv(vy - vy / 16 + ay * acc - jitter);
      w[4 * p + 0] = (w[4 * p + 0] + static_cast<uint32_t>(vx)) & static_cast<uint32_t>(kArenaMask);
      w[4 * p + 1] = (w[4 * p + 1] + static_cast<uint32_t>(vy)) & static_cast<uint32_t>(kArenaMask);
      w[4 * p + 2] = static_cast<uint32_t>(vx);
      w[4 * p + 3] = static_cast<uint32_t>(vy);
      w[MIX] = w[MIX] * 3u + status[p];  // InputStatus: 0 Confirmed, 1 Predicted, 2 Disconnected
    }
    w[RNG] = r;
    for (int i = 0; i < kPlayers; ++i)
      for (int j = i + 1; j < kPlayers; ++j) {
        const int32_t dx = static_cast<int32_t>(w[4 * i]) - static_cast<int32_t>(w[4 * j]);
        const int32_t dy = static_cast<int32_t>(w[4 * i + 1]) - static_cast<int32_t>(w[4 * j + 1]);
        if (iabs(dx) + iabs(dy) < kNear) w[HITS] += 1u;
      }
  }

  RB_GAME_FN static Checksum checksum(const uint32_t* w, int32_t frame) {
    uint64_t h = 0xcbf29ce484222325ull;
    auto word = [&h](uint32_t v) {
      for (int b = 0; b < 4; ++b) {
        h ^= (v >> (8 * b)) & 0xffu;
        h *= 0x100000001b3ull;
      }
    };
    word(static_cast<uint32_t>(frame));
    for (int k = 0; k < kStateWords; ++k) word(w[k]);
    return h;
  }
};
