// oracle/soa_baseline.cpp — TEST AND BASELINE INFRASTRUCTURE ONLY: the
// "optimized CPU" baseline of SURVEY.md §8(d), timed by bench.py's
// cpu_baseline leg beside the allocation-heavy "port" (oracle_capi.cpp
// bench_game).  Never part of the product path.
//
// Same work as the reference's SyncTestSession + ex_game on the same inputs:
// per steady tick (current frame c > check_distance) every session runs
//   LoadGameState(c-cd), AdvanceFrame, [SaveGameState(f), AdvanceFrame] x (cd-1),
//   SaveGameState(c), AdvanceFrame
// (sync_test_session.rs:85-146, 178-203), with State::advance's arithmetic
// (ex_game.rs:259-321: glibc sinf/cosf, f32 sqrt and division, rem_euclid),
// fletcher16 over the bincode image on every save (ex_game.rs:42-52, 88-93),
// the first-seen checksum history compare (sync_test_session.rs:159-176), and
// Game::last_checksum once per tick (ex_game.rs:104-108; the reference
// computes it after every AdvanceFrame, but only the last of a tick is
// observable).  What makes it "optimized" rather than a port:
//   * no allocation per request: states are plain floats in a per-session
//     snapshot ring [W][5P] (the request stream is executed inline, no
//     Vec<GGRSRequest>, no cloned heap State, no mutex cells, no HashMap);
//   * fletcher16 in closed form (s1 = sum b, s2 = sum (n-i) b, mod 255 once)
//     with the image's constant bytes folded in;
//   * sessions are processed in blocks that stay in L1/L2 for all the ticks of
//     the timed region (tick-major inside a block: the CPU analogue of the GPU's
//     fused launch, where a wave keeps its sessions for all ticks);
//   * all host threads the job may use, one contiguous session range each.
// Each tick's inputs are read from the pre-generated [T][P][S] array (the
// InputQueue holds exactly these: SyncTest inputs are always confirmed, and
// frame f's input is the one added at tick f - delay; blank before `delay`).
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

extern "C" void orc_synth_inputs(uint64_t seed, uint32_t mask, int32_t S, int32_t P, int32_t T, int32_t f0,
                                 int32_t input_bytes, void* out);

namespace {

constexpr float kFriction = 0.98f;
constexpr float kPi = 3.14159265358979323846264338327950288f;
const float kMovementSpeed = 15.0f / 60.0f;
const float kRotationSpeed = 2.5f / 60.0f;
constexpr float kMaxSpeed = 7.0f;
constexpr float kWidth = 600.0f, kHeight = 800.0f;

inline float rem_euclid(float x, float rhs) {
  const float r = std::fmod(x, rhs);
  return r < 0.0f ? r + std::fabs(rhs) : r;
}

// ex_game.rs:259-321 for one player; st = {x, y, vx, vy, rot}
inline void advance_player(float* st, uint8_t input) {
  float vx = st[2] * kFriction, vy = st[3] * kFriction, rot = st[4];
  const bool up = input & 1, down = input & 2, left = input & 4, right = input & 8;
  if (up != down) {
    const float c = cosf(rot), s = sinf(rot);
    if (up) {
      vx += kMovementSpeed * c;
      vy += kMovementSpeed * s;
    } else {
      vx -= kMovementSpeed * c;
      vy -= kMovementSpeed * s;
    }
  }
  if (left && !right) rot = rem_euclid(rot - kRotationSpeed, 2.0f * kPi);
  if (!left && right) rot = rem_euclid(rot + kRotationSpeed, 2.0f * kPi);
  const float mag = std::sqrt(vx * vx + vy * vy);
  if (mag > kMaxSpeed) {
    vx = (vx * kMaxSpeed) / mag;
    vy = (vy * kMaxSpeed) / mag;
  }
  float x = st[0] + vx, y = st[1] + vy;
  x = std::fmin(std::fmax(x, 0.0f), kWidth);
  y = std::fmin(std::fmax(y, 0.0f), kHeight);
  st[0] = x;
  st[1] = y;
  st[2] = vx;
  st[3] = vy;
  st[4] = rot;
}

// fletcher16 of the bincode image (frame i32 | P u64 | len u64 | pos 8P | len | vel 8P | len | rot 4P)
// in closed form; state words in session order {x, y, vx, vy, rot} per player.
struct Fletcher {
  int P, n;
  uint32_t c1, c2;  // the constant bytes (num_players and the three lengths: u64 = P)
  int off[4][5];    // image offset of each state word
  explicit Fletcher(int players) : P(players), n(36 + 20 * players) {
    const int offs[4] = {4, 12, 20 + 8 * P, 28 + 16 * P};
    c1 = c2 = 0;
    for (int o : offs) {
      c1 += static_cast<uint32_t>(P);
      c2 += static_cast<uint32_t>(P) * static_cast<uint32_t>(n - o);
    }
    for (int i = 0; i < P; ++i) {
      off[i][0] = 20 + 8 * i;
      off[i][1] = 24 + 8 * i;
      off[i][2] = 28 + 8 * P + 8 * i;
      off[i][3] = 32 + 8 * P + 8 * i;
      off[i][4] = 36 + 16 * P + 4 * i;
    }
  }
  static void word(uint32_t w, int o, int n, uint32_t& s1, uint32_t& s2) {
    for (int b = 0; b < 4; ++b) {
      const uint32_t v = (w >> (8 * b)) & 0xffu;
      s1 += v;
      s2 += v * static_cast<uint32_t>(n - o - b);
    }
  }
  uint16_t operator()(const float* st, int32_t frame) const {
    uint32_t s1 = c1, s2 = c2;
    word(static_cast<uint32_t>(frame), 0, n, s1, s2);
    for (int i = 0; i < P; ++i)
      for (int k = 0; k < 5; ++k) {
        uint32_t w;
        std::memcpy(&w, &st[5 * i + k], 4);
        word(w, off[i][k], n, s1, s2);
      }
    return static_cast<uint16_t>(((s2 % 255u) << 8) | (s1 % 255u));
  }
};

struct Block {
  int P, W, cd, delay, S, s0, s1;  // sessions [s0, s1) of an [T][P][S] input array
  const uint8_t* in;
  Fletcher fl;
  std::vector<float> live, snap;  // [ns][5P], [ns][W][5P]
  std::vector<uint16_t> cs, fs;   // [ns][W]
  std::vector<uint16_t> display;  // [ns] Game::last_checksum
  std::vector<int32_t> err;       // [ns] MismatchedChecksum frame, -1 healthy
  Block(int P_, int W_, int cd_, int delay_, int S_, int a, int b, const uint8_t* in_)
      : P(P_), W(W_), cd(cd_), delay(delay_), S(S_), s0(a), s1(b), in(in_), fl(P_) {
    const int ns = s1 - s0, nw = 5 * P;
    live.assign(static_cast<size_t>(ns) * nw, 0.0f);
    snap.assign(static_cast<size_t>(ns) * W * nw, 0.0f);
    cs.assign(static_cast<size_t>(ns) * W, 0);
    fs.assign(static_cast<size_t>(ns) * W, 0);
    display.assign(ns, 0);
    err.assign(ns, -1);
    const float r = kWidth / 4.0f;  // State::new (ex_game.rs:234-257)
    for (int s = 0; s < ns; ++s)
      for (int i = 0; i < P; ++i) {
        volatile float fi = static_cast<float>(i), fp = static_cast<float>(P);
        const float rot = fi / fp * 2.0f * kPi;
        float* st = &live[static_cast<size_t>(s) * nw + 5 * i];
        st[0] = kWidth / 2.0f + r * std::cos(rot);
        st[1] = kHeight / 2.0f + r * std::sin(rot);
        st[4] = std::fmod(rot + kPi, 2.0f * kPi);
      }
  }
  uint8_t input(int32_t frame, int p, int s) const {  // InputQueue::input of a confirmed frame
    const int32_t t = frame - delay;
    return t < 0 ? 0 : in[(static_cast<size_t>(t) * P + p) * S + s];
  }
  void advance(float* st, int32_t frame, int s) const {
    for (int i = 0; i < P; ++i) advance_player(st + 5 * i, input(frame, i, s));
  }
  // One tick of session j (global session s0 + j) at current frame c.
  void tick(int j, int32_t c) {
    if (err[j] >= 0) return;  // advance_frame keeps returning Err
    const int nw = 5 * P, s = s0 + j;
    float st[20];
    float* sn = &snap[static_cast<size_t>(j) * W * nw];
    uint16_t* csj = &cs[static_cast<size_t>(j) * W];
    uint16_t* fsj = &fs[static_cast<size_t>(j) * W];
    int32_t f0 = c;
    if (cd > 0 && c > cd) {
      f0 = c - cd;  // LoadGameState(c - cd)
      std::memcpy(st, sn + (f0 % W) * nw, sizeof(float) * nw);
    } else {
      std::memcpy(st, &live[static_cast<size_t>(j) * nw], sizeof(float) * nw);
    }
    int32_t mismatch = -1;
    for (int32_t f = f0; f <= c; ++f) {
      if (cd > 0 && (f > f0 || f0 == c)) {  // SaveGameState(f)
        const uint16_t v = fl(st, f);
        std::memcpy(sn + (f % W) * nw, st, sizeof(float) * nw);
        csj[f % W] = v;
        if (f == c) fsj[f % W] = v;  // first save of frame c: first-seen
        else if (v != fsj[f % W]) mismatch = f;
      }
      advance(st, f, s);
    }
    display[j] = fl(st, c + 1);
    std::memcpy(&live[static_cast<size_t>(j) * nw], st, sizeof(float) * nw);
    if (mismatch >= 0) err[j] = mismatch;
  }
  void run(int32_t c0, int32_t c1) {  // ticks c0 .. c1-1, tick-major over sub-blocks of sessions
    constexpr int kSub = 256;
    for (int a = 0; a < s1 - s0; a += kSub) {
      const int b = a + kSub < s1 - s0 ? a + kSub : s1 - s0;
      for (int32_t c = c0; c < c1; ++c)
        for (int j = a; j < b; ++j) tick(j, c);
    }
  }
};

double soa_run(int32_t P, int32_t cd, int32_t delay, int32_t W, int32_t S, int32_t warmup, int32_t ticks,
               int32_t threads, const uint8_t* in, float* states_out, uint16_t* cs_out, int32_t* n_err) {
  if (threads < 1) threads = 1;
  std::vector<Block> blocks;
  blocks.reserve(threads);
  for (int t = 0; t < threads; ++t)
    blocks.emplace_back(P, W, cd, delay, S, static_cast<int>(static_cast<int64_t>(S) * t / threads),
                        static_cast<int>(static_cast<int64_t>(S) * (t + 1) / threads), in);
  auto parallel = [&](auto fn) {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back([&, t] { fn(blocks[t]); });
    for (auto& x : th) x.join();
  };
  parallel([&](Block& b) { b.run(0, warmup); });
  const auto t0 = std::chrono::steady_clock::now();
  parallel([&](Block& b) { b.run(warmup, warmup + ticks); });
  const auto t1 = std::chrono::steady_clock::now();
  int32_t e = 0;
  for (auto& b : blocks) {
    for (int j = 0; j < b.s1 - b.s0; ++j) {
      e += b.err[j] >= 0;
      if (states_out)
        std::memcpy(states_out + static_cast<size_t>(b.s0 + j) * 5 * P, &b.live[static_cast<size_t>(j) * 5 * P],
                    sizeof(float) * 5 * P);
      if (cs_out) cs_out[b.s0 + j] = b.display[j];
    }
  }
  if (n_err) *n_err = e;
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // namespace

extern "C" {

// The optimized CPU baseline (bench.py cpu_baseline, kind "optimized"): the
// same synthetic inputs as orc_bench_exgame.  Returns wall seconds of the
// `ticks` timed ticks after `warmup` untimed ones (warmup must cover the
// check_distance + 1 start-up ticks).
double orc_bench_exgame_soa(int32_t num_players, int32_t check_distance, int32_t input_delay, int32_t max_prediction,
                            int32_t S, int32_t warmup, int32_t ticks, int32_t threads, uint64_t seed, int32_t* n_err) {
  if (num_players < 1 || num_players > 4 || check_distance >= max_prediction) return -1.0;
  const int32_t P = num_players, T = warmup + ticks;
  std::vector<uint8_t> in(static_cast<size_t>(T) * P * S);
  orc_synth_inputs(seed, 0x0F, S, P, T, 0, 1, in.data());
  return soa_run(P, check_distance, input_delay, max_prediction, S, warmup, ticks, threads, in.data(), nullptr,
                 nullptr, n_err);
}

// Parity hook for tests/test_oracle.py: T ticks from frame 0 on caller inputs
// [T][P][S]; writes the live states [S][5P] (x, y, vx, vy, rot per player) and
// Game::last_checksum [S] after the last tick.
int32_t orc_soa_exgame_run(int32_t P, int32_t cd, int32_t delay, int32_t W, int32_t S, int32_t T, int32_t threads,
                           const uint8_t* in, float* states_out, uint16_t* display_out) {
  int32_t e = 0;
  soa_run(P, cd, delay, W, S, T, 0, threads, in, states_out, display_out, &e);
  return e;
}

}  // extern "C"
