// ggrs_amd/csrc/engine.hip — MI355X batched rollback-resimulation engine: host side
// (rb_batch, the C ABI of include/ggrs_amd.h).  Kernels: kernels.hpp, instantiated
// per game in ops_exgame.hip / ops_exgame_lps.hip / ops_brawler.hip / ops_stub.hip.
//
//
// One rb_batch = S independent SyncTestSessions in lock-step.  Per tick the
// host mirror (planner.hpp) produces the reference's request stream and lowers
// it to a TickProgram; ONE kernel launch then executes that stream for every
// session: lane s owns session s, its state stays in VGPRs from the
// LoadGameState through every SaveGameState/AdvanceFrame of the tick, and
// HBM sees each snapshot written once (coalesced SoA planes) and the loaded
// slot read once.
//
// Device layout (Spad = S rounded up to 64; all planes contiguous over sessions):
//   snap  [W slots][NW words as planes of u32x4 / u32x2 / u32][Spad]   snapshot ring, slot = frame % W
//   cs    [W][Spad] CS        checksum stored by each SaveGameState (GameStateCell::checksum)
//   fs    [W][Spad] CS        first-seen checksum of the frame (SyncTestSession::checksum_history)
//   ring  [128][Spad] InRec   confirmed inputs, slot = frame % 128 (InputQueue::inputs)
//   live  [NW planes][Spad]   live game state between ticks when no LoadGameState follows
//   err   [Spad] i32          MismatchedChecksum{frame}, NULL_FRAME when healthy
//   frozen[Spad/64] u64       sessions whose advance_frame returns Err (they no longer advance)
#include <algorithm>
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <dlfcn.h>

#include "kernels.hpp"
#include "../../include/ggrs_amd_game.hpp"

// ---- game plugins (rb_register_game_plugin): dlopen'ed libraries built from
// plugin.hip, each creating the GameOps of one user game.  Entries live for the
// process (a batch may hold the plugin's GameOps and kernels).
namespace rb {
namespace {
struct Plugin {
  std::string path;
  void* handle;
  GameOps* (*make)(int32_t, int32_t);
};
std::mutex g_plugins_mu;
std::vector<Plugin> g_plugins;
}  // namespace

std::unique_ptr<GameOps> make_plugin_ops(int game, int players) {
  std::lock_guard<std::mutex> lk(g_plugins_mu);
  const int k = game - RB_GAME_PLUGIN_BASE;
  if (k < 0 || k >= static_cast<int>(g_plugins.size())) return nullptr;
  return std::unique_ptr<GameOps>(g_plugins[static_cast<size_t>(k)].make(players, RB_PLUGIN_ABI));
}
}  // namespace rb

namespace rb {
__global__ void sincos_kernel(const float* __restrict__ x, float* __restrict__ so, float* __restrict__ co, int64_t n,
                              uint32_t* unexpected) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const SinCos r = sincosf_glibc(x[i], unexpected);
  so[i] = r.s;
  co[i] = r.c;
}

// The in-range forms the fused steady ticks and the fan-out run (ExGame::prepare / advance<true>):
// for the floats with bits first + i, out[0][i] / out[1][i] = sincosf_glibc<true> (sin, cos),
// out[2..3][i] = rem_euclid_near<true>(x +- ROTATION_SPEED, 2 pi), out[4..5][i] =
// rem_euclid<true>(x +- ROTATION_SPEED, 2 pi) (rb_debug_exgame_inrange).
__global__ void inrange_kernel(uint32_t first, int64_t n, float* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  using E = ExGame<2, true>;
  const float x = __uint_as_float(first + static_cast<uint32_t>(i));
  const SinCos r = sincosf_glibc<true>(x, nullptr);
  out[i] = r.s;
  out[n + i] = r.c;
  out[2 * n + i] = rem_euclid_near<true>(x + E::kRotationSpeed, 2.0f * E::kPi);
  out[3 * n + i] = rem_euclid_near<true>(x + -E::kRotationSpeed, 2.0f * E::kPi);
  out[4 * n + i] = rem_euclid<true>(x + E::kRotationSpeed, 2.0f * E::kPi);
  out[5 * n + i] = rem_euclid<true>(x - E::kRotationSpeed, 2.0f * E::kPi);
}

__global__ void clamp_kernel(const float* __restrict__ vx, const float* __restrict__ vy, float* __restrict__ ox,
                             float* __restrict__ oy, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = vx[i], b = vy[i];
  ExGame<1, false>::speed_clamp(a, b);
  ox[i] = a;
  oy[i] = b;
}

}  // namespace rb

using namespace rb;

struct rb_batch {
  rb_config cfg{};
  std::unique_ptr<GameOps> ops;
  std::unique_ptr<SyncTestPlan> plan;
  int S = 0, Spad = 0, W = 0, P = 0, block = 256;
  bool plan_only = false;
  // the fused kernel's 32-bit ring offsets (kernels.hpp steady_saddr): rings of at least this many
  // bytes run per-tick launches.  4 GiB; RB_STEADY_RING_LIMIT lowers it (the fallback's parity test)
  size_t ring_limit = size_t{1} << 32;
  int device = 0;
  hipStream_t own_stream = nullptr, stream = nullptr;
  // device buffers
  uint32_t* snap = nullptr;
  uint32_t* live = nullptr;
  void* cs = nullptr;
  void* fs = nullptr;
  void* ring = nullptr;
  void* last_cs = nullptr;
  void* periodic_cs = nullptr;
  int32_t* err = nullptr;
  int32_t* live_frame = nullptr;
  unsigned long long* frozen = nullptr;
  uint32_t* counters = nullptr;
  // input staging for host pointers: [2][P][S*input_bytes]
  uint8_t* stage_dev = nullptr;
  uint8_t* stage_host = nullptr;
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  int stage_parity = 0;
  const void* in_ptr[4] = {nullptr, nullptr, nullptr, nullptr};
  int in_mode = 0;
  // checked mode
  // checked mode: a word of pinned, device-mapped host memory the kernels set to 1 when a session
  // fails (MismatchedChecksum), read after the call's stream wait; no copy packet per call
  volatile uint32_t* pinned_counters = nullptr;
  uint32_t* fail_flag_dev = nullptr;  // the device's address of pinned_counters[0]
  hipEvent_t tick_ev = nullptr;
  bool tick_pending = false;
  // live-state validity and bookkeeping
  bool live_valid = true;
  int32_t display_frame = kNullFrame;
  uint32_t tick = 0;
  // profiling
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev;  // pool, reused after rb_profile_take
  std::vector<int32_t> prof_ticks;                          // ticks covered by each timed launch
  size_t prof_used = 0;
  uint32_t prof_every = 8, prof_tick = 0;
  bool staged = false;  // this tick's inputs went through the host staging buffer
  std::string last_err;
  // Set when the device state and the host plan can no longer agree (an early
  // fused launch ran ticks whose host bookkeeping then failed): every later
  // call fails with RB_PANIC, as the reference process would have stopped.
  std::string poisoned;
  bool pipe = false;  // fused steady ticks with two ticks in flight (RB_STEADY_PIPE=1 at create; A/B, tests)
  uint32_t simds = 1024;  // SIMDs of the device (MI355X: 256 CUs x 4)
  uint32_t lds_pad = 0;  // RB_LDS_PAD (bytes) at create: dynamic LDS reserved per steady workgroup (A/B)
  LaunchClock clock;  // rb_launch_clock_arm
};

namespace {
thread_local std::string g_create_err;
constexpr size_t kProfPool = 256;  // HIP event pairs created by rb_profile_enable

rb_status fail(rb_batch* b, rb_status st, const std::string& msg) {
  if (b) b->last_err = msg; else g_create_err = msg;
  return st;
}
#define HIP_TRY(b, expr)                                                                          \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) return fail((b), RB_DEVICE_ERROR, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

rb_status destroy_device(rb_batch* b) {
  if (b->plan_only) return RB_OK;
  (void)hipSetDevice(b->device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  void* ptrs[] = {b->snap, b->live, b->cs, b->fs, b->ring, b->last_cs, b->periodic_cs, b->err, b->live_frame,
                  b->frozen, b->counters, b->stage_dev};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (b->stage_host) (void)hipHostFree(b->stage_host);
  if (b->pinned_counters) (void)hipHostFree(const_cast<uint32_t*>(b->pinned_counters));
  for (auto& e : b->stage_ev)
    if (e) (void)hipEventDestroy(e);
  if (b->tick_ev) (void)hipEventDestroy(b->tick_ev);
  for (auto& pr : b->prof_ev) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  b->clock.release();
  if (b->own_stream) (void)hipStreamDestroy(b->own_stream);
  return RB_OK;
}

rb_status launch_program(rb_batch* b, const TickProgram& tp, bool ingest, bool display, int32_t periodic_step) {
  KParams p{};
  p.snap = b->snap;
  p.live = b->live;
  p.cs = b->cs;
  p.fs = b->fs;
  p.ring = b->ring;
  p.last_cs = b->last_cs;
  p.periodic_cs = b->periodic_cs;
  p.err = b->err;
  p.live_frame = b->live_frame;
  p.frozen = b->frozen;
  p.counters = b->counters;
  p.fail_flag = b->fail_flag_dev;
  p.S = b->S;
  p.Spad = b->Spad;
  p.W = b->W;
  for (int i = 0; i < 4; ++i) p.in_ptr[i] = b->ring;  // valid dummies: the kernel always loads
  p.repl_src = 0;
  if (ingest) {
    p.in_mode = b->in_mode;
    for (int i = 0; i < 4; ++i)
      if (b->in_ptr[i]) p.in_ptr[i] = b->in_ptr[i];
    p.user_slot = tp.user_slot;
    p.n_repl = static_cast<int32_t>(tp.repl_dst.size());
    if (p.n_repl > kMaxRepl) return fail(b, RB_INVALID_REQUEST, "input delay above 8 is not supported by the device batch");
    for (int i = 0; i < p.n_repl; ++i) p.repl_dst[i] = tp.repl_dst[i];
    if (p.n_repl > 0) p.repl_src = tp.repl_src;
  } else {
    p.in_mode = 0;
    p.user_slot = -1;
  }
  p.load_slot = tp.load ? tp.load_frame % b->W : -1;
  p.f0 = tp.f0;
  p.n_steps = tp.n_steps;
  p.slot0 = tp.f0 % b->W;
  if (tp.n_steps > 2 * b->W) return fail(b, RB_PANIC, "tick program longer than two snapshot rings");
  for (int k = 0; k < tp.n_steps; ++k) {
    p.save_modes[k >> 4] |= static_cast<uint32_t>(tp.save_mode[k] & 3u) << ((k & 15) * 2);
  }
  p.live_out = tp.live_out ? 1 : 0;
  p.periodic_step = periodic_step;
  p.display = display ? 1 : 0;
  p.disc_mask = 0;
  p.seed = b->cfg.seed;
  p.nonce_base = (b->tick & 0xffffffu) << 8;
  p.debug = b->cfg.reserved[0];
  const bool timed = b->prof && (b->prof_tick++ % b->prof_every) == 0;  // sampled: an event pair costs host time
  LaunchEv ev;  // the kernel's own start / end (hipExtLaunchKernel), no marker packets around it
  if (timed) {
    if (b->prof_used == b->prof_ev.size()) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      HIP_TRY(b, hipEventCreate(&e0));
      HIP_TRY(b, hipEventCreate(&e1));
      b->prof_ev.push_back({e0, e1});
    }
    ev = LaunchEv{b->prof_ev[b->prof_used].first, b->prof_ev[b->prof_used].second};
  }
  HIP_TRY(b, b->ops->launch_tick(p, b->block, b->stream, ev));
  if (timed) {
    b->prof_ticks.resize(b->prof_ev.size());
    b->prof_ticks[b->prof_used] = 1;
    b->prof_used += 1;
  }
  return RB_OK;
}

rb_status read_words_slot(rb_batch* b, const uint32_t* dev_base, std::vector<uint32_t>& host) {
  host.resize(static_cast<size_t>(b->ops->nw) * b->Spad * b->ops->lanes);
  HIP_TRY(b, hipMemcpyAsync(host.data(), dev_base, host.size() * 4, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(b, hipStreamSynchronize(b->stream));
  return RB_OK;
}

// words [lanes][nw] of session s from a block of lane planes
void words_of(const rb_batch* b, const std::vector<uint32_t>& planes, int s, uint32_t* w) {
  const int L = b->ops->lanes, NW = b->ops->nw;
  for (int l = 0; l < L; ++l)
    for (int k = 0; k < NW; ++k) w[l * NW + k] = planes[word_index(NW, b->Spad * L, s * L + l, k)];
}

}  // namespace

extern "C" {

rb_status rb_register_game_plugin(const char* path, int32_t* game_id) {
  if (!path || !game_id) return fail(nullptr, RB_INVALID_REQUEST, "rb_register_game_plugin: null argument");
  std::lock_guard<std::mutex> lk(g_plugins_mu);
  for (size_t k = 0; k < g_plugins.size(); ++k)
    if (g_plugins[k].path == path) {
      *game_id = RB_GAME_PLUGIN_BASE + static_cast<int32_t>(k);
      return RB_OK;
    }
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(nullptr, RB_INVALID_REQUEST, std::string("cannot load game plugin: ") + dlerror());
  auto abi = reinterpret_cast<int32_t (*)()>(dlsym(h, "rb_plugin_abi"));
  auto make = reinterpret_cast<GameOps* (*)(int32_t, int32_t)>(dlsym(h, "rb_plugin_make_ops"));
  if (!abi || !make || abi() != RB_PLUGIN_ABI) {
    dlclose(h);
    return fail(nullptr, RB_INVALID_REQUEST, "not a game plugin of this engine (rb_plugin_abi / rb_plugin_make_ops)");
  }
  g_plugins.push_back(Plugin{path, h, make});
  *game_id = RB_GAME_PLUGIN_BASE + static_cast<int32_t>(g_plugins.size() - 1);
  return RB_OK;
}

void rb_config_init(rb_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->abi_version = RB_ABI_VERSION;
  c->game = RB_GAME_EX_GAME;
  c->num_sessions = 1;
  c->num_players = 2;     // builder.rs:13
  c->max_prediction = 8;  // builder.rs:20
  c->check_distance = 2;  // builder.rs:21
  c->input_delay = 0;     // builder.rs:16
  c->device = 0;
  c->flags = RB_FLAG_CHECKED;
}

const char* rb_last_error(const rb_batch* b) { return b ? b->last_err.c_str() : g_create_err.c_str(); }

rb_status rb_synctest_create(const rb_config* cfg, rb_batch** out) {
  *out = nullptr;
  if (!cfg || cfg->abi_version != RB_ABI_VERSION) return fail(nullptr, RB_INVALID_REQUEST, "rb_config.abi_version mismatch");
  // builder.rs:136-145
  if (cfg->max_prediction <= 0)
    return fail(nullptr, RB_INVALID_REQUEST, "Currently, only prediction windows above 0 are supported");
  if (cfg->check_distance < 0 || cfg->input_delay < 0 || cfg->num_players <= 0 || cfg->num_sessions <= 0)
    return fail(nullptr, RB_INVALID_REQUEST, "negative or zero size in rb_config");
  // builder.rs:342-347
  if (cfg->check_distance >= cfg->max_prediction) return fail(nullptr, RB_INVALID_REQUEST, "Check distance too big.");
  if (cfg->max_prediction > kMaxSteps)
    return fail(nullptr, RB_INVALID_REQUEST, "max_prediction above 64 is not supported by the device batch");
  if (cfg->input_delay > kQueueLen - cfg->max_prediction - 2)
    return fail(nullptr, RB_INVALID_REQUEST, "input delay does not fit the 128-entry input queue");
  auto ops = make_game(cfg->game, cfg->num_players, (cfg->flags & RB_FLAG_LANE_PER_SESSION) != 0);
  if (!ops) return fail(nullptr, RB_INVALID_REQUEST, "unsupported game / num_players combination (RB_FLAG_LANE_PER_SESSION: A/B builds only)");
  // every snapshot word offset (slot * NW * lanes * Spad + ...) is 32-bit inside the kernels
  if (static_cast<uint64_t>(cfg->max_prediction) * ops->nw * ops->lanes *
          ((static_cast<uint64_t>(cfg->num_sessions) + 63) / 64 * 64) >= (1ull << 32))
    return fail(nullptr, RB_INVALID_REQUEST, "batch too large for 32-bit snapshot offsets");

  auto b = std::make_unique<rb_batch>();
  b->cfg = *cfg;
  b->ops = std::move(ops);
  b->plan = std::make_unique<SyncTestPlan>(cfg->num_players, cfg->max_prediction, cfg->check_distance, cfg->input_delay);
  b->S = cfg->num_sessions;
  b->Spad = (cfg->num_sessions + 63) / 64 * 64;
  b->W = cfg->max_prediction;
  b->P = cfg->num_players;
  b->block = cfg->block_size ? static_cast<int>(cfg->block_size) : 256;
#if RB_EXPERIMENTS  // (A/B builds only: the knob measured no effect, round 4)
  if (const char* env = std::getenv("RB_LDS_PAD")) b->lds_pad = static_cast<uint32_t>(std::clamp(std::atoi(env), 0, 64 * 1024));
#endif
#if RB_EXPERIMENTS  // steady_pipe_kernel exists in A/B builds only
  if (const char* env = std::getenv("RB_STEADY_PIPE")) b->pipe = std::atoi(env) != 0;
#endif
  if (const char* env = std::getenv("RB_STEADY_RING_LIMIT"))
    b->ring_limit = std::min(b->ring_limit, static_cast<size_t>(std::strtoull(env, nullptr, 10)));
  if (b->block % 64 != 0 || b->block > 256) return fail(nullptr, RB_INVALID_REQUEST, "block_size must be 64, 128, 192 or 256");
  b->plan_only = cfg->device < 0;
  b->device = cfg->device;
  if (b->plan_only) {
    *out = b.release();
    return RB_OK;
  }
  rb_batch* bp = b.get();
  auto hip_fail = [&](hipError_t e, const char* what) {
    g_create_err = std::string(what) + ": " + hipGetErrorString(e);
    destroy_device(bp);
    return RB_DEVICE_ERROR;
  };
#define HIP_CREATE(expr)                          \
  do {                                            \
    hipError_t _e = (expr);                       \
    if (_e != hipSuccess) return hip_fail(_e, #expr); \
  } while (0)
  HIP_CREATE(hipSetDevice(b->device));
  int cus = 0;
  HIP_CREATE(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, b->device));
  b->simds = 4 * cus;  // 4 SIMDs per CU (CDNA)
  HIP_CREATE(hipStreamCreateWithFlags(&b->own_stream, hipStreamNonBlocking));
  b->stream = b->own_stream;
  const size_t Sp = b->Spad, NW = b->ops->nw, W = b->W, L = b->ops->lanes, Gp = Sp * L;
  HIP_CREATE(hipMalloc(&b->snap, W * NW * Gp * 4));
  HIP_CREATE(hipMalloc(&b->live, NW * Gp * 4));
  HIP_CREATE(hipMalloc(&b->cs, W * Sp * b->ops->cs_bytes));
  HIP_CREATE(hipMalloc(&b->fs, W * Sp * b->ops->cs_bytes));
  HIP_CREATE(hipMalloc(&b->ring, kQueueLen * Sp * b->ops->inrec_bytes));
  HIP_CREATE(hipMalloc(&b->last_cs, Sp * b->ops->cs_bytes));
  HIP_CREATE(hipMalloc(&b->periodic_cs, Sp * b->ops->cs_bytes));
  HIP_CREATE(hipMalloc(&b->err, Sp * 4));
  HIP_CREATE(hipMalloc(&b->live_frame, Sp * 4));
  HIP_CREATE(hipMalloc(&b->frozen, Sp / 64 * 8));
  HIP_CREATE(hipMalloc(&b->counters, 16));
  const size_t stage = 2ull * b->P * Sp * b->ops->input_bytes;
  HIP_CREATE(hipMalloc(&b->stage_dev, stage));
  HIP_CREATE(hipHostMalloc(&b->stage_host, stage));
  {
    void* pc = nullptr;
    HIP_CREATE(hipHostMalloc(&pc, 16, hipHostMallocMapped | hipHostMallocCoherent));
    b->pinned_counters = static_cast<volatile uint32_t*>(pc);
    b->pinned_counters[0] = 0;
    void* dp = nullptr;
    HIP_CREATE(hipHostGetDevicePointer(&dp, pc, 0));
    b->fail_flag_dev = static_cast<uint32_t*>(dp);
  }
  HIP_CREATE(hipEventCreateWithFlags(&b->stage_ev[0], hipEventDisableTiming));
  HIP_CREATE(hipEventCreateWithFlags(&b->stage_ev[1], hipEventDisableTiming));
  HIP_CREATE(hipEventCreateWithFlags(&b->tick_ev, hipEventDisableTiming));
  HIP_CREATE(hipMemsetAsync(b->snap, 0, W * NW * Gp * 4, b->stream));
  HIP_CREATE(hipMemsetAsync(b->cs, 0, W * Sp * b->ops->cs_bytes, b->stream));
  HIP_CREATE(hipMemsetAsync(b->fs, 0, W * Sp * b->ops->cs_bytes, b->stream));
  HIP_CREATE(hipMemsetAsync(b->ring, 0, kQueueLen * Sp * b->ops->inrec_bytes, b->stream));  // blank inputs
  HIP_CREATE(hipMemsetAsync(b->last_cs, 0, Sp * b->ops->cs_bytes, b->stream));
  HIP_CREATE(hipMemsetAsync(b->periodic_cs, 0, Sp * b->ops->cs_bytes, b->stream));
  HIP_CREATE(hipMemsetAsync(b->err, 0xff, Sp * 4, b->stream));  // NULL_FRAME
  HIP_CREATE(hipMemsetAsync(b->live_frame, 0xff, Sp * 4, b->stream));
  HIP_CREATE(hipMemsetAsync(b->frozen, 0, Sp / 64 * 8, b->stream));
  HIP_CREATE(hipMemsetAsync(b->counters, 0, 16, b->stream));
  // State::new for every session (ex_game.rs:234-257), host-evaluated once.
  std::vector<uint32_t> w0(L * NW), planes(NW * Gp);
  b->ops->init_words(w0.data());
  for (size_t s = 0; s < Sp; ++s)
    for (size_t l = 0; l < L; ++l)
      for (size_t k = 0; k < NW; ++k)
        planes[word_index(static_cast<int>(NW), static_cast<int>(Gp), static_cast<int>(s * L + l), static_cast<int>(k))] =
            w0[l * NW + k];
  HIP_CREATE(hipMemcpyAsync(b->live, planes.data(), planes.size() * 4, hipMemcpyHostToDevice, b->stream));
  HIP_CREATE(hipStreamSynchronize(b->stream));
#undef HIP_CREATE
  *out = b.release();
  return RB_OK;
}

void rb_destroy(rb_batch* b) {
  if (!b) return;
  destroy_device(b);
  delete b;
}

rb_status rb_set_stream(rb_batch* b, void* s) {
  if (b->plan_only) return RB_OK;
  HIP_TRY(b, hipStreamSynchronize(b->stream));
  b->stream = s ? static_cast<hipStream_t>(s) : b->own_stream;
  return RB_OK;
}

void* rb_get_stream(const rb_batch* b) { return b->plan_only ? nullptr : static_cast<void*>(b->stream); }

int32_t rb_current_frame(const rb_batch* b) { return b->plan->current; }
int32_t rb_num_sessions(const rb_batch* b) { return b->S; }
int32_t rb_state_bytes(const rb_batch* b) { return b->ops->image_bytes; }
int32_t rb_input_bytes(const rb_batch* b) { return b->ops->input_bytes; }

rb_status rb_add_local_input(rb_batch* b, int32_t handle, const void* inputs, int32_t on_device) {
  // sync_test_session.rs:66-70
  if (!b->plan->add_local_input(handle))
    return fail(b, RB_INVALID_REQUEST, "The player handle you provided is not valid.");
  if (b->plan_only) return RB_OK;
  if (handle >= 4) return fail(b, RB_INVALID_REQUEST, "at most 4 players per session");
  if (b->in_mode == 2) {  // switching from packed: every handle must be given again
    for (auto& q : b->in_ptr) q = nullptr;
  }
  b->in_mode = 1;
  if (on_device) {
    b->in_ptr[handle] = inputs;
    return RB_OK;
  }
  const size_t bytes = static_cast<size_t>(b->S) * b->ops->input_bytes;
  const size_t off = (static_cast<size_t>(b->stage_parity) * b->P + handle) * b->Spad * b->ops->input_bytes;
  HIP_TRY(b, hipEventSynchronize(b->stage_ev[b->stage_parity]));  // previous copy out of this slot is done
  std::memcpy(b->stage_host + off, inputs, bytes);
  HIP_TRY(b, hipMemcpyAsync(b->stage_dev + off, b->stage_host + off, bytes, hipMemcpyHostToDevice, b->stream));
  b->in_ptr[handle] = b->stage_dev + off;
  b->staged = true;
  return RB_OK;
}

rb_status rb_add_local_inputs_packed(rb_batch* b, const void* inputs, int32_t on_device) {
  for (int h = 0; h < b->P; ++h) b->plan->add_local_input(h);
  if (b->plan_only) return RB_OK;
  b->in_mode = 2;
  if (on_device) {
    b->in_ptr[0] = inputs;
    return RB_OK;
  }
  const size_t bytes = static_cast<size_t>(b->S) * b->P * b->ops->input_bytes;
  const size_t off = static_cast<size_t>(b->stage_parity) * b->P * b->Spad * b->ops->input_bytes;
  HIP_TRY(b, hipEventSynchronize(b->stage_ev[b->stage_parity]));
  std::memcpy(b->stage_host + off, inputs, bytes);
  HIP_TRY(b, hipMemcpyAsync(b->stage_dev + off, b->stage_host + off, bytes, hipMemcpyHostToDevice, b->stream));
  b->in_ptr[0] = b->stage_dev + off;
  b->staged = true;
  return RB_OK;
}

rb_status rb_advance_frame(rb_batch* b) {
  if (!b->poisoned.empty()) return fail(b, RB_PANIC, b->poisoned);
  rb_status result = RB_OK;
  // Checked mode: sessions frozen by the previous tick fail this call
  // (sync_test_session.rs:91-98 returns MismatchedChecksum before any work).
  if (!b->plan_only && (b->cfg.flags & RB_FLAG_CHECKED) && b->tick_pending) {
    HIP_TRY(b, hipEventSynchronize(b->tick_ev));
    b->tick_pending = false;
    if (b->pinned_counters[0] > 0) result = RB_MISMATCHED_CHECKSUM;
  }
  TickProgram tp;
  std::string info;
  int rc;
  try {
    rc = b->plan->advance(tp, info);
  } catch (const Panic& e) {
    return fail(b, RB_PANIC, e.what());
  }
  if (rc == 2) return fail(b, RB_INVALID_REQUEST, info);
  if (rc == 1) return fail(b, RB_PREDICTION_THRESHOLD, "Prediction threshold is reached, cannot proceed without catching up.");
  if (b->plan_only) return result;
  if (b->in_mode == 1)
    for (int h = 0; h < b->P; ++h)
      if (!b->in_ptr[h]) return fail(b, RB_PANIC, "input pointer missing for a handle");
  // ex_game's periodic checksum: frame % CHECKSUM_PERIOD == 0 after an advance (ex_game.rs:109-111)
  int32_t periodic_step = -1;
  if (b->ops->display)
    for (int k = 0; k < tp.n_steps; ++k)
      if ((tp.f0 + k + 1) % 100 == 0) periodic_step = k;
  rb_status st = launch_program(b, tp, true, b->ops->display, periodic_step);
  if (st != RB_OK) return st;
  // the staging slot used by this tick may be refilled once this point passes
  if (b->staged) {
    HIP_TRY(b, hipEventRecord(b->stage_ev[b->stage_parity], b->stream));
    b->stage_parity ^= 1;
    b->staged = false;
  }
  b->in_mode = 0;
  for (auto& q : b->in_ptr) q = nullptr;
  b->live_valid = tp.live_out;
  b->display_frame = tp.f0 + tp.n_steps;
  b->tick += 1;
  if (b->cfg.flags & RB_FLAG_CHECKED) {
    HIP_TRY(b, hipEventRecord(b->tick_ev, b->stream));  // (the kernel sets pinned_counters[0] itself)
    b->tick_pending = true;
  }
  if (result != RB_OK) b->last_err = "Detected checksum mismatch during rollback (see rb_mismatches).";
  return result;
}

namespace {
bool is_steady_shape(const rb_batch* b, const TickProgram& tp) {
  const int cd = b->cfg.check_distance;
  if (cd < 1 || !tp.load || tp.load_frame != tp.f0 || tp.n_steps != cd + 1 || tp.live_out || !tp.repl_dst.empty())
    return false;
  if (tp.user_slot != ((tp.f0 + cd + b->cfg.input_delay) & (kQueueLen - 1))) return false;
  if (tp.save_mode[0] != SAVE_NONE || tp.save_mode[cd] != SAVE_RECORD) return false;
  for (int k = 1; k < cd; ++k)
    if (tp.save_mode[k] != SAVE_COMPARE) return false;
  return true;
}

// Launch `n` fused steady ticks whose first current frame is c0.
rb_status launch_steady_run(rb_batch* b, const uint8_t* tick_inputs, int64_t stride, int32_t c0, int32_t n,
                            uint32_t tick0) {
  RunParams r{};
  r.snap = b->snap;
  r.cs = b->cs;
  r.fs = b->fs;
  r.ring = b->ring;
  r.last_cs = b->last_cs;
  r.periodic_cs = b->periodic_cs;
  r.live = b->live;
  r.err = b->err;
  r.live_frame = b->live_frame;
  r.frozen = b->frozen;
  r.counters = b->counters;
  r.fail_flag = b->fail_flag_dev;
  r.in_base = tick_inputs;
  r.in_stride = stride;
  r.S = b->S;
  r.Spad = b->Spad;
  r.W = b->W;
  r.delay = b->cfg.input_delay;
  r.c0 = c0;
  r.T = n;
  r.tick0 = tick0;
  r.live_out_last = 0;
  r.seed = b->cfg.seed;
  r.debug = b->cfg.reserved[0];
  r.pipe = b->pipe ? 1 : 0;
  r.lds_pad = b->lds_pad;
  r.many_waves = static_cast<uint64_t>(b->Spad) * b->ops->lanes > 2ull * 64ull * b->simds ? 1u : 0u;
  r.launch_clock = b->clock.next();
  const bool timed = b->prof;
  LaunchEv ev;  // the kernel's own start / end (hipExtLaunchKernel), no marker packets around it
  if (timed) {
    if (b->prof_used == b->prof_ev.size()) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      HIP_TRY(b, hipEventCreate(&e0));
      HIP_TRY(b, hipEventCreate(&e1));
      b->prof_ev.push_back({e0, e1});
    }
    ev = LaunchEv{b->prof_ev[b->prof_used].first, b->prof_ev[b->prof_used].second};
  }
  hipError_t e = b->ops->launch_steady(r, b->cfg.check_distance, b->block, b->stream, ev);
  if (e != hipSuccess) return fail(b, RB_DEVICE_ERROR, std::string("steady_kernel: ") + hipGetErrorString(e));
  if (timed) {
    b->prof_ticks.resize(b->prof_ev.size());
    b->prof_ticks[b->prof_used] = n;
    b->prof_used += 1;
  }
  return RB_OK;
}
}  // namespace

rb_status rb_run_ticks(rb_batch* b, int32_t n_ticks, const void* inputs, int64_t tick_stride_bytes,
                       int32_t on_device, int32_t* ticks_done) {
  if (ticks_done) *ticks_done = 0;
  if (!b->poisoned.empty()) return fail(b, RB_PANIC, b->poisoned);
  if (n_ticks <= 0) return RB_OK;
  const size_t player_bytes = static_cast<size_t>(b->S) * b->ops->input_bytes;
  if (b->plan_only) {  // host bookkeeping only
    int32_t done = 0;
    rb_status st = RB_OK;
    for (; done < n_ticks && st == RB_OK; ++done) {
      for (int h = 0; h < b->P; ++h) b->plan->add_local_input(h);
      st = rb_advance_frame(b);
      if (st != RB_OK) break;
    }
    if (ticks_done) *ticks_done = done;
    return st;
  }
  // Host inputs: one upload of all ticks into a device buffer.
  const uint8_t* dev_in = static_cast<const uint8_t*>(inputs);
  int64_t stride = tick_stride_bytes;
  void* tmp = nullptr;
  if (!on_device) {
    const size_t tick_bytes = player_bytes * b->P;
    HIP_TRY(b, hipMallocAsync(&tmp, tick_bytes * n_ticks, b->stream));
    HIP_TRY(b, hipMemcpy2DAsync(tmp, tick_bytes, inputs, static_cast<size_t>(tick_stride_bytes), tick_bytes, n_ticks,
                                hipMemcpyHostToDevice, b->stream));
    dev_in = static_cast<const uint8_t*>(tmp);
    stride = static_cast<int64_t>(tick_bytes);
  }
  rb_status result = RB_OK;
  if ((b->cfg.flags & RB_FLAG_CHECKED) && b->tick_pending) {
    HIP_TRY(b, hipEventSynchronize(b->tick_ev));
    b->tick_pending = false;
  }
  const size_t ring_bytes = std::max(static_cast<size_t>(b->W) * b->ops->nw * b->Spad * b->ops->lanes * 4,
                                     static_cast<size_t>(b->W) * b->Spad * b->ops->cs_bytes);  // cells, checksums
  const bool can_fuse = b->ops->launch_steady_supported(b->cfg.check_distance, ring_bytes, b->ring_limit);
  int32_t run_start = -1, run_c0 = 0;
  uint32_t run_tick0 = 0;
  auto flush = [&](int32_t end) -> rb_status {
    if (run_start < 0) return RB_OK;
    rb_status st = launch_steady_run(b, dev_in + static_cast<int64_t>(run_start) * stride, stride, run_c0,
                                     end - run_start, run_tick0);
    run_start = -1;
    return st;
  };
  // Early launch.  Once past the start-up ticks (current frame > check
  // distance) every SyncTest tick has the steady shape: run_ticks supplies
  // every handle's input, PredictionThreshold cannot trigger (frames ahead =
  // check distance < max prediction) and nothing else in the bookkeeping
  // depends on values.  So the fused launch of all n ticks goes to the GPU
  // first and the host bookkeeping of those ticks runs while it executes;
  // each tick's lowered program is still checked against the steady shape.
  const int32_t cur0 = b->plan->current;
  const bool early = can_fuse && cur0 > b->cfg.check_distance;
  if (early) {
    rb_status st = launch_steady_run(b, dev_in, stride, cur0, n_ticks, b->tick);
    if (st != RB_OK) {
      if (tmp) (void)hipFreeAsync(tmp, b->stream);
      return st;
    }
  }
  int32_t done = 0;
  for (; done < n_ticks; ++done) {
    for (int h = 0; h < b->P; ++h) b->plan->add_local_input(h);
    TickProgram tp;
    std::string info;
    int rc;
    try {
      rc = b->plan->advance(tp, info);
    } catch (const Panic& e) {
      flush(done);
      result = fail(b, RB_PANIC, e.what());
      break;
    }
    if (rc != 0) {
      flush(done);
      result = rc == 2 ? fail(b, RB_INVALID_REQUEST, info) : fail(b, RB_PREDICTION_THRESHOLD, "Prediction threshold is reached, cannot proceed without catching up.");
      break;
    }
    if (early) {
      if (!is_steady_shape(b, tp) || tp.f0 + b->cfg.check_distance != cur0 + done) {
        result = fail(b, RB_PANIC, "internal: a tick after the start-up ticks did not have the steady shape");
        break;
      }
    } else if (can_fuse && is_steady_shape(b, tp)) {
      if (run_start < 0) {
        run_start = done;
        run_c0 = tp.f0 + b->cfg.check_distance;
        run_tick0 = b->tick;
      }
    } else {
      rb_status st = flush(done);
      if (st != RB_OK) { result = st; break; }
      const uint8_t* t = dev_in + static_cast<int64_t>(done) * stride;
      b->in_mode = 1;
      for (int h = 0; h < b->P; ++h) b->in_ptr[h] = t + h * player_bytes;
      int32_t periodic_step = -1;
      if (b->ops->display)
        for (int k = 0; k < tp.n_steps; ++k)
          if ((tp.f0 + k + 1) % 100 == 0) periodic_step = k;
      st = launch_program(b, tp, true, b->ops->display, periodic_step);
      b->in_mode = 0;
      for (auto& q : b->in_ptr) q = nullptr;
      if (st != RB_OK) { result = st; break; }
    }
    b->live_valid = tp.live_out;
    b->display_frame = tp.f0 + tp.n_steps;
    b->tick += 1;
  }
  if (result == RB_OK) result = flush(done);
  else flush(done);
  if (early && done < n_ticks)  // the device already ran all n ticks: it is ahead of the plan for good
    b->poisoned = "batch poisoned: a fused launch ran " + std::to_string(n_ticks) + " ticks but the host bookkeeping stopped after " +
                  std::to_string(done) + " (" + b->last_err + ")";
  if (tmp) (void)hipFreeAsync(tmp, b->stream);
  if (ticks_done) *ticks_done = done;
  if (result == RB_OK && (b->cfg.flags & RB_FLAG_CHECKED)) {
    // The status waits for the call's launches (the kernels set pinned_counters[0] themselves: nothing
    // is copied).  Measured on the driver's 20-tick call: 86-88 us of wall against 81-83 unchecked;
    // polling a completion event instead took 88-91 (profiles/r06_ab_checked.log).
    HIP_TRY(b, hipStreamSynchronize(b->stream));
    if (b->pinned_counters[0] > 0) {
      b->last_err = "Detected checksum mismatch during rollback (see rb_mismatches).";
      result = RB_MISMATCHED_CHECKSUM;
    }
  }
  return result;
}

rb_status rb_synchronize(rb_batch* b) {
  if (b->plan_only) return RB_OK;
  HIP_TRY(b, hipStreamSynchronize(b->stream));
  return RB_OK;
}

rb_status rb_mismatches(rb_batch* b, int32_t* frames_out, int32_t* count_out) {
  if (b->plan_only) {
    if (count_out) *count_out = 0;
    return RB_OK;
  }
  std::vector<int32_t> e(b->Spad);
  HIP_TRY(b, hipMemcpyAsync(e.data(), b->err, b->Spad * 4, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(b, hipStreamSynchronize(b->stream));
  int32_t n = 0;
  for (int s = 0; s < b->S; ++s) {
    if (e[s] != kNullFrame) ++n;
    if (frames_out) frames_out[s] = e[s];
  }
  if (count_out) *count_out = n;
  return RB_OK;
}

int32_t rb_last_requests(const rb_batch* b, int32_t* kinds, int32_t* frames, int32_t cap) {
  const auto& t = b->plan->trace;
  const int32_t n = static_cast<int32_t>(t.size());
  for (int32_t i = 0; i < n && i < cap; ++i) {
    if (kinds) kinds[i] = t[i].kind;
    if (frames) frames[i] = t[i].frame;
  }
  return n;
}

rb_status rb_read_cell(rb_batch* b, int32_t frame, void* images, uint64_t* checksums) {
  if (b->plan_only) return fail(b, RB_INVALID_REQUEST, "plan-only batch holds no states");
  if (frame < 0 || b->plan->cell_frame[frame % b->W] != frame)
    return fail(b, RB_INVALID_REQUEST, "no cell holds frame " + std::to_string(frame));
  const size_t slot = static_cast<size_t>(frame % b->W);
  std::vector<uint32_t> planes;
  rb_status st = read_words_slot(b, b->snap + slot * b->ops->nw * b->Spad * b->ops->lanes, planes);
  if (st != RB_OK) return st;
  std::vector<uint8_t> csh(static_cast<size_t>(b->Spad) * b->ops->cs_bytes);
  HIP_TRY(b, hipMemcpy(csh.data(), static_cast<uint8_t*>(b->cs) + slot * b->Spad * b->ops->cs_bytes, csh.size(),
                       hipMemcpyDeviceToHost));
  // A session that stopped on MismatchedChecksum keeps the cells of its last
  // tick: its slot holds the newest frame <= (its final frame - 1) of that slot.
  std::vector<int32_t> stop(static_cast<size_t>(b->Spad));
  HIP_TRY(b, hipMemcpy(stop.data(), b->live_frame, stop.size() * 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> w(b->ops->nw * b->ops->lanes);
  for (int s = 0; s < b->S; ++s) {
    words_of(b, planes, s, w.data());
    int32_t f = frame;
    if (stop[s] != kNullFrame) {
      const int32_t last = stop[s] - 1;
      f = last - ((last - static_cast<int32_t>(slot)) % b->W + b->W) % b->W;
    }
    if (images) b->ops->image(w.data(), f, static_cast<uint8_t*>(images) + static_cast<size_t>(s) * b->ops->image_bytes);
    if (checksums) {
      U128 c = b->ops->cs_at(csh.data(), s);
      checksums[2 * s] = c.lo;
      checksums[2 * s + 1] = c.hi;
    }
  }
  return RB_OK;
}

rb_status rb_read_live(rb_batch* b, void* images, uint64_t* display_checksums, int32_t* display_frames) {
  if (b->plan_only) return fail(b, RB_INVALID_REQUEST, "plan-only batch holds no states");
  const int32_t cur = b->plan->current;
  if (!b->live_valid) {
    // The last tick ended right before a LoadGameState, so its final state
    // was not stored: replay it from the cell it saved (frame cur-1) and the
    // confirmed input of that frame.  Deterministic, touches nothing else.
    TickProgram tp;
    tp.load = true;
    tp.load_frame = cur - 1;
    tp.f0 = cur - 1;
    tp.n_steps = 1;
    tp.live_out = true;
    if (b->plan->cell_frame[(cur - 1) % b->W] != cur - 1)
      return fail(b, RB_PANIC, "live-state replay: cell for the last frame is missing");
    rb_status st = launch_program(b, tp, false, false, -1);
    if (st != RB_OK) return st;
    b->live_valid = true;
  }
  std::vector<uint32_t> planes;
  rb_status st = read_words_slot(b, b->live, planes);
  if (st != RB_OK) return st;
  std::vector<uint8_t> dcs(static_cast<size_t>(b->Spad) * b->ops->cs_bytes);
  HIP_TRY(b, hipMemcpy(dcs.data(), b->last_cs, dcs.size(), hipMemcpyDeviceToHost));
  std::vector<int32_t> e(b->Spad), lf(b->Spad);
  HIP_TRY(b, hipMemcpy(e.data(), b->err, b->Spad * 4, hipMemcpyDeviceToHost));
  HIP_TRY(b, hipMemcpy(lf.data(), b->live_frame, b->Spad * 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> w(b->ops->nw * b->ops->lanes);
  for (int s = 0; s < b->S; ++s) {
    words_of(b, planes, s, w.data());
    // a failed session stopped advancing at the end of the tick that detected it
    const int32_t fr = e[s] != kNullFrame ? lf[s] : cur;
    if (images) b->ops->image(w.data(), fr, static_cast<uint8_t*>(images) + static_cast<size_t>(s) * b->ops->image_bytes);
    if (display_checksums) display_checksums[s] = b->ops->display ? b->ops->cs_at(dcs.data(), s).lo : 0;
    if (display_frames) display_frames[s] = b->ops->display ? (e[s] != kNullFrame ? lf[s] : b->display_frame) : kNullFrame;
  }
  return RB_OK;
}

rb_status rb_export_checksum_report(rb_batch* b, int32_t frame, void* dev_out) {
  if (b->plan_only) return fail(b, RB_INVALID_REQUEST, "plan-only batch holds no states");
  if (frame < 0 || b->plan->cell_frame[frame % b->W] != frame)
    return fail(b, RB_INVALID_REQUEST, "no cell holds frame " + std::to_string(frame));
  const size_t slot = static_cast<size_t>(frame % b->W);
  HIP_TRY(b, b->ops->launch_report(static_cast<uint8_t*>(b->cs) + slot * b->Spad * b->ops->cs_bytes, b->err, b->S,
                                   frame, dev_out, b->stream));
  return RB_OK;
}

namespace rb {
// rb_export_compact_report: 4 B per session (16-bit checksums only).
__global__ void compact_report_kernel(const uint16_t* __restrict__ cs, const int32_t* __restrict__ err, int S,
                                      int32_t frame, uint32_t* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const int32_t e = err[s];
  uint32_t r = cs[s];
  if (e != kNullFrame) r |= 0x80000000u | (static_cast<uint32_t>(min(max(frame - e, 0), 0x7FFF)) << 16);
  out[s] = r;
}

}  // namespace rb

rb_status rb_export_compact_report(rb_batch* b, int32_t frame, void* dev_out) {
  if (b->plan_only) return fail(b, RB_INVALID_REQUEST, "plan-only batch holds no states");
  if (b->ops->cs_bytes != 2)
    return fail(b, RB_INVALID_REQUEST, "compact reports carry 16-bit checksums: use rb_export_checksum_report");
  if (frame < 0 || b->plan->cell_frame[frame % b->W] != frame)
    return fail(b, RB_INVALID_REQUEST, "no cell holds frame " + std::to_string(frame));
  const size_t slot = static_cast<size_t>(frame % b->W);
  hipLaunchKernelGGL(rb::compact_report_kernel, dim3((b->S + 255) / 256), dim3(256), 0, b->stream,
                     reinterpret_cast<const uint16_t*>(static_cast<uint8_t*>(b->cs) + slot * b->Spad * 2), b->err, b->S,
                     frame, static_cast<uint32_t*>(dev_out));
  HIP_TRY(b, hipGetLastError());
  return RB_OK;
}

rb_status rb_debug_corrupt_cell(rb_batch* b, int32_t session, int32_t frame, int32_t word, uint32_t xor_mask) {
  if (b->plan_only) return fail(b, RB_INVALID_REQUEST, "plan-only batch holds no states");
  if (session < 0 || session >= b->S || word < 0 || word >= b->ops->canon_words)
    return fail(b, RB_INVALID_REQUEST, "session/word out of range");
  if (frame < 0 || b->plan->cell_frame[frame % b->W] != frame)
    return fail(b, RB_INVALID_REQUEST, "no cell holds frame " + std::to_string(frame));
  int lane, wk;
  b->ops->word_loc(word, &lane, &wk);
  const int L = b->ops->lanes;
  uint32_t* p = b->snap + static_cast<size_t>(frame % b->W) * b->ops->nw * b->Spad * L +
                word_index(b->ops->nw, b->Spad * L, session * L + lane, wk);
  uint32_t v;
  HIP_TRY(b, hipStreamSynchronize(b->stream));
  HIP_TRY(b, hipMemcpy(&v, p, 4, hipMemcpyDeviceToHost));
  v ^= xor_mask;
  HIP_TRY(b, hipMemcpy(p, &v, 4, hipMemcpyHostToDevice));
  return RB_OK;
}

}  // extern "C"

// Element-wise device evaluation for the parity tests: (a[i], b[i]) -> (o1[i], o2[i]).
template <class Launch>
static rb_status debug_map2(const char* what, int32_t device, const float* a, const float* b, float* o1, float* o2,
                            int64_t n, Launch launch) {
  rb_batch* none = nullptr;
  if (n <= 0) return RB_OK;
  HIP_TRY(none, hipSetDevice(device));
  float *da = nullptr, *db = nullptr, *d1 = nullptr, *d2 = nullptr;
  uint32_t* du = nullptr;
  const size_t bytes = static_cast<size_t>(n) * 4;
  hipError_t e = hipMalloc(&da, bytes);
  if (e == hipSuccess) e = hipMalloc(&db, bytes);
  if (e == hipSuccess) e = hipMalloc(&d1, bytes);
  if (e == hipSuccess) e = hipMalloc(&d2, bytes);
  if (e == hipSuccess) e = hipMalloc(&du, 4);
  if (e == hipSuccess) e = hipMemset(du, 0, 4);
  if (e == hipSuccess) e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess && b) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    launch(dim3(static_cast<unsigned>((n + 255) / 256)), da, db, d1, d2, du);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(o1, d1, bytes, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(o2, d2, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(d1);
  (void)hipFree(d2);
  (void)hipFree(du);
  if (e != hipSuccess) return fail(nullptr, RB_DEVICE_ERROR, std::string(what) + ": " + hipGetErrorString(e));
  return RB_OK;
}

extern "C" {

rb_status rb_debug_sincosf(int32_t device, const float* x, float* so, float* co, int64_t n) {
  return debug_map2("rb_debug_sincosf", device, x, nullptr, so, co, n,
                    [n](dim3 grid, float* da, float*, float* d1, float* d2, uint32_t* du) {
                      hipLaunchKernelGGL(sincos_kernel, grid, dim3(256), 0, nullptr, da, d1, d2, n, du);
                    });
}

rb_status rb_debug_exgame_inrange(int32_t device, uint32_t first_bits, int64_t n, float* dev_out) {
  if (n <= 0 || !dev_out) return RB_INVALID_REQUEST;
  // the in-range forms are exact on [+0, 6.5) only (games.hpp ExGame::in_range)
  if (first_bits >= 0x40D00000u || static_cast<uint64_t>(first_bits) + static_cast<uint64_t>(n) > 0x40D00000ull)
    return RB_INVALID_REQUEST;
  if (hipSetDevice(device) != hipSuccess) return RB_DEVICE_ERROR;
  hipLaunchKernelGGL(inrange_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, nullptr, first_bits, n,
                     dev_out);
  if (hipGetLastError() != hipSuccess) return RB_DEVICE_ERROR;
  return hipDeviceSynchronize() == hipSuccess ? RB_OK : RB_DEVICE_ERROR;
}

rb_status rb_debug_speed_clamp(int32_t device, const float* vx, const float* vy, float* ox, float* oy, int64_t n) {
  return debug_map2("rb_debug_speed_clamp", device, vx, vy, ox, oy, n,
                    [n](dim3 grid, float* da, float* db, float* d1, float* d2, uint32_t*) {
                      hipLaunchKernelGGL(clamp_kernel, grid, dim3(256), 0, nullptr, da, db, d1, d2, n);
                    });
}

rb_status rb_profile_enable(rb_batch* b, int32_t on) {
  b->prof = on != 0;
  b->prof_every = on > 1 ? static_cast<uint32_t>(on) : 8u;
  b->prof_tick = 0;
  // Create the event pool now, outside any timed region: a first hipEventCreate
  // inside one costs tens of microseconds of host time.
  if (b->prof && !b->plan_only) {
    HIP_TRY(b, hipSetDevice(b->device));
    const size_t fresh = b->prof_ev.size();
    while (b->prof_ev.size() < kProfPool) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      HIP_TRY(b, hipEventCreate(&e0));
      HIP_TRY(b, hipEventCreate(&e1));
      b->prof_ev.push_back({e0, e1});
    }
    // ... and record every new event once: the runtime sets an event's
    // completion signal up at its first record, which costs host time that
    // would otherwise land in the first timed call
    for (size_t i = fresh; i < b->prof_ev.size(); ++i) {
      HIP_TRY(b, hipEventRecord(b->prof_ev[i].first, b->stream));
      HIP_TRY(b, hipEventRecord(b->prof_ev[i].second, b->stream));
    }
    HIP_TRY(b, hipStreamSynchronize(b->stream));
    b->prof_ticks.resize(b->prof_ev.size());
  }
  return RB_OK;
}

rb_status rb_launch_clock_arm(rb_batch* b, int32_t launches) {
  if (b->plan_only || launches <= 0) return fail(b, RB_INVALID_REQUEST, "rb_launch_clock_arm: plan-only batch or no launches");
  HIP_TRY(b, hipSetDevice(b->device));
  HIP_TRY(b, b->clock.arm((static_cast<size_t>(b->Spad) * b->ops->lanes + 63) / 64, static_cast<size_t>(launches), b->stream));
  return RB_OK;
}

rb_status rb_launch_clock_read(rb_batch* b, uint64_t* start_end, int32_t cap, int32_t* launches) {
  if (!b->clock.armed) return fail(b, RB_INVALID_REQUEST, "rb_launch_clock_read: not armed");
  HIP_TRY(b, b->clock.read(start_end, cap, launches, b->stream));
  return RB_OK;
}

rb_status rb_profile_take(rb_batch* b, double* total_ms, int32_t* launches) {
  double t = 0;
  int32_t ticks = 0;
  if (!b->plan_only && b->prof_used > 0) {
    HIP_TRY(b, hipEventSynchronize(b->prof_ev[b->prof_used - 1].second));
    for (size_t i = 0; i < b->prof_used; ++i) {
      float ms = 0;
      HIP_TRY(b, hipEventElapsedTime(&ms, b->prof_ev[i].first, b->prof_ev[i].second));
      t += ms;
      ticks += b->prof_ticks[i];
    }
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = ticks;
  b->prof_used = 0;
  return RB_OK;
}

}  // extern "C"
