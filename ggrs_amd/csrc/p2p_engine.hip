// ggrs_amd/csrc/p2p_engine.hip — host side of the P2PSession batches
// (include/ggrs_amd.h rb_p2p_*): buffers, validation (builder.rs), launches of
// p2p_kernel (p2p.hpp) and the read-backs the parity tests use.
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernels.hpp"

using namespace rb;

struct rb_p2p {
  rb_p2p_config cfg{};
  std::unique_ptr<GameOps> ops;
  int S = 0, Spad = 0, W = 0, P = 0, block = 256;
  int device = 0;
  uint32_t simds = 1024;  // SIMDs of the device (MI355X: 256 CUs x 4)
  hipStream_t own_stream = nullptr, stream = nullptr;
  uint32_t* snap = nullptr;
  void* cs = nullptr;
  int32_t* tag = nullptr;
  void* ring = nullptr;
  uint32_t* live = nullptr;
  int32_t* qs = nullptr;
  int32_t* status = nullptr;
  int32_t* trace = nullptr;
  uint32_t* counters = nullptr;
  unsigned long long* stats = nullptr;  // [ST_COUNT][Spad]
  bool fanout = false;
  bool per_player = false;   // RB_P2P_FLAG_FANOUT_PER_PLAYER
  bool sync_ticks = false;   // RB_P2P_SYNC_TICKS=1 at create: lock-step ticks (p2p.hpp kAsync off)
  bool fan_generic = false;  // RB_FANOUT_GENERIC=1 at create: fanout_kernel for every game
  uint32_t* spec_state = nullptr;
  uint32_t* spec_cells = nullptr;
  void* spec_cs = nullptr;
  int32_t* spec_meta = nullptr;
  std::vector<uint8_t> disconnected;  // host mirror [P][S] of ConnectionStatus::disconnected (validation)
  uint8_t* disc_mask = nullptr;       // [S] device copy of rb_p2p_disconnect_player's session mask
  DesyncParams ds{};                  // desync detection buffers (desync_interval > 0)
  PeerParams peer{};                  // peers' connect-status reports (RB_P2P_FLAG_PEER_STATUS)
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev;
  size_t prof_used = 0;
  LaunchClock clock;  // rb_p2p_launch_clock_arm
  // the adaptive fan-out (RB_P2P_FLAG_FANOUT without _ALWAYS, include/ggrs_amd.h)
  struct FanPolicy {
    bool adaptive = false;
    bool active = true;          // presimulating
    bool open = false;           // a measurement window is open (its start sums are in host[0..1])
    bool pending = false;        // its end sums are on their way to host[2..3] (event `ev`)
    int32_t ticks = 0;           // ticks into the window (active) or into the pause (inactive)
    int32_t since_end = 0;       // ticks since the pending window ended (the decision waits kFanDecideTicks)
    uint32_t min_permille = 150;
    unsigned long long* dev = nullptr;   // [4] device sums: selects, loads (window start; end)
    unsigned long long* host = nullptr;  // [4] pinned copies
    hipEvent_t ev = nullptr;
    double last_frac = -1.0;
    int32_t windows = 0, turned_off = 0;
  } fan;
  std::string last_err;
};
constexpr int32_t kFanProbeTicks = 64, kFanPauseTicks = 960;
constexpr uint64_t kFanMinRollbacks = 64;  // a window with fewer rollbacks decides nothing

namespace {
thread_local std::string g_p2p_err;

rb_status pfail(rb_p2p* b, rb_status st, const std::string& msg) {
  if (b) b->last_err = msg;
  else g_p2p_err = msg;
  return st;
}
#define P2P_TRY(b, expr)                                                                                    \
  do {                                                                                                      \
    hipError_t _e = (expr);                                                                                 \
    if (_e != hipSuccess) return pfail((b), RB_DEVICE_ERROR, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

void free_all(rb_p2p* b) {
  (void)hipSetDevice(b->device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  void* ptrs[] = {b->snap,   b->cs,      b->tag,       b->ring,       b->live,    b->qs,       b->status,
                  b->trace,  b->counters, b->stats, b->spec_state, b->spec_cells, b->spec_cs, b->spec_meta,
                  b->disc_mask};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  void* dptrs[] = {b->ds.lh_frame, b->ds.lh_cs,    b->ds.rh_frame, b->ds.rh_lo,     b->ds.rh_hi,
                   b->ds.rh_meta,  b->ds.ob_frame, b->ds.ob_cs,    b->ds.ob_n,      b->ds.ev_n,
                   b->ds.ev_frame, b->ds.ev_handle, b->ds.ev_local, b->ds.ev_remote};
  for (void* q : dptrs)
    if (q) (void)hipFree(q);
  if (b->fan.dev) (void)hipFree(b->fan.dev);
  if (b->fan.host) (void)hipHostFree(b->fan.host);
  if (b->fan.ev) (void)hipEventDestroy(b->fan.ev);
  if (b->peer.last) (void)hipFree(b->peer.last);
  if (b->peer.disc) (void)hipFree(b->peer.disc);
  for (auto& pr : b->prof_ev) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  b->clock.release();
  if (b->own_stream) (void)hipStreamDestroy(b->own_stream);
}

template <class T>
rb_status read_rows(rb_p2p* b, const T* dev, size_t rows, std::vector<T>& host) {
  host.resize(rows * static_cast<size_t>(b->Spad));
  P2P_TRY(b, hipMemcpyAsync(host.data(), dev, host.size() * sizeof(T), hipMemcpyDeviceToHost, b->stream));
  P2P_TRY(b, hipStreamSynchronize(b->stream));
  return RB_OK;
}

// session s's words [lanes][nw] from a block of lane planes, as its canonical image
// disconnect_player_at_frame (p2p_session.rs:555-581) for one remote handle:
// mark it disconnected and, if the session already simulated past its last
// input, set disconnect_frame = last_frame + 1
// The adaptive fan-out's measurement: selects and LoadGameStates summed over the batch into out[0..1].
__global__ void fan_sums_kernel(const unsigned long long* __restrict__ stats, int S, int Spad,
                                unsigned long long* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long sel = s < S ? stats[static_cast<size_t>(ST_SELECT) * Spad + s] : 0ull;
  unsigned long long ld = s < S ? stats[static_cast<size_t>(ST_LOAD) * Spad + s] : 0ull;
  for (int o = 32; o > 0; o >>= 1) {
    sel += __shfl_down(sel, o, 64);
    ld += __shfl_down(ld, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&out[0], sel);
    atomicAdd(&out[1], ld);
  }
}

__global__ void p2p_disconnect_kernel(int32_t* qs, const uint8_t* mask, int32_t S, int32_t Spad, int32_t h) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S || (mask && !mask[s])) return;
  const size_t sp = static_cast<size_t>(Spad);
  auto row = [&](int field) -> int32_t& { return qs[(QS_PLAYER0 + field * 4 + h) * sp + s]; };
  const int32_t cur = qs[QS_CUR * sp + s];
  const uint32_t m = static_cast<uint32_t>(row(QF_MISC));
  const int32_t last = (m & kQmEsc) ? row(QF_ABS0 + 1) : fd_dec(static_cast<uint32_t>(row(QF_LA_CONN)) >> 16, cur);
  row(QF_MISC) = static_cast<int32_t>(m | kQmDisc);
  if (cur > last) qs[QS_DISC_FRAME * sp + s] = last + 1;
}

// UdpProtocol::on_checksum_report (protocol.rs:710-722) for the endpoint of
// remote handle h in every session: the peer's reports, oldest first,
// in[k * S + s] for k < K (frame NULL_FRAME = none).
__global__ void p2p_receive_reports_kernel(DesyncParams d, const rb_checksum_report* __restrict__ in, int K, int S,
                                           int Spad, int h) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  auto at = [&](size_t k) { return k * static_cast<size_t>(Spad) + static_cast<size_t>(s); };
  const size_t m = static_cast<size_t>(h) * 3;
  int head = d.rh_meta[at(m)], n = d.rh_meta[at(m + 1)], last = d.rh_meta[at(m + 2)];
  for (int k = 0; k < K; ++k) {
    const rb_checksum_report r = in[static_cast<size_t>(k) * S + s];
    if (r.frame == kNullFrame || !(last < r.frame)) continue;
    if (n > kMaxChecksumHistory) {  // retain(|&frame, _| frame > last_added - MAX): the oldest leave the front
      while (n > 0 && d.rh_frame[at(static_cast<size_t>(h) * kCsHist + static_cast<size_t>(head))] <= last - kMaxChecksumHistory) {
        head = (head + 1) % kCsHist;
        --n;
      }
    }
    last = r.frame;
    if (n >= kCsHist) continue;  // cannot happen: at most 33 entries
    const size_t slot = static_cast<size_t>(h) * kCsHist + static_cast<size_t>((head + n) % kCsHist);
    d.rh_frame[at(slot)] = r.frame;
    d.rh_lo[at(slot)] = r.checksum_lo;
    d.rh_hi[at(slot)] = r.checksum_hi;
    ++n;
  }
  d.rh_meta[at(m)] = head;
  d.rh_meta[at(m + 1)] = n;
  d.rh_meta[at(m + 2)] = last;
}

// The reports sent since the last take, oldest first, out[k * S + s] for
// k < kOutbox (only the newest kOutbox are kept); resets the outbox.
__global__ void p2p_take_reports_kernel(DesyncParams d, rb_checksum_report* __restrict__ out, int S, int Spad) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  auto at = [&](int k) { return static_cast<size_t>(k) * static_cast<size_t>(Spad) + static_cast<size_t>(s); };
  const uint32_t n = d.ob_n[s];
  const uint32_t cnt = n < static_cast<uint32_t>(kOutbox) ? n : static_cast<uint32_t>(kOutbox);
  for (int k = 0; k < kOutbox; ++k) {
    rb_checksum_report r{0, 0, kNullFrame, kNullFrame};
    if (static_cast<uint32_t>(k) < cnt) {
      const int q = static_cast<int>((n - cnt + static_cast<uint32_t>(k)) % kOutbox);
      r.frame = d.ob_frame[at(q)];
      r.checksum_lo = d.ob_cs[at(q)];
    }
    out[static_cast<size_t>(k) * S + s] = r;
  }
  d.ob_n[s] = 0;
}

// UdpProtocol::on_input's connect-status merge (protocol.rs:627-636) for one endpoint
__global__ void p2p_peer_status_kernel(PeerParams pp, const int32_t* __restrict__ last, const uint8_t* __restrict__ disc,
                                       int S, int Spad, int P, int e) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  for (int i = 0; i < P; ++i) {
    const size_t o = (static_cast<size_t>(e) * 4 + static_cast<size_t>(i)) * Spad + s;
    pp.last[o] = max(pp.last[o], last[static_cast<size_t>(i) * S + s]);
    pp.disc[o] = pp.disc[o] | (disc[static_cast<size_t>(i) * S + s] ? 1 : 0);
  }
}

void image_from_planes(const rb_p2p* b, const std::vector<uint32_t>& planes, int s, int32_t frame, uint8_t* out) {
  const int L = b->ops->lanes, NW = b->ops->nw;
  std::vector<uint32_t> w(static_cast<size_t>(L) * NW);
  for (int l = 0; l < L; ++l)
    for (int k = 0; k < NW; ++k) w[l * NW + k] = planes[word_index(NW, b->Spad * L, s * L + l, k)];
  b->ops->image(w.data(), frame, out);
}
}  // namespace

extern "C" {

void rb_p2p_config_init(rb_p2p_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->abi_version = RB_ABI_VERSION;
  c->game = RB_GAME_EX_GAME;
  c->num_sessions = 1;
  c->num_players = 2;     // builder.rs:13
  c->max_prediction = 8;  // builder.rs:20
  c->input_delay = 0;     // builder.rs:16
  c->device = 0;
  c->local_mask = 1u;     // handle 0 local, handle 1 remote (ex_game_p2p.rs's two-peer setup)
  c->remote_delay = 0;
  c->sparse_saving = 0;   // builder.rs:17 DEFAULT_SAVE_MODE
  c->fanout_candidates = kSpecBranches;
}

const char* rb_p2p_last_error(const rb_p2p* b) { return b ? b->last_err.c_str() : g_p2p_err.c_str(); }

rb_status rb_p2p_create(const rb_p2p_config* cfg, rb_p2p** out) {
  *out = nullptr;
  if (!cfg || cfg->abi_version != RB_ABI_VERSION) return pfail(nullptr, RB_INVALID_REQUEST, "rb_p2p_config.abi_version mismatch");
  if (cfg->max_prediction <= 0)  // builder.rs:136-145
    return pfail(nullptr, RB_INVALID_REQUEST, "Currently, only prediction windows above 0 are supported");
  if (cfg->num_players <= 0 || cfg->num_players > 4 || cfg->num_sessions <= 0 || cfg->input_delay < 0 ||
      cfg->remote_delay < 0 || cfg->desync_interval < 0)
    return pfail(nullptr, RB_INVALID_REQUEST, "num_players must be 1..4; sizes and delays non-negative");
  const uint32_t all = (1u << cfg->num_players) - 1u;
  if ((cfg->local_mask & ~all) != 0)  // builder.rs:103-115: handles must be < num_players
    return pfail(nullptr, RB_INVALID_REQUEST,
                 "The player handle you provided is invalid. For a local player, the handle should be between 0 and num_players");
  if (cfg->local_mask == 0 || cfg->local_mask == all)
    return pfail(nullptr, RB_INVALID_REQUEST, "a P2P batch needs at least one local and one remote handle");
  if (cfg->max_prediction > 64 || cfg->input_delay + cfg->max_prediction + 2 > kQueueLen)
    return pfail(nullptr, RB_INVALID_REQUEST, "max_prediction / input delay do not fit the 128-entry input queue");
  if (cfg->game != RB_GAME_EX_GAME && cfg->game != RB_GAME_STUB && cfg->game != RB_GAME_STUB_ENUM &&
      cfg->game != RB_GAME_BRAWLER && cfg->game < RB_GAME_PLUGIN_BASE)
    return pfail(nullptr, RB_INVALID_REQUEST,
                 "P2P batches support ex_game, the stub games, the brawler and registered plugin games");
  auto ops = make_game(cfg->game, cfg->num_players, (cfg->flags & RB_FLAG_LANE_PER_SESSION) != 0);
  if (!ops) return pfail(nullptr, RB_INVALID_REQUEST, "unsupported game / num_players combination (RB_FLAG_LANE_PER_SESSION: A/B builds only)");
  const bool fanout = (cfg->flags & RB_P2P_FLAG_FANOUT) != 0;
  if (fanout && (!ops->fanout_supported || cfg->sparse_saving))
    return pfail(nullptr, RB_INVALID_REQUEST,
                 "speculative fan-out needs ex_game with one lane per player or the brawler, no sparse saving");
  if (fanout && (cfg->fanout_candidates < 1 || cfg->fanout_candidates > kSpecBranches))
    return pfail(nullptr, RB_INVALID_REQUEST, "fanout_candidates must be 1..16");
  const bool per_player = fanout && (cfg->flags & RB_P2P_FLAG_FANOUT_PER_PLAYER) != 0;
  if (per_player && (!ops->inlane_fanout || ops->input_alphabet > static_cast<uint32_t>(cfg->fanout_candidates)))
    return pfail(nullptr, RB_INVALID_REQUEST,
                 "per-player speculation needs independent players (ex_game) and fanout_candidates covering the "
                 "input alphabet");
  if (static_cast<uint64_t>(cfg->max_prediction) * ops->nw * ops->lanes *
          ((static_cast<uint64_t>(cfg->num_sessions) + 63) / 64 * 64) >= (1ull << 32))
    return pfail(nullptr, RB_INVALID_REQUEST, "batch too large for 32-bit snapshot offsets");
  // the fan-out's branch planes: a slot's offset is 64-bit (p2p.hpp), the words inside one slot
  // (planes x columns, load_words / store_words) are int offsets: at most 2^31 words per slot (the
  // brawler at 65,536 sessions is exactly that: 32 planes of 2^26 columns, the last plane's int
  // offset 31 x 2^26)
  if (fanout && static_cast<uint64_t>(ops->nw) * ops->lanes * (kSpecBranches + (per_player ? 1 : 0)) *
                        ((static_cast<uint64_t>(cfg->num_sessions) + 63) / 64 * 64) > (1ull << 31))
    return pfail(nullptr, RB_INVALID_REQUEST, "batch too large for the fan-out's 31-bit branch-plane offsets");

  auto b = std::make_unique<rb_p2p>();
  b->cfg = *cfg;
  b->ops = std::move(ops);
  b->S = cfg->num_sessions;
  b->Spad = (cfg->num_sessions + 63) / 64 * 64;
  b->W = cfg->max_prediction;
  b->P = cfg->num_players;
  b->block = cfg->block_size ? static_cast<int>(cfg->block_size) : 256;
  if (b->block % 64 != 0 || b->block > 256) return pfail(nullptr, RB_INVALID_REQUEST, "block_size must be 64, 128, 192 or 256");
  b->device = cfg->device;
  b->fanout = fanout;
  b->per_player = per_player;
  if (const char* e = std::getenv("RB_P2P_SYNC_TICKS")) b->sync_ticks = std::atoi(e) != 0;
  if (const char* e = std::getenv("RB_FANOUT_GENERIC")) b->fan_generic = std::atoi(e) != 0;
  rb_p2p* bp = b.get();
  auto hip_fail = [&](hipError_t e, const char* what) {
    g_p2p_err = std::string(what) + ": " + hipGetErrorString(e);
    free_all(bp);
    return RB_DEVICE_ERROR;
  };
#define P2P_CREATE(expr)                              \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return hip_fail(_e, #expr); \
  } while (0)
  P2P_CREATE(hipSetDevice(b->device));
  int cus = 0;
  P2P_CREATE(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, b->device));
  b->simds = 4 * cus;  // 4 SIMDs per CU (CDNA)
  P2P_CREATE(hipStreamCreateWithFlags(&b->own_stream, hipStreamNonBlocking));
  b->stream = b->own_stream;
  const size_t Sp = b->Spad, NW = b->ops->nw, W = b->W, L = b->ops->lanes, Gp = Sp * L;
  const size_t ring_bytes = static_cast<size_t>(kQueueLen) * b->P * Sp * b->ops->input_bytes;
  P2P_CREATE(hipMalloc(&b->snap, W * NW * Gp * 4));
  P2P_CREATE(hipMalloc(&b->cs, W * Sp * b->ops->cs_bytes));
  P2P_CREATE(hipMalloc(&b->tag, W * Sp * 4));
  P2P_CREATE(hipMalloc(&b->ring, ring_bytes));
  P2P_CREATE(hipMalloc(&b->live, NW * Gp * 4));
  P2P_CREATE(hipMalloc(&b->qs, kQsFields * Sp * 4));
  P2P_CREATE(hipMalloc(&b->status, Sp * 4));
  P2P_CREATE(hipMalloc(&b->trace, Sp * 4));
  P2P_CREATE(hipMalloc(&b->counters, 16));
  P2P_CREATE(hipMalloc(&b->stats, ST_COUNT * Sp * 8));
  P2P_CREATE(hipMemsetAsync(b->snap, 0, W * NW * Gp * 4, b->stream));
  P2P_CREATE(hipMemsetAsync(b->cs, 0, W * Sp * b->ops->cs_bytes, b->stream));
  P2P_CREATE(hipMemsetAsync(b->tag, 0xff, W * Sp * 4, b->stream));  // GameState::default frame = NULL_FRAME
  P2P_CREATE(hipMemsetAsync(b->ring, 0, ring_bytes, b->stream));     // blank inputs
  P2P_CREATE(hipMemsetAsync(b->status, 0, Sp * 4, b->stream));
  P2P_CREATE(hipMemsetAsync(b->trace, 0xff, Sp * 4, b->stream));  // no tick yet: NULL load frame (at frame 0), counts 0xFF
  P2P_CREATE(hipMemsetAsync(b->counters, 0, 16, b->stream));
  P2P_CREATE(hipMemsetAsync(b->stats, 0, ST_COUNT * Sp * 8, b->stream));
  if (b->fanout) {
    // branch columns per lane column: 16 (fanout_kernel: [session][branch][lane]; the one-player in-kernel
    // fan-out uses 16 + L of 16 * L), plus one own chain per lane for the per-player form
    const size_t K = kSpecBranches + (per_player ? 1 : 0);
    P2P_CREATE(hipMalloc(&b->spec_state, K * NW * Gp * 4));
    P2P_CREATE(hipMalloc(&b->spec_cells, W * K * NW * Gp * 4));
    P2P_CREATE(hipMalloc(&b->spec_cs, W * K * Sp * b->ops->cs_bytes));
    P2P_CREATE(hipMalloc(&b->spec_meta, SM_COUNT * Sp * 4));
    P2P_CREATE(hipMemsetAsync(b->spec_meta, 0, SM_COUNT * Sp * 4, b->stream));  // nothing valid yet
    b->fan.adaptive = (cfg->flags & RB_P2P_FLAG_FANOUT_ALWAYS) == 0;
    if (cfg->fanout_min_select_permille) b->fan.min_permille = cfg->fanout_min_select_permille;
    if (b->fan.adaptive) {
      P2P_CREATE(hipMalloc(&b->fan.dev, 4 * sizeof(unsigned long long)));
      P2P_CREATE(hipHostMalloc(&b->fan.host, 4 * sizeof(unsigned long long)));
      P2P_CREATE(hipEventCreateWithFlags(&b->fan.ev, hipEventDisableTiming));
    }
  }
  // SyncLayer::new / InputQueue::new / ConnectionStatus::default: every frame NULL, current 0,
  // connected, length 0, the first input at frame 0 (q_pack)
  std::vector<int32_t> qs(kQsFields * Sp, kNullFrame);
  const QPacked q0 = q_pack(QFields{kNullFrame, kNullFrame, kNullFrame, kNullFrame, kNullFrame, 0, 0, false, 0u}, 0);
  for (size_t s = 0; s < Sp; ++s) {
    qs[QS_CUR * Sp + s] = 0;
    qs[QS_SAVED_CONF * Sp + s] = static_cast<int32_t>(fd_enc(kNullFrame, 0) | fd_enc(kNullFrame, 0) << 16);
    for (int h = 0; h < 4; ++h) {
      for (int i = 0; i < 4; ++i) qs[(QS_PLAYER0 + (QF_LA_CONN + i) * 4 + h) * Sp + s] = static_cast<int32_t>(q0.w[i]);
      qs[(QS_PLAYER0 + QF_PRED_VAL * 4 + h) * Sp + s] = 0;
      qs[(QS_PLAYER0 + QF_MTF_N * 4 + h) * Sp + s] = 0;  // the fan-out's candidate list starts empty
    }
  }
  b->disconnected.assign(static_cast<size_t>(b->P) * b->S, 0);
  P2P_CREATE(hipMalloc(&b->disc_mask, Sp));
  P2P_CREATE(hipMemcpyAsync(b->qs, qs.data(), qs.size() * 4, hipMemcpyHostToDevice, b->stream));
  if (cfg->flags & RB_P2P_FLAG_PEER_STATUS) {  // ConnectionStatus::default for every (endpoint, player)
    P2P_CREATE(hipMalloc(&b->peer.last, 16 * Sp * 4));
    P2P_CREATE(hipMalloc(&b->peer.disc, 16 * Sp * 4));
    P2P_CREATE(hipMemsetAsync(b->peer.last, 0xff, 16 * Sp * 4, b->stream));  // NULL_FRAME
    P2P_CREATE(hipMemsetAsync(b->peer.disc, 0, 16 * Sp * 4, b->stream));
    b->peer.on = 1;
  }
  if (cfg->desync_interval > 0) {  // empty histories, outbox and event rings
    DesyncParams& d = b->ds;
    d.interval = cfg->desync_interval;
    const size_t H = kCsHist, R = 4;
    P2P_CREATE(hipMalloc(&d.lh_frame, H * Sp * 4));
    P2P_CREATE(hipMalloc(&d.lh_cs, H * Sp * 8));
    P2P_CREATE(hipMalloc(&d.rh_frame, R * H * Sp * 4));
    P2P_CREATE(hipMalloc(&d.rh_lo, R * H * Sp * 8));
    P2P_CREATE(hipMalloc(&d.rh_hi, R * H * Sp * 8));
    P2P_CREATE(hipMalloc(&d.rh_meta, R * 3 * Sp * 4));
    P2P_CREATE(hipMalloc(&d.ob_frame, kOutbox * Sp * 4));
    P2P_CREATE(hipMalloc(&d.ob_cs, kOutbox * Sp * 8));
    P2P_CREATE(hipMalloc(&d.ob_n, Sp * 4));
    P2P_CREATE(hipMalloc(&d.ev_n, Sp * 4));
    P2P_CREATE(hipMalloc(&d.ev_frame, kEvents * Sp * 4));
    P2P_CREATE(hipMalloc(&d.ev_handle, kEvents * Sp * 4));
    P2P_CREATE(hipMalloc(&d.ev_local, kEvents * Sp * 8));
    P2P_CREATE(hipMalloc(&d.ev_remote, kEvents * Sp * 8));
    P2P_CREATE(hipMemsetAsync(d.lh_frame, 0xff, H * Sp * 4, b->stream));  // NULL_FRAME: empty slot
    P2P_CREATE(hipMemsetAsync(d.lh_cs, 0, H * Sp * 8, b->stream));
    P2P_CREATE(hipMemsetAsync(d.rh_frame, 0xff, R * H * Sp * 4, b->stream));
    std::vector<int32_t> meta(R * 3 * Sp, 0);  // head 0, length 0, last_added_checksum_frame NULL_FRAME
    for (size_t h = 0; h < R; ++h)
      for (size_t s = 0; s < Sp; ++s) meta[(h * 3 + 2) * Sp + s] = kNullFrame;
    P2P_CREATE(hipMemcpy(d.rh_meta, meta.data(), meta.size() * 4, hipMemcpyHostToDevice));
    P2P_CREATE(hipMemsetAsync(d.ob_n, 0, Sp * 4, b->stream));
    P2P_CREATE(hipMemsetAsync(d.ev_n, 0, Sp * 4, b->stream));
    P2P_CREATE(hipMemsetAsync(d.ev_frame, 0xff, kEvents * Sp * 4, b->stream));
    P2P_CREATE(hipMemsetAsync(d.ev_handle, 0xff, kEvents * Sp * 4, b->stream));
  }
  // State::new for every session
  std::vector<uint32_t> w0(L * NW), planes(NW * Gp);
  b->ops->init_words(w0.data());
  for (size_t s = 0; s < Sp; ++s)
    for (size_t l = 0; l < L; ++l)
      for (size_t k = 0; k < NW; ++k)
        planes[word_index(static_cast<int>(NW), static_cast<int>(Gp), static_cast<int>(s * L + l), static_cast<int>(k))] =
            w0[l * NW + k];
  P2P_CREATE(hipMemcpyAsync(b->live, planes.data(), planes.size() * 4, hipMemcpyHostToDevice, b->stream));
  P2P_CREATE(hipStreamSynchronize(b->stream));
#undef P2P_CREATE
  *out = b.release();
  return RB_OK;
}

void rb_p2p_destroy(rb_p2p* b) {
  if (!b) return;
  free_all(b);
  delete b;
}

rb_status rb_p2p_set_stream(rb_p2p* b, void* s) {
  P2P_TRY(b, hipStreamSynchronize(b->stream));
  b->stream = s ? static_cast<hipStream_t>(s) : b->own_stream;
  return RB_OK;
}

void* rb_p2p_get_stream(const rb_p2p* b) { return static_cast<void*>(b->stream); }

int32_t rb_p2p_state_bytes(const rb_p2p* b) { return b->ops->image_bytes; }
int32_t rb_p2p_input_bytes(const rb_p2p* b) { return b->ops->input_bytes; }

namespace {
// The batch's buffers and configuration for a P2P launch (the per-call tensors are the caller's).
P2PParams base_params(const rb_p2p* b) {
  P2PParams p{};
  p.snap = b->snap;
  p.cs = b->cs;
  p.tag = b->tag;
  p.ring = b->ring;
  p.live = b->live;
  p.qs = b->qs;
  p.status = b->status;
  p.trace = b->trace;
  p.counters = b->counters;
  p.stats = b->stats;
  p.S = b->S;
  p.Spad = b->Spad;
  p.W = b->W;
  p.delay = b->cfg.input_delay;
  p.remote_delay = b->cfg.remote_delay;
  p.local_mask = b->cfg.local_mask;
  p.sparse = b->cfg.sparse_saving != 0;
  p.sync_ticks = b->sync_ticks ? 1 : 0;
  p.many_waves = static_cast<uint64_t>(b->Spad) * b->ops->lanes > 2ull * 64ull * b->simds ? 1 : 0;
  p.fan_generic = b->fan_generic ? 1 : 0;
  p.fan_k = b->cfg.fanout_candidates;
  p.spec_on = b->fanout ? 1 : 0;
  p.spec_per_player = b->per_player && !b->fan_generic ? 1 : 0;
  p.spec_state = b->spec_state;
  p.spec_cells = b->spec_cells;
  p.spec_cs = b->spec_cs;
  p.spec_meta = b->spec_meta;
  p.ds = b->ds;
  p.peer = b->peer;
  return p;
}
}  // namespace

namespace {
// The adaptive fan-out (include/ggrs_amd.h RB_P2P_FLAG_FANOUT_ALWAYS).  Windows of kFanProbeTicks
// ticks back to back while presimulating; each window's select and LoadGameState sums are reduced on
// the device into pinned memory at its end (host[2..3], event `ev`) and its start (host[0..1]: the
// previous window's end).  The decision is taken kFanDecideTicks ticks after a window's end, at the
// first call from then on, waiting for the event (long complete by then): so whether a tick
// speculates depends only on the batch's inputs and call sizes, never on when a copy landed.
constexpr int32_t kFanDecideTicks = 16;
rb_status fan_snapshot(rb_p2p* b, int off) {
  P2P_TRY(b, hipMemsetAsync(b->fan.dev + off, 0, 2 * sizeof(unsigned long long), b->stream));
  hipLaunchKernelGGL(fan_sums_kernel, dim3((b->S + 255) / 256), dim3(256), 0, b->stream, b->stats, b->S, b->Spad,
                     b->fan.dev + off);
  P2P_TRY(b, hipGetLastError());
  P2P_TRY(b, hipMemcpyAsync(b->fan.host + off, b->fan.dev + off, 2 * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost, b->stream));
  return RB_OK;
}
// Branches are valid only for the tick right after the launch that made them (SM_END == current
// frame); a pause's plain ticks leave the metadata as it was, so it is cleared when presimulation
// stops and again when it restarts.
rb_status fan_invalidate(rb_p2p* b) {
  P2P_TRY(b, hipMemsetAsync(b->spec_meta + static_cast<size_t>(SM_VALID) * b->Spad, 0, static_cast<size_t>(b->Spad) * 4,
                            b->stream));
  return RB_OK;
}
rb_status fan_before(rb_p2p* b) {
  auto& f = b->fan;
  if (!f.adaptive) return RB_OK;
  if (f.pending && f.since_end >= kFanDecideTicks) {
    P2P_TRY(b, hipEventSynchronize(f.ev));
    f.pending = false;
    const uint64_t sel = f.host[2] - f.host[0], ld = f.host[3] - f.host[1];
    f.windows += 1;
    if (sel + ld >= kFanMinRollbacks) {
      f.last_frac = static_cast<double>(sel) / static_cast<double>(sel + ld);
      if (sel * 1000ull < static_cast<uint64_t>(f.min_permille) * (sel + ld)) {
        f.active = false;  // a pause of kFanPauseTicks plain ticks
        f.open = false;
        f.ticks = 0;
        f.turned_off += 1;
        rb_status r = fan_invalidate(b);
        if (r != RB_OK) return r;
      }
    }
    if (f.active) {  // the next window started at this one's end
      f.host[0] = f.host[2];
      f.host[1] = f.host[3];
    }
  }
  if (!f.active && f.ticks >= kFanPauseTicks) {  // measure again
    f.active = true;
    f.open = false;
    rb_status r = fan_invalidate(b);
    if (r != RB_OK) return r;
  }
  if (f.active && !f.open) {
    rb_status r = fan_snapshot(b, 0);
    if (r != RB_OK) return r;
    f.open = true;
    f.ticks = 0;
  }
  return RB_OK;
}
rb_status fan_after(rb_p2p* b, int32_t n) {
  auto& f = b->fan;
  if (!f.adaptive) return RB_OK;
  f.ticks += n;
  if (f.pending) f.since_end += n;
  if (f.active && f.open && !f.pending && f.ticks >= kFanProbeTicks) {
    rb_status r = fan_snapshot(b, 2);
    if (r != RB_OK) return r;
    P2P_TRY(b, hipEventRecord(f.ev, b->stream));
    f.pending = true;
    f.since_end = 0;
    f.ticks = 0;
  }
  return RB_OK;
}
// hipSetDevice for the batch's calls, the caller's current device restored on every return
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
}  // namespace

rb_status rb_p2p_fanout_state(rb_p2p* b, int32_t* active, double* select_fraction, int32_t* windows,
                              int32_t* turned_off) {
  if (!b->fanout) return pfail(b, RB_INVALID_REQUEST, "the batch has no fan-out");
  if (active) *active = (!b->fan.adaptive || b->fan.active) ? 1 : 0;
  if (select_fraction) *select_fraction = b->fan.last_frac;
  if (windows) *windows = b->fan.windows;
  if (turned_off) *turned_off = b->fan.turned_off;
  return RB_OK;
}

rb_status rb_p2p_run_ticks(rb_p2p* b, int32_t n_ticks, const void* local_inputs, int64_t local_stride,
                           const int32_t* remote_upto, const void* remote_inputs, int32_t remote_frames) {
  if (n_ticks <= 0) return RB_OK;
  if (!local_inputs || !remote_upto || !remote_inputs || remote_frames <= 0)
    return pfail(b, RB_INVALID_REQUEST, "rb_p2p_run_ticks: missing input tensor");
  P2PParams p = base_params(b);
  p.local_in = static_cast<const uint8_t*>(local_inputs);
  p.local_stride = local_stride;
  p.upto = remote_upto;
  p.upto_stride = static_cast<int64_t>(b->P) * b->S;
  p.remote_in = static_cast<const uint8_t*>(remote_inputs);
  p.remote_frames = remote_frames;
  p.T = n_ticks;
  DeviceScope dev_scope(b->device);
  if (b->fanout) {
    rb_status r = fan_before(b);
    if (r != RB_OK) return r;
  }
  const bool spec = b->fanout && (!b->fan.adaptive || b->fan.active);
  p.spec_on = spec ? 1 : 0;
  FanParams fp{};
  fp.status = b->status;
  fp.snap = b->snap;
  fp.tag = b->tag;
  fp.ring = b->ring;
  fp.qs = b->qs;
  fp.spec_state = b->spec_state;
  fp.spec_cells = b->spec_cells;
  fp.spec_cs = b->spec_cs;
  fp.spec_meta = b->spec_meta;
  fp.stats = b->stats;
  fp.counters = b->counters;
  fp.S = b->S;
  fp.Spad = b->Spad;
  fp.W = b->W;
  fp.local_mask = b->cfg.local_mask;
  fp.fan_generic = b->fan_generic ? 1 : 0;
  fp.fan_k = b->cfg.fanout_candidates;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (b->prof) {
    if (b->prof_used == b->prof_ev.size()) {
      P2P_TRY(b, hipEventCreate(&e0));
      P2P_TRY(b, hipEventCreate(&e1));
      b->prof_ev.emplace_back(e0, e1);
    }
    e0 = b->prof_ev[b->prof_used].first;
    e1 = b->prof_ev[b->prof_used].second;
  }
  const bool one_launch = !spec || (b->ops->inlane_fanout && !b->fan_generic);
  hipError_t e = hipSuccess;
  if (one_launch) {
    // all ticks in one launch (with the in-kernel fan-out); timed by the kernel's own start / end
    p.launch_clock = b->clock.next();
    e = b->ops->launch_p2p(p, b->block, b->stream, LaunchEv{e0, e1});
  } else {
    if (e0) P2P_TRY(b, hipEventRecord(e0, b->stream));
    // fanout_kernel between ticks needs every lane of a session's branches: one
    // P2P launch and one fan-out launch per tick
    P2PParams pt = p;
    pt.T = 1;
    for (int32_t t = 0; t < n_ticks && e == hipSuccess; ++t) {
      pt.local_in = p.local_in + static_cast<int64_t>(t) * p.local_stride;
      pt.upto = p.upto + static_cast<int64_t>(t) * p.upto_stride;
      pt.launch_clock = b->clock.next();
      e = b->ops->launch_p2p(pt, b->block, b->stream);
      fp.launch_clock = b->clock.next();
      if (e == hipSuccess) e = b->ops->launch_fanout(fp, b->block, b->stream);
    }
  }
  if (e != hipSuccess) return pfail(b, RB_DEVICE_ERROR, std::string("p2p launch: ") + hipGetErrorString(e));
  if (e1 && !one_launch) P2P_TRY(b, hipEventRecord(e1, b->stream));
  if (e0) ++b->prof_used;  // only a launch that went out has its event pair recorded
  if (b->fanout) return fan_after(b, n_ticks);
  return RB_OK;
}

rb_status rb_p2p_run_ticks_packets(rb_p2p* b, int32_t n_ticks, const void* local_inputs, int64_t local_stride,
                                   const uint8_t* packets, int64_t packet_stride, const int32_t* lengths,
                                   const int32_t* start_frames, int32_t* decode_status, int32_t* acks) {
  if (n_ticks <= 0) return RB_OK;
  if (!local_inputs || !packets || !lengths || !start_frames)
    return pfail(b, RB_INVALID_REQUEST, "rb_p2p_run_ticks_packets: missing input tensor");
  if (packet_stride < 32 || packet_stride % 16 != 0 || reinterpret_cast<uintptr_t>(packets) % 16 != 0)
    return pfail(b, RB_INVALID_REQUEST, "rb_p2p_run_ticks_packets: packets need 16-byte alignment and a stride of at least 32");
  if (b->cfg.sparse_saving || b->fanout || b->ds.interval > 0 || b->peer.on)
    return pfail(b, RB_INVALID_REQUEST,
                 "rb_p2p_run_ticks_packets: sparse saving, the fan-out and network reports take rb_p2p_run_ticks");
  // a packet's reference input (frame start - 1) may be as old as the newest received frame -
  // 2 * max_prediction (recv_inputs' retain, protocol.rs:684-686); the 128-entry input queue ring
  // holds the newest 128 frames, so that frame must be younger than last - 127
  if (2 * b->W >= kQueueLen)
    return pfail(b, RB_INVALID_REQUEST, "rb_p2p_run_ticks_packets: needs 2 * max_prediction < 128 (the input ring)");
  P2PParams p = base_params(b);
  p.local_in = static_cast<const uint8_t*>(local_inputs);
  p.local_stride = local_stride;
  p.T = n_ticks;
  p.packets = packets;
  p.packet_stride = packet_stride;
  p.pk_len = lengths;
  p.pk_start = start_frames;
  p.pk_status = decode_status;
  p.acks = acks;
  p.launch_clock = b->clock.next();
  DeviceScope dev_scope(b->device);
  LaunchEv ev;  // the kernel's own start / end (hipExtLaunchKernel)
  if (b->prof) {
    if (b->prof_used == b->prof_ev.size()) {
      hipEvent_t e0 = nullptr, e2 = nullptr;
      P2P_TRY(b, hipEventCreate(&e0));
      P2P_TRY(b, hipEventCreate(&e2));
      b->prof_ev.emplace_back(e0, e2);
    }
    ev = LaunchEv{b->prof_ev[b->prof_used].first, b->prof_ev[b->prof_used].second};
  }
  hipError_t e = b->ops->launch_p2p(p, b->block, b->stream, ev);
  if (e != hipSuccess) return pfail(b, RB_DEVICE_ERROR, std::string("p2p launch: ") + hipGetErrorString(e));
  if (ev.start) ++b->prof_used;  // only a launch that went out has its event pair recorded
  return RB_OK;
}

rb_status rb_p2p_disconnect_player(rb_p2p* b, int32_t handle, const uint8_t* session_mask) {
  if (handle < 0 || handle >= b->P) return pfail(b, RB_INVALID_REQUEST, "Invalid Player Handle.");
  if ((b->cfg.local_mask >> handle) & 1u) return pfail(b, RB_INVALID_REQUEST, "Local Player cannot be disconnected.");
  if (b->peer.on) {  // peers' reports disconnect players inside the ticks: refresh the mirror
    std::vector<int32_t> qs;
    rb_status r = read_rows(b, b->qs, kQsFields, qs);
    if (r != RB_OK) return r;
    for (int h = 0; h < b->P; ++h)
      for (int s = 0; s < b->S; ++s)
        b->disconnected[static_cast<size_t>(h) * b->S + s] = (static_cast<uint32_t>(qs[(QS_PLAYER0 + QF_MISC * 4 + h) * b->Spad + s]) & kQmDisc) != 0;
  }
  uint8_t* d = b->disconnected.data() + static_cast<size_t>(handle) * b->S;
  for (int s = 0; s < b->S; ++s)
    if ((!session_mask || session_mask[s]) && d[s]) return pfail(b, RB_INVALID_REQUEST, "Player already disconnected.");
  for (int s = 0; s < b->S; ++s)
    if (!session_mask || session_mask[s]) d[s] = 1;
  P2P_TRY(b, hipSetDevice(b->device));
  if (session_mask) {
    P2P_TRY(b, hipMemcpyAsync(b->disc_mask, session_mask, b->S, hipMemcpyHostToDevice, b->stream));
    P2P_TRY(b, hipStreamSynchronize(b->stream));  // the host mask may be reused as soon as we return
  }
  const int blocks = (b->S + 255) / 256;
  hipLaunchKernelGGL(p2p_disconnect_kernel, dim3(blocks), dim3(256), 0, b->stream, b->qs,
                     session_mask ? b->disc_mask : nullptr, b->S, b->Spad, handle);
  P2P_TRY(b, hipGetLastError());
  return RB_OK;
}

rb_status rb_p2p_read_status(rb_p2p* b, int32_t* status, int32_t* load_frame, int32_t* n_adv, int32_t* n_save) {
  std::vector<int32_t> st, tr, cur;
  rb_status r = read_rows(b, b->status, 1, st);
  if (r == RB_OK) r = read_rows(b, b->trace, 1, tr);
  if (r == RB_OK) r = read_rows(b, b->qs + QS_CUR * b->Spad, 1, cur);
  if (r != RB_OK) return r;
  for (int s = 0; s < b->S; ++s) {  // trace_pack
    const uint32_t t = static_cast<uint32_t>(tr[s]);
    const int32_t na = static_cast<int32_t>((t >> 16) & 0xFFu), ns = static_cast<int32_t>(t >> 24);
    if (status) status[s] = st[s] == kP2PStatusPanic ? RB_PANIC : st[s];
    if (load_frame) load_frame[s] = fd_dec(t, cur[s]);
    if (n_adv) n_adv[s] = na == 0xFF ? -1 : na;
    if (n_save) n_save[s] = ns == 0xFF ? -1 : ns;
  }
  return RB_OK;
}

rb_status rb_p2p_read_frames(rb_p2p* b, int32_t* current, int32_t* confirmed) {
  std::vector<int32_t> qs;
  rb_status r = read_rows(b, b->qs, kQsFields, qs);
  if (r != RB_OK) return r;
  for (int s = 0; s < b->S; ++s) {
    if (current) current[s] = qs[QS_CUR * b->Spad + s];
    if (confirmed) {
      const size_t Sp = b->Spad;
      const uint32_t sc = static_cast<uint32_t>(qs[QS_SAVED_CONF * Sp + s]);
      confirmed[s] = sc == kQsEscWord ? qs[QS_ABS_CONF * Sp + s] : fd_dec(sc >> 16, qs[QS_CUR * Sp + s]);
    }
  }
  return RB_OK;
}

rb_status rb_p2p_read_queues(rb_p2p* b, int32_t* out) {
  std::vector<int32_t> qs;
  rb_status r = read_rows(b, b->qs, kQsFields, qs);
  if (r != RB_OK) return r;
  static_assert(RB_P2P_QUEUE_FIELDS == 8, "last added, tail, length, last requested, prediction, first incorrect, connection, disconnected");
  const size_t Sp = b->Spad;
  for (int s = 0; s < b->S; ++s)
    for (int h = 0; h < b->P; ++h) {
      auto row = [&](int field) { return qs[(QS_PLAYER0 + field * 4 + h) * Sp + s]; };
      uint32_t w[4];
      int32_t ab[7];
      for (int i = 0; i < 4; ++i) w[i] = static_cast<uint32_t>(row(QF_LA_CONN + i));
      for (int i = 0; i < 7; ++i) ab[i] = row(QF_ABS0 + i);
      const QFields f = q_unpack(w, qs[QS_CUR * Sp + s], ab);
      const int32_t v[RB_P2P_QUEUE_FIELDS] = {f.la, f.tail, f.len, f.req, f.pred, f.fi, f.conn, f.disc ? 1 : 0};
      for (int k = 0; k < RB_P2P_QUEUE_FIELDS; ++k) out[(static_cast<size_t>(s) * b->P + h) * RB_P2P_QUEUE_FIELDS + k] = v[k];
    }
  return RB_OK;
}

rb_status rb_p2p_read_cells(rb_p2p* b, int32_t* tags, void* images, uint64_t* checksums) {
  std::vector<int32_t> tg;
  rb_status r = read_rows(b, b->tag, b->W, tg);
  if (r != RB_OK) return r;
  const size_t Sp = b->Spad, L = b->ops->lanes, NW = b->ops->nw, B = b->ops->image_bytes;
  std::vector<uint8_t> csh(b->W * Sp * b->ops->cs_bytes);
  P2P_TRY(b, hipMemcpy(csh.data(), b->cs, csh.size(), hipMemcpyDeviceToHost));
  std::vector<uint32_t> planes;
  for (int w = 0; w < b->W; ++w) {
    if (images) {
      r = read_rows(b, b->snap + static_cast<size_t>(w) * NW * Sp * L, NW * L, planes);
      if (r != RB_OK) return r;
    }
    for (int s = 0; s < b->S; ++s) {
      const int32_t f = tg[w * Sp + s];
      if (tags) tags[static_cast<size_t>(w) * b->S + s] = f;
      if (images) image_from_planes(b, planes, s, f, static_cast<uint8_t*>(images) + (static_cast<size_t>(w) * b->S + s) * B);
      if (checksums) {
        const U128 c = b->ops->cs_at(csh.data(), static_cast<size_t>(w) * Sp + s);
        checksums[(static_cast<size_t>(w) * b->S + s) * 2] = c.lo;
        checksums[(static_cast<size_t>(w) * b->S + s) * 2 + 1] = c.hi;
      }
    }
  }
  return RB_OK;
}

rb_status rb_p2p_read_live(rb_p2p* b, void* images) {
  std::vector<int32_t> qs;
  std::vector<uint32_t> planes;
  rb_status r = read_rows(b, b->qs, kQsFields, qs);
  if (r == RB_OK) r = read_rows(b, b->live, static_cast<size_t>(b->ops->nw) * b->ops->lanes, planes);
  if (r != RB_OK) return r;
  for (int s = 0; s < b->S; ++s)
    image_from_planes(b, planes, s, qs[QS_CUR * b->Spad + s],
                      static_cast<uint8_t*>(images) + static_cast<size_t>(s) * b->ops->image_bytes);
  return RB_OK;
}

rb_status rb_p2p_counters(rb_p2p* b, uint32_t* out3) {
  uint32_t c[4];
  P2P_TRY(b, hipStreamSynchronize(b->stream));
  P2P_TRY(b, hipMemcpy(c, b->counters, 16, hipMemcpyDeviceToHost));
  for (int i = 0; i < 3; ++i) out3[i] = c[i];
  return RB_OK;
}

rb_status rb_p2p_totals(rb_p2p* b, uint64_t* out5) {
  std::vector<unsigned long long> st;
  rb_status r = read_rows(b, b->stats, ST_COUNT, st);
  if (r != RB_OK) return r;
  for (int i = 0; i < ST_COUNT; ++i) {
    uint64_t t = 0;
    for (int s = 0; s < b->S; ++s) t += st[static_cast<size_t>(i) * b->Spad + s];
    out5[i] = t;
  }
  return RB_OK;
}

rb_status rb_p2p_take_checksum_reports(rb_p2p* b, void* dev_out) {
  if (b->ds.interval <= 0) return pfail(b, RB_INVALID_REQUEST, "desync detection is off (desync_interval = 0)");
  P2P_TRY(b, hipSetDevice(b->device));
  hipLaunchKernelGGL(p2p_take_reports_kernel, dim3((b->S + 255) / 256), dim3(256), 0, b->stream, b->ds,
                     static_cast<rb_checksum_report*>(dev_out), b->S, b->Spad);
  P2P_TRY(b, hipGetLastError());
  return RB_OK;
}

rb_status rb_p2p_receive_checksum_reports(rb_p2p* b, int32_t handle, const void* dev_in, int32_t count) {
  if (b->ds.interval <= 0) return pfail(b, RB_INVALID_REQUEST, "desync detection is off (desync_interval = 0)");
  if (handle < 0 || handle >= b->P || ((b->cfg.local_mask >> handle) & 1u))
    return pfail(b, RB_INVALID_REQUEST, "checksum reports come from a remote handle's endpoint");
  if (count <= 0) return RB_OK;
  P2P_TRY(b, hipSetDevice(b->device));
  hipLaunchKernelGGL(p2p_receive_reports_kernel, dim3((b->S + 255) / 256), dim3(256), 0, b->stream, b->ds,
                     static_cast<const rb_checksum_report*>(dev_in), count, b->S, b->Spad, handle);
  P2P_TRY(b, hipGetLastError());
  return RB_OK;
}

rb_status rb_p2p_receive_peer_connect_status(rb_p2p* b, int32_t endpoint, const int32_t* last_frames,
                                             const uint8_t* disconnected) {
  if (!b->peer.on) return pfail(b, RB_INVALID_REQUEST, "peer connect status needs RB_P2P_FLAG_PEER_STATUS");
  if (endpoint < 0 || endpoint >= b->P || ((b->cfg.local_mask >> endpoint) & 1u))
    return pfail(b, RB_INVALID_REQUEST, "connect-status reports come from a remote handle's endpoint");
  if (!last_frames || !disconnected) return pfail(b, RB_INVALID_REQUEST, "missing connect-status tensor");
  P2P_TRY(b, hipSetDevice(b->device));
  hipLaunchKernelGGL(p2p_peer_status_kernel, dim3((b->S + 255) / 256), dim3(256), 0, b->stream, b->peer, last_frames,
                     disconnected, b->S, b->Spad, b->P, endpoint);
  P2P_TRY(b, hipGetLastError());
  return RB_OK;
}

rb_status rb_p2p_read_desync_events(rb_p2p* b, uint32_t* counts, int32_t* frames, int32_t* handles,
                                    uint64_t* local_checksums, uint64_t* remote_checksums) {
  if (b->ds.interval <= 0) return pfail(b, RB_INVALID_REQUEST, "desync detection is off (desync_interval = 0)");
  const size_t Sp = b->Spad, E = kEvents;
  std::vector<uint32_t> n;
  std::vector<int32_t> fr, hd;
  std::vector<uint64_t> lo, ro;
  rb_status r = read_rows(b, b->ds.ev_n, 1, n);
  if (r == RB_OK) r = read_rows(b, b->ds.ev_frame, E, fr);
  if (r == RB_OK) r = read_rows(b, b->ds.ev_handle, E, hd);
  if (r == RB_OK) r = read_rows(b, b->ds.ev_local, E, lo);
  if (r == RB_OK) r = read_rows(b, b->ds.ev_remote, E, ro);
  if (r != RB_OK) return r;
  for (int s = 0; s < b->S; ++s) {
    const uint32_t cnt = n[s], kept = cnt < E ? cnt : static_cast<uint32_t>(E);
    if (counts) counts[s] = cnt;
    for (size_t e = 0; e < E; ++e) {  // oldest kept first
      const bool has = e < kept;
      const size_t q = (cnt - kept + e) % E, o = static_cast<size_t>(s) * E + e;
      if (frames) frames[o] = has ? fr[q * Sp + s] : kNullFrame;
      if (handles) handles[o] = has ? hd[q * Sp + s] : -1;
      if (local_checksums) local_checksums[o] = has ? lo[q * Sp + s] : 0;
      if (remote_checksums) remote_checksums[o] = has ? ro[q * Sp + s] : 0;
    }
  }
  return RB_OK;
}

rb_status rb_p2p_debug_corrupt(rb_p2p* b, int32_t session, int32_t word, uint32_t xor_mask) {
  if (session < 0 || session >= b->S || word < 0 || word >= b->ops->canon_words)
    return pfail(b, RB_INVALID_REQUEST, "rb_p2p_debug_corrupt: session or word out of range");
  int lane = 0, w = 0;
  b->ops->word_loc(word, &lane, &w);
  const int L = b->ops->lanes, NW = b->ops->nw;
  const size_t idx = word_index(NW, b->Spad * L, session * L + lane, w);
  P2P_TRY(b, hipSetDevice(b->device));
  P2P_TRY(b, hipStreamSynchronize(b->stream));
  const size_t plane = static_cast<size_t>(NW) * b->Spad * L;
  std::vector<uint32_t*> where{b->live + idx};
  for (int k = 0; k < b->W; ++k) where.push_back(b->snap + k * plane + idx);
  for (uint32_t* q : where) {
    uint32_t v = 0;
    P2P_TRY(b, hipMemcpy(&v, q, 4, hipMemcpyDeviceToHost));
    v ^= xor_mask;
    P2P_TRY(b, hipMemcpy(q, &v, 4, hipMemcpyHostToDevice));
  }
  return RB_OK;
}

rb_status rb_p2p_launch_clock_arm(rb_p2p* b, int32_t launches) {
  if (launches <= 0) return pfail(b, RB_INVALID_REQUEST, "rb_p2p_launch_clock_arm: no launches");
  DeviceScope dev_scope(b->device);
  // one slot holds the widest launch of the batch: fanout_kernel's 16 branches per session
  const size_t lanes = static_cast<size_t>(b->Spad) * b->ops->lanes * (b->fanout ? kSpecBranches : 1);
  P2P_TRY(b, b->clock.arm((lanes + 63) / 64, static_cast<size_t>(launches), b->stream));
  return RB_OK;
}

rb_status rb_p2p_launch_clock_read(rb_p2p* b, uint64_t* start_end, int32_t cap, int32_t* launches) {
  if (!b->clock.armed) return pfail(b, RB_INVALID_REQUEST, "rb_p2p_launch_clock_read: not armed");
  DeviceScope dev_scope(b->device);
  P2P_TRY(b, b->clock.read(start_end, cap, launches, b->stream));
  return RB_OK;
}

rb_status rb_p2p_profile_enable(rb_p2p* b, int32_t on) {
  b->prof = on != 0;
  // the event pool is created here, outside any timed region
  if (b->prof) {
    P2P_TRY(b, hipSetDevice(b->device));
    const size_t fresh = b->prof_ev.size();
    while (b->prof_ev.size() < 256) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      P2P_TRY(b, hipEventCreate(&e0));
      P2P_TRY(b, hipEventCreate(&e1));
      b->prof_ev.emplace_back(e0, e1);
    }
    for (size_t i = fresh; i < b->prof_ev.size(); ++i) {  // first records (signal set-up) outside timed regions
      P2P_TRY(b, hipEventRecord(b->prof_ev[i].first, b->stream));
      P2P_TRY(b, hipEventRecord(b->prof_ev[i].second, b->stream));
    }
    P2P_TRY(b, hipStreamSynchronize(b->stream));
  }
  return RB_OK;
}

rb_status rb_p2p_profile_take(rb_p2p* b, double* total_ms, int32_t* launches) {
  double t = 0;
  if (b->prof_used > 0) {
    P2P_TRY(b, hipEventSynchronize(b->prof_ev[b->prof_used - 1].second));
    for (size_t i = 0; i < b->prof_used; ++i) {
      float ms = 0;
      P2P_TRY(b, hipEventElapsedTime(&ms, b->prof_ev[i].first, b->prof_ev[i].second));
      t += ms;
    }
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = static_cast<int32_t>(b->prof_used);
  b->prof_used = 0;
  return RB_OK;
}

}  // extern "C"
