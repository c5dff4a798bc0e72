// ggrs_amd/csrc/p2p.hpp — device side of batched P2PSession rollback
// (sessions/p2p_session.rs:253-337, 621-673, 778-802 over sync_layer.rs and
// input_queue.rs), without the network layer.
//
// S independent P2P sessions, each seen from one peer: handles in
// `local_mask` are PlayerType::Local (input delay applies), the others are
// PlayerType::Remote.  UdpProtocol's only job on this path is to turn packets
// into Event::Input{input, player} in frame order (p2p_session.rs:838-852);
// here the caller hands the engine, per tick and remote handle, the newest
// delivered frame (`upto`) plus the inputs by frame — the device input tensor
// a batched packet decoder would fill.
//
// Unlike SyncTest, P2P bookkeeping is data dependent: a remote input that
// differs from its prediction sets the InputQueue's first_incorrect_frame, and
// the next advance_frame rolls back to it (per session).  So the whole
// request-stream state machine runs on the device, one lane group per session:
// with one lane per player (ex_game) each lane owns its player's InputQueue
// (the input_queue.rs state lives in that lane's registers) and the session
// values (confirmed frame, first incorrect frame) are lane-group minima (DPP).
// The game state stays in registers across the fused ticks of a launch; every
// SaveGameState stores the cell (SoA planes), its checksum and its frame tag.
//
// Device layout (Spad = S rounded up to 64; L lanes per session):
//   snap  [W][NW planes][Spad*L]  cells, slot = frame % W (sync_layer.rs:71-75)
//   cs    [W][Spad] CS            GameStateCell::checksum
//   tag   [W][Spad] i32           GameStateCell::frame (per session: sessions drift apart)
//   ring  [128][P][Spad] Input    InputQueue::inputs, slot = frame % 128
//   live  [NW planes][Spad*L]     game state between launches
//   qs    [kQsFields][Spad] i32   session + per-player queue scalars (QS_* below)
#pragma once
#include <hip/hip_runtime.h>

#include "games.hpp"

namespace rb {

// The persistent bookkeeping of a P2P session (P2PParams::qs, [kQsFields][Spad] i32), packed: every
// frame number is a 16-bit delta from the session's current frame (fd_enc), so a one-tick launch
// reads and writes 4 words per player instead of 9 and 8 (the bookkeeping was
// 6.2x the tick's algorithmic bytes).  The deltas a session can hold are bounded by the input queue
// (128 frames) and the prediction window, except a disconnected player's frozen frames and extreme
// deliveries: a value outside the 16-bit range sets the row's escape code and is kept in absolute
// rows, written and read only then, so every value stays exact.
enum : int {
  QS_CUR = 0,         // SyncLayer::current_frame
  QS_SAVED_CONF = 1,  // SyncLayer::last_saved_frame | last_confirmed_frame << 16 (deltas; kQsEscWord: absolute rows)
  QS_DISC_FRAME = 2,  // P2PSession::disconnect_frame (p2p_session.rs:130), stored only when it changes
  QS_ABS_SAVED = 3,   // the absolute frames behind kQsEscWord
  QS_ABS_CONF = 4,
  QS_PLAYER0 = 5,     // + field * 4 + player (4 player slots)
};
enum : int {
  QF_LA_CONN = 0,   // InputQueue::last_added_frame | ConnectionStatus::last_frame << 16 (messages.rs:5-18), deltas
  QF_PRED_FI = 1,   // InputQueue::prediction.frame | first_incorrect_frame << 16, deltas
  QF_REQ_TAIL = 2,  // InputQueue::last_requested_frame | frame of inputs[tail] << 16 (input_queue.rs:83-101), deltas
  QF_MISC = 3,      // InputQueue::length (i16) | disconnected << 16 | escape << 17 | prediction.input << 24 (1-byte inputs)
  QF_PRED_VAL = 4,  // InputQueue::prediction.input of inputs wider than a byte
  QF_ABS0 = 5,      // 7 rows behind the escape bit: last added, connection, prediction, first incorrect, requested, tail, length
  // the fan-out's candidate list (not GGRS state): the queue's 16 most recent distinct
  // inputs, newest first, as two u64 (4 rows), and their count
  QF_MTF0 = 12,
  QF_MTF_N = 16,
  QF_COUNT = 17,
};
constexpr int kQsFields = QS_PLAYER0 + QF_COUNT * 4;
constexpr uint32_t kFdNull = 0x8000u, kFdEsc = 0x8001u;  // 16-bit codes: NULL_FRAME, escaped
constexpr uint32_t kQsEscWord = kFdEsc | kFdEsc << 16;
constexpr uint32_t kQmDisc = 1u << 16, kQmEsc = 1u << 17;
__host__ __device__ __forceinline__ bool fd_fits(int32_t f, int32_t base) {
  return f == kNullFrame || (f - base >= -32766 && f - base <= 32767);
}
__host__ __device__ __forceinline__ uint32_t fd_enc(int32_t f, int32_t base) {
  return f == kNullFrame ? kFdNull : static_cast<uint32_t>(f - base) & 0xFFFFu;
}
__host__ __device__ __forceinline__ int32_t fd_dec(uint32_t v, int32_t base) {
  v &= 0xFFFFu;
  return v == kFdNull ? kNullFrame : base + static_cast<int32_t>(static_cast<int16_t>(static_cast<uint16_t>(v)));
}
// One player's queue fields and their packed rows QF_LA_CONN .. QF_MISC (esc: the absolute rows hold them)
struct QFields {
  int32_t la, conn, pred, fi, req, tail, len;
  bool disc;
  uint32_t pv;  // prediction.input (the QF_MISC byte for 1-byte inputs)
};
struct QPacked {
  uint32_t w[4];
  bool esc;
};
__host__ __device__ __forceinline__ QPacked q_pack(const QFields& f, int32_t cur) {
  const bool esc = !(fd_fits(f.la, cur) && fd_fits(f.conn, cur) && fd_fits(f.pred, cur) && fd_fits(f.fi, cur) &&
                     fd_fits(f.req, cur) && fd_fits(f.tail, cur) && f.len >= -32768 && f.len <= 32767);
  QPacked r;
  r.w[0] = fd_enc(f.la, cur) | fd_enc(f.conn, cur) << 16;
  r.w[1] = fd_enc(f.pred, cur) | fd_enc(f.fi, cur) << 16;
  r.w[2] = fd_enc(f.req, cur) | fd_enc(f.tail, cur) << 16;
  r.w[3] = (static_cast<uint32_t>(f.len) & 0xFFFFu) | (f.disc ? kQmDisc : 0u) | (esc ? kQmEsc : 0u) | (f.pv & 0xFFu) << 24;
  r.esc = esc;
  return r;
}
// abs: the 7 absolute rows (read only when the escape bit is set)
__host__ __device__ __forceinline__ QFields q_unpack(const uint32_t (&w)[4], int32_t cur, const int32_t (&abs)[7]) {
  QFields f;
  const bool esc = (w[3] & kQmEsc) != 0;
  f.la = esc ? abs[0] : fd_dec(w[0], cur);
  f.conn = esc ? abs[1] : fd_dec(w[0] >> 16, cur);
  f.pred = esc ? abs[2] : fd_dec(w[1], cur);
  f.fi = esc ? abs[3] : fd_dec(w[1] >> 16, cur);
  f.req = esc ? abs[4] : fd_dec(w[2], cur);
  f.tail = esc ? abs[5] : fd_dec(w[2] >> 16, cur);
  f.len = esc ? abs[6] : static_cast<int32_t>(static_cast<int16_t>(static_cast<uint16_t>(w[3] & 0xFFFFu)));
  f.disc = (w[3] & kQmDisc) != 0;
  f.pv = w[3] >> 24;
  return f;
}
// trace word (the last tick of the last launch): LoadGameState frame as a delta from the current
// frame | AdvanceFrame count << 16 | SaveGameState count << 24 (at most 2 * 64 + 1 each; 0xFF: none yet)
__host__ __device__ __forceinline__ uint32_t trace_pack(int32_t load_frame, int32_t nadv, int32_t nsave, int32_t cur) {
  return fd_enc(load_frame, cur) | (static_cast<uint32_t>(nadv) & 0xFFu) << 16 | (static_cast<uint32_t>(nsave) & 0xFFu) << 24;
}
constexpr int32_t kP2PStatusOk = 0, kP2PStatusThreshold = 1, kP2PStatusPanic = 101;
// decode status of a packet-fed tick's endpoint (the codes of wire.hip's rb_decode_input_packets):
// inputs added, nothing new, malformed (the reference panics, protocol.rs:656; also a length past
// the packet row), a gap (a packet starting past the frame after the last one received: the
// reference's assert!, protocol.rs:639-642, so inside a tick the session panics too)
constexpr int32_t kWireOk = 0, kWireNothing = 1, kWirePanic = -1, kWireGap = -2;
// executed work: AdvanceFrames, SaveGameStates, LoadGameStates, rollbacks
// replaced by a speculative branch select, branch frames presimulated
enum : int { ST_ADV = 0, ST_SAVE = 1, ST_LOAD = 2, ST_SELECT = 3, ST_BRANCH = 4, ST_COUNT = 5 };
// Speculative fan-out: branch k holds candidate input cand[k] for one remote
// player over its unconfirmed frames.  Up to kSpecBranches
// candidates: the game's whole input alphabet when it has at most that many
// values (ex_game's 4 bits: cand[k] = k), else the K most likely values
// (fan_candidates below).
constexpr int kSpecBranches = 16;
// spec_meta rows: first speculated frame (base), frame the branch states are at
// (end), speculated handle, valid flag, then the 16 candidate inputs (1-byte
// inputs, 4 per row; 0xFF..: no branch) the branches presimulated
enum : int { SM_BASE = 0, SM_END = 1, SM_PLAYER = 2, SM_VALID = 3, SM_CAND = 4, SM_COUNT = 8 };

// The input alphabet a game's fan-out draws candidates from: G::kInputAlphabet,
// else every value of its Input.
template <class G, class = void>
struct InputAlphabet {
  static constexpr uint32_t value = G::kInputBytes >= 2 ? 0xFFFFFFFFu : 256u;
};
template <class G>
struct InputAlphabet<G, std::void_t<decltype(G::kInputAlphabet)>> {
  static constexpr uint32_t value = G::kInputAlphabet;
};

// The K candidate inputs of the speculated player (K <= kSpecBranches, 1-byte
// inputs): with an alphabet of at most K values, the alphabet in value order
// (branch k = input k); otherwise the most recently confirmed distinct values,
// newest first (the reference's prediction, repeat-last, input_queue.rs:126-140,
// is candidate 0) — the player's queue keeps them as a move-to-front list of
// its 16 most recent distinct inputs, updated as each input is added (mtf_push),
// so picking the candidates reads no input history (the list is kept only by
// launches that speculate, kSpec && kMtf: while the adaptive fan-out pauses,
// p2p_engine.hip, or with peers' connect-status reports on, the plain kernels
// leave it as it was, and the first speculating launch after a pause draws its
// candidates from that older list — a worse guess, never a wrong result: a
// select takes a branch only when the confirmed inputs hold its candidate on
// every frame, try_select) — then, while the queue has
// seen fewer than K distinct values, the smallest values not yet taken.  Packed
// 4 per word, unused slots 0xFF.  For the in-kernel fan-out, whose branches are
// input classes (InputCanon), the list holds classes (DevQueue::mcanon) and the
// fill takes only class representatives (`allowed`): ex_game's K = 8 then
// covers 8 of its 9 classes instead of the classes of 8 raw inputs.
// The fill of fan_candidates: the smallest values of the alphabet not among the first `take` list
// entries, into list slots take .. K-1.  Out of line: it runs only while a queue has seen fewer
// than K distinct inputs, and its bitmaps would otherwise hold registers in the fan-out kernels.
struct CandList {
  uint64_t lo, hi;
};
__device__ __noinline__ CandList fan_fill(uint64_t lo, uint64_t hi, int take, uint32_t alphabet, int K,
                                         uint64_t allowed) {
  uint64_t present[4] = {~allowed, 0ull, 0ull, 0ull};  // values never filled count as taken
  for (int i = 0; i < take; ++i) {
    const uint32_t v = static_cast<uint32_t>((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 0xFFull);
    present[v >> 6] |= 1ull << (v & 63);
  }
  for (int i = take; i < K; ++i) {
    int q = 0;
    while (q < 3 && present[q] == ~0ull) ++q;
    const uint32_t x = static_cast<uint32_t>(q * 64 + __builtin_ctzll(~present[q]));
    if (x >= alphabet) break;
    const uint64_t m = 0xFFull << (8 * (i & 7)), xv = static_cast<uint64_t>(x) << (8 * (i & 7));
    if (i < 8) lo = (lo & ~m) | xv;
    else hi = (hi & ~m) | xv;
    present[q] |= 1ull << (x & 63);
  }
  return CandList{lo, hi};
}
__device__ __forceinline__ void fan_candidates(uint64_t mlo, uint64_t mhi, int32_t mn, uint32_t alphabet, int K,
                                               uint32_t (&packed)[4], uint64_t allowed = ~0ull) {
  if (alphabet <= static_cast<uint32_t>(K)) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t i = static_cast<uint32_t>(4 * w + b);
        x |= (i < alphabet ? i : 0xFFu) << (8 * b);
      }
      packed[w] = x;
    }
    return;
  }
  const int take = min(mn, K);  // the first `take` list entries, the rest 0xFF
  const uint64_t klo = take >= 8 ? ~0ull : ((1ull << (8 * take)) - 1ull);
  const uint64_t khi = take <= 8 ? 0ull : (take >= 16 ? ~0ull : ((1ull << (8 * (take - 8))) - 1ull));
  uint64_t lo = (mlo & klo) | ~klo, hi = (mhi & khi) | ~khi;
  if (take < K) {  // a queue that has seen fewer than K distinct inputs
    const CandList c = fan_fill(lo, hi, take, alphabet, K, allowed);
    lo = c.lo;
    hi = c.hi;
  }
  packed[0] = static_cast<uint32_t>(lo);
  packed[1] = static_cast<uint32_t>(lo >> 32);
  packed[2] = static_cast<uint32_t>(hi);
  packed[3] = static_cast<uint32_t>(hi >> 32);
}
// The inputs a fan-out lane's player feeds its branch frames base .. base+7
// (confirmed ones from the ring, the repeat-last prediction past the last
// added frame), all loaded before the frame loop: inside it each frame's ring
// read would wait a global-memory round trip on the dependent chain.
constexpr int kFanPre = 8;
template <class R>
__device__ __forceinline__ void fan_prefetch(const R& ring, int h, unsigned s, int32_t base, int32_t cur, bool confirmed_all,
                                             int32_t la_h, uint32_t pred, uint32_t (&vin)[kFanPre]) {
  uint32_t raw[kFanPre];
#pragma unroll
  for (int j = 0; j < kFanPre; ++j) raw[j] = ring.get(min(base + j, max(cur - 1, base)), h, s);
#pragma unroll
  for (int j = 0; j < kFanPre; ++j) {
    const int32_t f = base + j;
    vin[j] = (confirmed_all || (la_h != kNullFrame && f <= la_h)) ? raw[j] : pred;
  }
}
// the prefetched window as 8 bytes: input of frame base + j = byte j (1-byte inputs)
__device__ __forceinline__ uint64_t fan_pack(const uint32_t (&vin)[kFanPre]) {
  uint64_t x = 0;
#pragma unroll
  for (int j = 0; j < kFanPre; ++j) x |= static_cast<uint64_t>(vin[j] & 0xFFu) << (8 * j);
  return x;
}
__device__ __forceinline__ uint32_t fan_input(uint64_t packed, int j) {
  return static_cast<uint32_t>(packed >> (8 * j)) & 0xFFu;
}
// The slot of candidate value v among the first K packed candidates, or -1:
// a zero-byte search over (packed ^ v in every byte) (the lowest zero byte
// of x is the lowest set bit of (x - 0x01..) & ~x & 0x80..).
__device__ __forceinline__ int32_t cand_find(const uint32_t (&packed)[4], uint32_t v, int K) {
  const uint64_t rep = 0x0101010101010101ull * (v & 0xFFu);
  const uint64_t lo = (static_cast<uint64_t>(packed[1]) << 32 | packed[0]) ^ rep;
  const uint64_t hi = (static_cast<uint64_t>(packed[3]) << 32 | packed[2]) ^ rep;
  const uint64_t zl = (lo - 0x0101010101010101ull) & ~lo & 0x8080808080808080ull;
  const uint64_t zh = (hi - 0x0101010101010101ull) & ~hi & 0x8080808080808080ull;
  const int32_t i = zl ? static_cast<int32_t>(__builtin_ctzll(zl) >> 3)
                       : (zh ? 8 + static_cast<int32_t>(__builtin_ctzll(zh) >> 3) : kSpecBranches);
  return (i < K && v <= 0xFFu) ? i : -1;
}
__device__ __forceinline__ uint32_t cand_at(const uint32_t (&packed)[4], int k) {
  uint32_t w = packed[0];
#pragma unroll
  for (int q = 1; q < 4; ++q) w = (k >> 2) == q ? packed[q] : w;
  return (w >> (8 * (k & 3))) & 0xFFu;
}

// Inputs that act identically on a player's own state (G::canon_input: the
// game's representative of each class), else every input its own class.  The
// in-kernel fan-out presimulates one branch per class of its candidates: two
// candidates of one class give bit-identical trajectories (ex_game's
// State::advance reads only up != down, up, left != right and left,
// ex_game.rs:281-296), so a held input selects its class's branch.
template <class G, class = void>
struct InputCanon {
  static constexpr bool value = false;
  __host__ __device__ static constexpr uint32_t apply(uint32_t v) { return v; }
};
template <class G>
struct InputCanon<G, std::void_t<decltype(G::canon_input(0u))>> {
  static constexpr bool value = true;
  __host__ __device__ static constexpr uint32_t apply(uint32_t v) { return G::canon_input(v); }
};
// The distinct classes of a whole alphabet of at most kSpecBranches values, in
// value order, packed like the candidates (0xFF: unused), and their count.
template <class G>
struct AlphabetClasses {
  struct T {
    uint32_t packed[4];
    int n;
  };
  static constexpr T make() {
    T t{{~0u, ~0u, ~0u, ~0u}, 0};
    constexpr uint32_t A = InputAlphabet<G>::value;
    for (uint32_t v = 0; v < A && v < static_cast<uint32_t>(kSpecBranches); ++v) {
      const uint32_t c = InputCanon<G>::apply(v) & 0xFFu;
      bool seen = false;
      for (int i = 0; i < t.n; ++i) seen = seen || ((t.packed[i >> 2] >> (8 * (i & 3))) & 0xFFu) == c;
      if (!seen) {
        t.packed[t.n >> 2] = (t.packed[t.n >> 2] & ~(0xFFu << (8 * (t.n & 3)))) | (c << (8 * (t.n & 3)));
        ++t.n;
      }
    }
    return t;
  }
  static constexpr T value = make();
};
// The index of class value c in an AlphabetClasses list (-1: absent), at compile time
template <class T>
__host__ __device__ constexpr int class_slot(const T& t, uint32_t c) {
  for (int i = 0; i < t.n; ++i)
    if (((t.packed[i >> 2] >> (8 * (i & 3))) & 0xFFu) == c) return i;
  return -1;
}
// The values v < 64 that represent their class (canon(v) == v): what the fill of a class list
// may add (every value for a game without classes).
template <class G>
constexpr uint64_t canon_reps() {
  uint64_t m = 0;
  for (uint32_t v = 0; v < 64; ++v) m |= (InputCanon<G>::apply(v) == v) ? 1ull << v : 0ull;
  return m;
}

// ---------------------------------------------------------------------------
// Desync detection (p2p_session.rs:154-157, 313-316, 873-928; the UdpProtocol
// side: protocol.rs:27, 176-178, 710-742).  Per session, all of it touched
// only by the session's lead lane and only on ticks where current_frame %
// interval == 0 (DesyncDetection::On{interval}):
//   lh   local_checksum_history  HashMap<Frame, u128>: unordered slots, NULL_FRAME = empty
//   rh   per remote handle, UdpProtocol::checksum_history: a FIFO — on_checksum_report
//        only inserts frames above last_added_checksum_frame, so insertion order is
//        frame order and its retain (frame > last_added - 32) pops from the front
//   ob   the ChecksumReports sent since the last rb_p2p_take_checksum_reports (ring)
//   ev   GGRSEvent::DesyncDetected{frame, local, remote, addr} (ring of the newest)
// Both histories hold at most MAX_CHECKSUM_HISTORY_SIZE + 1 = 33 entries at
// any time (the retain runs once the map has more than 32).
constexpr int32_t kMaxChecksumHistory = 32;  // protocol.rs:27 MAX_CHECKSUM_HISTORY_SIZE
constexpr int kCsHist = 34;
constexpr int kOutbox = 8;   // = RB_P2P_REPORTS_PER_TAKE
constexpr int kEvents = 16;  // = RB_P2P_EVENTS_KEPT
struct DesyncParams {
  int32_t* lh_frame;  // [kCsHist][Spad]
  uint64_t* lh_cs;    // [kCsHist][Spad]
  int32_t* rh_frame;  // [4][kCsHist][Spad] FIFO ring per remote handle
  uint64_t* rh_lo;    // [4][kCsHist][Spad]
  uint64_t* rh_hi;    // [4][kCsHist][Spad]
  int32_t* rh_meta;   // [4][3][Spad]: head, length, last_added_checksum_frame
  int32_t* ob_frame;  // [kOutbox][Spad]
  uint64_t* ob_cs;    // [kOutbox][Spad]
  uint32_t* ob_n;     // [Spad] reports sent since the last take
  uint32_t* ev_n;     // [Spad] DesyncDetected events since create
  int32_t* ev_frame;  // [kEvents][Spad] ring, slot = event index % kEvents
  int32_t* ev_handle;
  uint64_t* ev_local;
  uint64_t* ev_remote;
  int32_t interval;   // 0 = DesyncDetection::Off
};

// Peers' connect-status reports (UdpProtocol::peer_connect_status,
// protocol.rs:158-160, 627-636) for update_player_disconnects
// (p2p_session.rs:707-742): what the peer behind remote handle e last reported
// about player i, merged by rb_p2p_receive_peer_connect_status.
struct PeerParams {
  int32_t* last;  // [4 endpoints][4 players][Spad] ConnectionStatus::last_frame
  int32_t* disc;  // [4][4][Spad] ConnectionStatus::disconnected (0 / 1)
  int32_t on;     // RB_P2P_FLAG_PEER_STATUS
};

struct P2PParams {
  uint32_t* snap;
  void* cs;
  int32_t* tag;
  void* ring;
  uint32_t* live;
  int32_t* qs;
  int32_t* status;          // [Spad] rb_status of the session's last advance_frame
  int32_t* trace;           // [Spad] trace_pack words
  uint32_t* counters;       // [0] threshold hits, [1] unexpected-path count, [2] panics
  // work counters [ST_COUNT][Spad]: a wave's sum at its first session's column (or per session,
  // see the end of p2p_kernel); only their sums are read
  unsigned long long* stats;
  // speculative fan-out (spec_on = 0: plain P2P).  fanout_kernel (below, a
  // launch of its own between one-tick P2P launches): branch-major columns
  // (s * kSpecBranches + k) * L + lane, so one session's 16 branches x L lanes
  // store 64 consecutive words per plane.  The in-kernel fan-out (kInFan),
  // the speculated player's words only: branch k in plane k / L at column
  // (k / L) * Spad * L + s * L + lane (the lane that runs it), the other
  // players' own chains at Spad * 16 + s * L + lane (planes Spad * (16 + L)
  // wide); the per-player form: class k of lane l's player at k * Spad * L +
  // s * L + l, a local player's chain at 16 * Spad * L + s * L + l (planes
  // Spad * L * 17 wide).  Every chain slot of a wave stores 64 consecutive words.
  uint32_t* spec_state;  // [NW planes][Spad*16*L] branch states at meta end
  uint32_t* spec_cells;  // [W][NW planes][Spad*16*L] branch cells
  const void* spec_cs;   // [W][Spad][16] CS (fanout_kernel)
  int32_t* spec_meta;    // [SM_COUNT][Spad]
  int32_t spec_on;
  int32_t spec_per_player;  // the in-kernel fan-out speculates every remote player (RB_P2P_FLAG_FANOUT_PER_PLAYER)
  int32_t fan_generic;  // the branches come from fanout_kernel (RB_FANOUT_GENERIC=1, or a game without kInFan)
  int32_t fan_k;        // candidates (branches) per session, <= kSpecBranches
  const uint8_t* local_in;  // tick t, handle h: local_in + t * local_stride + (h * S + s) * IB
  int64_t local_stride;
  const int32_t* upto;      // tick t, handle h: upto[t * upto_stride + h * S + s]
  int64_t upto_stride;
  const uint8_t* remote_in;  // frame f, handle h: remote_in + ((f * P + h) * S + s) * IB
  int32_t remote_frames;
  int32_t S, Spad, W, delay, remote_delay, T;
  uint32_t local_mask;
  int32_t sparse;
  int32_t sync_ticks;  // 1: lock-step ticks on the plain path too (no kAsync; A/B and tests)
  int32_t many_waves;  // the batch puts more than two waves on a SIMD of this device (launch_p2p_as_m)
  DesyncParams ds;
  PeerParams peer;
  // kWire (rb_p2p_run_ticks_packets): the remote inputs arrive as the peers'
  // input packets (wire.hip's format), decoded inside the tick instead of the
  // delivery tensors above.  Tick t, remote handle h, session s: the packet at
  // packets + ((t * P + h) * S + s) * packet_stride, its length and start frame
  // at pk_len / pk_start[(t * P + h) * S + s].
  const uint8_t* packets;
  int64_t packet_stride;
  const int32_t* pk_len;
  const int32_t* pk_start;
  int32_t* pk_status;  // [P][S] the last tick's decode status per endpoint (wire.hip codes), or null
  int32_t* acks;       // [P][S] after the launch: the newest frame received per endpoint (the ack), or null
  unsigned long long* launch_clock;  // rb_p2p_launch_clock_arm: this launch's [waves][start, end], or null
};

// The cells as check_checksum_send_interval sees them.  It runs inside
// advance_frame, before the user executes the requests that advance_frame
// returns, so the cell it reads (frame last_saved_frame - 1) carries what the
// requests of EARLIER ticks saved, not this tick's rollback saves.  The
// device executes a tick's saves as it goes, so the lead lane snapshots the
// cells the send can read before the tick's rollback: the frame saved last is
// the current frame, the confirmed frame (sparse adjust) or the previous
// last saved frame, so frame_to_send is one of those minus one.
struct CellSnap {
  int32_t frame[3], tag[3];
  uint64_t cs[3];
};
template <class CS>
__device__ __forceinline__ CellSnap snap_send_cells(const CS* __restrict__ cs, const int32_t* __restrict__ tag, unsigned s,
                                                    unsigned Spad, int32_t W, int32_t cur, int32_t confirmed,
                                                    int32_t last_saved) {
  CellSnap c;
  const int32_t f[3] = {cur - 1, confirmed - 1, last_saved - 1};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    c.frame[k] = f[k];
    const unsigned slot = static_cast<unsigned>(f[k] >= 0 ? f[k] % W : 0);
    c.tag[k] = f[k] >= 0 ? tag[slot * Spad + s] : kNullFrame;
    c.cs[k] = to_u128(cs[slot * Spad + s]).lo;  // P2P games' checksums are < 2^64
  }
  return c;
}

// check_checksum_send_interval + compare_local_checksums_against_peers
// (p2p_session.rs:873-928) for session s at current frame `cur`, after
// set_last_confirmed_frame (:306-316).  Lead lane only.  Returns false when the
// reference would panic ("cell not found!", :907-910).  The compare walks the
// remote handles in ascending order and each history in frame order (the
// reference iterates HashMaps; the order of its events is unspecified).
__device__ __noinline__ bool desync_step(const DesyncParams& d, const CellSnap& cells, unsigned s, unsigned Spad,
                                         int32_t cur, int32_t last_saved, int32_t W, int P, uint32_t local_mask) {
  if (cur % d.interval != 0) return true;  // both steps act on interval frames only
  auto at = [&](int k) { return static_cast<size_t>(k) * Spad + s; };
  int32_t lf[kCsHist];
#pragma unroll
  for (int k = 0; k < kCsHist; ++k) lf[k] = d.lh_frame[at(k)];
  const int32_t frame_to_send = last_saved - 1;
  if (frame_to_send > W) {
    int ci = -1;
#pragma unroll
    for (int k = 2; k >= 0; --k) ci = cells.frame[k] == frame_to_send ? k : ci;
    if (ci < 0) return false;  // cannot happen (see CellSnap)
    const int32_t ctag = ci == 0 ? cells.tag[0] : (ci == 1 ? cells.tag[1] : cells.tag[2]);
    if (ctag != frame_to_send) return false;  // saved_state_by_frame(..).unwrap_or_else(panic)
    const uint64_t c = ci == 0 ? cells.cs[0] : (ci == 1 ? cells.cs[1] : cells.cs[2]);
    const uint32_t n = d.ob_n[s];  // send_checksum_report to every remote endpoint
    d.ob_frame[at(static_cast<int>(n % kOutbox))] = frame_to_send;
    d.ob_cs[at(static_cast<int>(n % kOutbox))] = c;
    d.ob_n[s] = n + 1;
    int slot_of = -1, empty = -1;  // local_checksum_history.insert(frame_to_send, checksum)
#pragma unroll
    for (int k = kCsHist - 1; k >= 0; --k) {
      slot_of = lf[k] == frame_to_send ? k : slot_of;
      empty = lf[k] == kNullFrame ? k : empty;
    }
    const int k = slot_of >= 0 ? slot_of : empty;
    if (k < 0) return false;  // cannot happen: at most 33 entries
    d.lh_frame[at(k)] = frame_to_send;
    d.lh_cs[at(k)] = c;
#pragma unroll
    for (int j = 0; j < kCsHist; ++j) lf[j] = j == k ? frame_to_send : lf[j];
  }
  int len = 0;
#pragma unroll
  for (int k = 0; k < kCsHist; ++k) len += lf[k] != kNullFrame;
  if (len > kMaxChecksumHistory) {  // retain(|&frame, _| frame > current - MAX_CHECKSUM_HISTORY_SIZE)
#pragma unroll
    for (int k = 0; k < kCsHist; ++k)
      if (lf[k] != kNullFrame && lf[k] <= cur - kMaxChecksumHistory) {
        lf[k] = kNullFrame;
        d.lh_frame[at(k)] = kNullFrame;
      }
  }
  for (int h = 0; h < P; ++h) {  // compare_local_checksums_against_peers
    if ((local_mask >> h) & 1u) continue;
    const size_t m = static_cast<size_t>(h) * 3;
    const int head = d.rh_meta[at(static_cast<int>(m))], n = d.rh_meta[at(static_cast<int>(m + 1))];
    for (int i = 0; i < n; ++i) {
      const size_t r = static_cast<size_t>(h) * kCsHist + static_cast<size_t>((head + i) % kCsHist);
      const int32_t rf = d.rh_frame[at(static_cast<int>(r))];
      int li = -1;
#pragma unroll
      for (int k = 0; k < kCsHist; ++k) li = lf[k] == rf ? k : li;
      if (li < 0) continue;
      const uint64_t lc = d.lh_cs[at(li)], rlo = d.rh_lo[at(static_cast<int>(r))];
      const uint64_t rhi = d.rh_hi[at(static_cast<int>(r))];
      if (lc != rlo || rhi != 0) {  // local u128 checksums are < 2^64 for every P2P game
        const uint32_t e = d.ev_n[s];
        const int q = static_cast<int>(e % kEvents);
        d.ev_frame[at(q)] = rf;
        d.ev_handle[at(q)] = h;
        d.ev_local[at(q)] = lc;
        d.ev_remote[at(q)] = rlo;
        d.ev_n[s] = e + 1;
      }
    }
  }
  return true;
}


// Lane-group reductions over groups of L consecutive lanes (1, 2, 4 or 64).
template <int L>
__device__ __forceinline__ int32_t group_min(int32_t v) {
  if constexpr (L == 64) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = min(v, __shfl_xor(v, m, 64));
  } else {
    if constexpr (L >= 2) v = min(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    if constexpr (L >= 4) v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  }
  return v;
}

// One InputQueue (input_queue.rs) in registers; the inputs live in the ring
// (HBM, or LDS inside a launch).  `tail` is the frame of inputs[tail] and
// `len` the queue's length, restated exactly: every queue's first input is
// frame 0 (the delay fill, :227-231) and inputs are added in frame order, so
// ring slot k holds the newest frame <= last_added congruent to k mod 128 (or
// none), which is all the reference's index arithmetic ever reads.  A frame is
// Confirmed iff 0 <= f - tail < len (:118-127); for a connected player that is
// f <= last_added.  `bad` records a reference assert / checked-arithmetic
// panic inside a tick: input() below the tail (:113) and a discard that
// would take `length` below zero (:99, a subtract-with-overflow panic in the
// reference's test builds); the kernel folds it into the tick's status.
struct DevQueue {
  int32_t last_added, pred_frame, first_inc, last_req, conn_last;
  uint32_t pred_val;
  bool disc;  // ConnectionStatus::disconnected: rb_p2p_disconnect_player, or peers' reports (kNet)
  bool bad;
  int32_t tail, len;
  // the fan-out's move-to-front list of the most recent distinct inputs (fan_candidates), kept
  // only by fan-out batches whose alphabet is larger than K (mtf); bytes 0-7 / 8-15 newest first.
  // mcanon: the list holds input classes (InputCanon), for the in-kernel fan-out, whose branches
  // are classes: K recent classes cover more of the moves than K recent raw inputs
  bool mtf, mcanon;
  uint64_t mlo, mhi;
  int32_t mn;
};
// Input v (1 byte) to the front of the queue's list: removed where it was, or the
// entry past the list's end (the oldest of a full list) dropped, the entries
// before it moved back one place.
__device__ __forceinline__ void mtf_push(DevQueue& q, uint32_t v) {
  v &= 0xFFu;
  const uint64_t rep = 0x0101010101010101ull * v;
  const uint64_t xl = q.mlo ^ rep, xh = q.mhi ^ rep;
  const uint64_t zl = (xl - 0x0101010101010101ull) & ~xl & 0x8080808080808080ull;  // lowest zero byte: exact
  const uint64_t zh = (xh - 0x0101010101010101ull) & ~xh & 0x8080808080808080ull;
  int i = zl ? static_cast<int>(__builtin_ctzll(zl) >> 3) : (zh ? 8 + static_cast<int>(__builtin_ctzll(zh) >> 3) : 16);
  if (i >= q.mn) {  // not in the list
    i = min(q.mn, kSpecBranches - 1);
    q.mn = min(q.mn + 1, kSpecBranches);
  }
  const int nb = i + 1;  // bytes 0 .. i are rewritten: byte 0 = v, bytes 1 .. i = the old bytes 0 .. i-1
  const uint64_t klo = nb >= 8 ? 0ull : (~0ull << (8 * nb));
  const uint64_t khi = nb <= 8 ? ~0ull : (nb >= 16 ? 0ull : (~0ull << (8 * (nb - 8))));
  const uint64_t slo = q.mlo << 8, shi = (q.mhi << 8) | (q.mlo >> 56);
  q.mlo = (q.mlo & klo) | (slo & ~klo) | v;
  q.mhi = (q.mhi & khi) | (shi & ~khi);
}
// input_queue.rs:181 assert!(self.length <= INPUT_QUEUE_LENGTH): a caller of
// the batch trips it by delivering remote inputs more than 128 frames past the
// frames the session has discarded.  length only grows in add_input_by_frame,
// so after a poll it is above 128 iff the assert fired during the poll.
__device__ __forceinline__ bool q_overflow(const DevQueue& q) { return q.len > kQueueLen; }

template <int IB>
struct RingIO {
  uint8_t* ring;
  int P, Spad;
  __device__ __forceinline__ uint32_t get(int32_t f, int h, unsigned s) const {
    const size_t i = (static_cast<size_t>(f & (kQueueLen - 1)) * P + h) * Spad + s;
    if constexpr (IB == 4) return reinterpret_cast<const uint32_t*>(ring)[i];
    else return ring[i];
  }
  __device__ __forceinline__ void put(int32_t f, int h, unsigned s, uint32_t v) const {
    const size_t i = (static_cast<size_t>(f & (kQueueLen - 1)) * P + h) * Spad + s;
    if constexpr (IB == 4) reinterpret_cast<uint32_t*>(ring)[i] = v;
    else ring[i] = static_cast<uint8_t>(v);
  }
};

// The same ring in LDS, for a kernel whose lanes own one player each
// (p2p_lds_queue below): column = thread, row = frame % 128.  p2p_kernel
// copies in the HBM frames a launch can read and writes back the frames it
// adds.  Inside the launch an input read is an LDS read: LDS has its own
// counter, so it never waits for the tick's snapshot stores the way a global
// load issued after them does (vmcnt retires loads and stores in order).
struct LdsRing {
  uint8_t* col;       // this thread's column: lds + threadIdx.x
  unsigned row;       // bytes per frame row (blockDim.x)
  __device__ uint32_t get(int32_t f, int, unsigned) const { return col[static_cast<unsigned>(f & (kQueueLen - 1)) * row]; }
  __device__ void put(int32_t f, int, unsigned, uint32_t v) const {
    col[static_cast<unsigned>(f & (kQueueLen - 1)) * row] = static_cast<uint8_t>(v);
  }
};
// LDS queues: 1-byte inputs, one player per lane (ex_game lane per player, the brawler).
template <class G>
constexpr bool p2p_lds_queue() {
  return G::kInputBytes == 1 && (G::kLanes > 1 || G::kPlayers == 1);
}
// ... in a launch whose snapshot ring is (kLdsC) or is not in LDS.  Launches of
// few ticks keep the snapshot ring in HBM, and the input ring too: filling the
// LDS copy (byte loads in dependent rounds) and writing it back cost more than
// the handful of ring reads a short launch makes (measured, one tick per
// launch at 65,536 sessions: 14.8 -> 13.1 us, the packet-fed tick 18.9 -> 16.7).
#ifndef RB_SHORT_HBM_RING
#define RB_SHORT_HBM_RING 1  // 0: the LDS input ring in every launch (A/B builds)
#endif
template <class G, bool kLdsC>
constexpr bool p2p_lds_queue_in() {
  return p2p_lds_queue<G>() && (kLdsC || !RB_SHORT_HBM_RING);
}
template <class G, bool kLdsC = false>
constexpr size_t p2p_lds_bytes(int block) {
  return p2p_lds_queue_in<G, kLdsC>() ? static_cast<size_t>(kQueueLen) * static_cast<size_t>(block) : 0;
}
// The snapshot ring in LDS (p2p_kernel kLdsC): for the launch, the W cells
// (words [W][NWL][block], frame tags and checksums [W][block / kLanes]) live
// after the queue in LDS; the launch loads them from HBM first and writes
// them back last.  Every SaveGameState and LoadGameState inside is an LDS
// access, and the tick loop issues no global store at all: CDNA's vmcnt
// retires loads and stores in issue order, so with a tick's snapshot stores
// in flight, waiting for the next tick's prefetched deliveries would wait for
// the stores too (the compiler cannot count stores issued in a loop of
// data-dependent length and drains the counter).  Up to kLdsCellsMaxW cells:
// at W = 8, 512 threads per CU (two waves per SIMD) take 156 KiB of the 160.
constexpr int kLdsCellsMaxW = 8;
template <class G>
constexpr size_t p2p_lds_cell_bytes(int block, int W) {
  return static_cast<size_t>(W) * (static_cast<size_t>(G::NWL) * 4 * block +
                                   (4 + sizeof(typename G::CS)) * static_cast<size_t>(block / G::kLanes));
}
// ... when the queue and the cells of a block fit half of a CU's 160 KiB (two
// blocks per CU): ex_game's 40 B cells do (79 KiB at 256 threads, W = 8), the
// brawler's 8 KiB cells do not and stay in HBM.
constexpr size_t kLdsPerBlockMax = 80 * 1024;
#ifndef RB_LDS_CELLS_MIN_TICKS
#define RB_LDS_CELLS_MIN_TICKS 24
#endif
// launches of fewer ticks keep the cells in HBM (and lock-step ticks): copying the
// ring in and out costs more than it saves below about 24 ticks (measured: HBM
// cells 4.8 us per tick at 16 ticks per launch, LDS cells 4.1 at 32)
constexpr int kLdsCellsMinTicks = RB_LDS_CELLS_MIN_TICKS;
// Launches of kLdsQMinTicks up to kLdsCellsMinTicks ticks keep the cells in HBM but the input ring
// in LDS (p2p_kernel kQ; plain path and sparse saving, ex_game's lane-per-player layout).  Measured
// at 65,536 sessions, us per tick (HBM ring / LDS ring / LDS cells): 2 ticks per launch 7.6 / 8.0 /
// 12.7, 4: 6.34 / 6.08 / 8.44, 8: 5.57 / 5.02 / 5.97, 16: 5.07 / 4.36 / 4.55 (round 4, interleaved A/B, tools/ab.py).
#ifndef RB_LDSQ_MIN_TICKS
#define RB_LDSQ_MIN_TICKS 4
#endif
constexpr int kLdsQMinTicks = RB_LDSQ_MIN_TICKS;
template <class G>
constexpr bool p2p_lds_cells(int W, int block) {
  return p2p_lds_queue<G>() && W <= kLdsCellsMaxW &&
         p2p_lds_bytes<G, true>(block) + p2p_lds_cell_bytes<G>(block, W) <= kLdsPerBlockMax;
}

// input_queue.rs:167-204 add_input_by_frame (Cn: the game's InputCanon, for the fan-out's list)
template <class Cn, class R>
__device__ __forceinline__ void q_add_by_frame(DevQueue& q, const R& r, int h, unsigned s, int32_t f, uint32_t v) {
  r.put(f, h, s, v);
  if (q.mtf) mtf_push(q, q.mcanon ? Cn::apply(v) : v);
  q.last_added = f;
  q.len += 1;
  // the prediction bookkeeping as selects (no branch: every call site is in the hot poll)
  const bool pr = q.pred_frame != kNullFrame;
  q.first_inc = (pr && q.first_inc == kNullFrame && v != q.pred_val) ? f : q.first_inc;
  const bool done = q.pred_frame == q.last_req && q.first_inc == kNullFrame;
  q.pred_frame = pr ? (done ? kNullFrame : q.pred_frame + 1) : q.pred_frame;
}
// input_queue.rs:149-163 + 207-239 add_input with the delay already applied to
// `f`: replicate the entry before head (blank before the first add) up to f.
template <class Cn, class R>
__device__ __forceinline__ int32_t q_add(DevQueue& q, const R& r, int h, unsigned s, int32_t f, uint32_t v) {
  int32_t expected = q.last_added == kNullFrame ? 0 : q.last_added + 1;
  if (expected > f) return kNullFrame;
  if (expected < f) {  // only a queue's first add replicates (the input-delay fill)
    const uint32_t rep = q.last_added == kNullFrame ? 0u : r.get(q.last_added, h, s);
    for (; expected < f; ++expected) q_add_by_frame<Cn>(q, r, h, s, expected, rep);
  }
  q_add_by_frame<Cn>(q, r, h, s, f, v);
  return f;
}
// input_queue.rs:83-101 discard_confirmed_frames(frame).  "Delete all but the
// most recent" sets tail = head, whose slot holds last_added - 127 (nothing, a
// NULL frame, before 127 frames were added) and length 1; only a disconnected
// player reaches it (the confirmed frame skips it), and from then on its
// queue answers Predicted for the frames it still holds (:118-142).
__device__ __forceinline__ void q_discard(DevQueue& q, int32_t frame) {
  if (q.last_req != kNullFrame) frame = min(frame, q.last_req);
  if (frame >= q.last_added) {
    q.tail = max(q.last_added - (kQueueLen - 1), kNullFrame);
    q.len = 1;
  } else if (frame > q.tail) {
    const int32_t off = frame - q.tail;
    q.bad |= off > q.len;  // `self.length -= offset` would underflow
    q.len -= off;
    // tail moves `off` slots: onto frame `frame`, except from a NULL head slot
    // (fewer than 127 frames added), where slot last_added + 2 holds frame 0
    // only if last_added == 126
    q.tail = (q.tail == kNullFrame && q.last_added != kQueueLen - 2) ? kNullFrame : frame;
  }
}
// input_queue.rs:104-146 input(requested_frame).  kSel: the same decisions as selects around one
// ring read (the confirmed frame's entry, or the last added one a new prediction repeats; an unused
// read of a valid slot otherwise), with no divergent branch and so no exec-mask bookkeeping in every
// AdvanceFrame's input fetch.  Measured (interleaved A/B, profiles/r05_ab_qsel.log): one-tick
// launches 11.20 -> 10.44 us of wall per tick, 50-tick launches 3.48 -> 3.43 us; with sparse saving
// 9.70 -> 10.27 us, so the sparse kernels keep the branches.
// Attribution builds (tools/mkvar.sh -DRB_P2P_EXP=...): 1 drops the game's
// AdvanceFrame math, 2 its save checksum, 32 returns at entry (the launch
// floor), 64 drops the trace rows and work counters, 128 the sparse dry run, 256
// every input-ring read of InputQueue::input (and with it every prediction, so no
// session rolls back: the rollback work).  Always 0 in the product.
#ifndef RB_P2P_EXP
#define RB_P2P_EXP 0
#endif
template <bool kSel, class R>
__device__ __forceinline__ uint32_t q_input(DevQueue& q, const R& r, int h, unsigned s, int32_t f) {
  q.last_req = f;
  if constexpr ((RB_P2P_EXP & 256) != 0) return q.pred_val;  // (attribution builds only: no ring read)
  q.bad |= f < q.tail;  // assert!(requested_frame >= self.inputs[self.tail].frame) (:113)
  if constexpr (kSel) {
    const bool np = q.pred_frame < 0;
    const bool conf = np && f - q.tail < q.len;               // Confirmed (:118-127)
    const bool blank = f == 0 || q.last_added == kNullFrame;  // blank_input
    const uint32_t rv = r.get(conf ? f : q.last_added, h, s);
    const bool newpred = np && !conf;
    q.pred_val = newpred ? (blank ? 0u : rv) : q.pred_val;
    q.pred_frame = newpred ? (blank ? 0 : q.last_added + 1) : q.pred_frame;  // (0: NULL_FRAME + 1)
    return conf ? rv : q.pred_val;
  }
  if (q.pred_frame < 0) {
    if (f - q.tail < q.len) return r.get(f, h, s);  // Confirmed (:118-127)
    if (f == 0 || q.last_added == kNullFrame) {
      q.pred_val = 0u;  // blank_input
      q.pred_frame = 0;  // NULL_FRAME + 1
    } else {
      q.pred_val = r.get(q.last_added, h, s);
      q.pred_frame = q.last_added + 1;
    }
  }
  return q.pred_val;  // Predicted
}

// The in-kernel fan-out (p2p_kernel kSpec, kInFan).  For a game whose players
// move independently (G::kIndependentPlayers: every player's state follows from
// its own inputs alone, ex_game.rs:259-321) and that reads no input status, the
// 16 branches of a session differ only in the speculated player's words, and
// the other players' words in every branch are those of the main trajectory:
// a select (try_select) is only taken when no other player mispredicted, so
// their cells and states are already what the rollback would compute.  So the
// fan-out simulates the speculated player alone, 16 / L branches in each of
// the session's L lanes (independent chains: ILP), at the end of every tick
// inside p2p_kernel itself; the spec columns are per branch (column
// s * 16 + k, branch k = b * L + lane is owned by lane k % L, which alone
// writes and reads it back: same thread, program order).  A select takes the
// branch's words for the speculated player's column and rebuilds each cell's
// checksum from per-player fletcher parts (the branch's part and the other
// players' parts of their own cell words).  The fan-out running in the tick
// lets a launch hold many ticks (the two-launch fan-out needed one P2P launch
// per tick: every lane of a session's branches ran between ticks).
template <class G>
constexpr bool inlane_fan() {
  if constexpr (IndepPlayers<G>::value) return G::kLanes > 1 && G::kLanes <= 4 && !G::kUsesStatus && G::kInputBytes == 1;
  else return false;
}
#ifndef RB_FAN_GROUP
#define RB_FAN_GROUP 4  // A/B (tools/ab.py, round 4): 3 measured the same at C4 (206 VGPRs, still 2 waves per
#endif                  // SIMD); 3 with a 3-waves cap (168 VGPRs, 160 B spilled) 8% slower
constexpr int kFanGroup = RB_FAN_GROUP;  // chains a lane advances together (independent: instruction-level parallelism)
#ifndef RB_FAN_INRANGE
#define RB_FAN_INRANGE 1  // 0: the fan-out's chains always take the general AdvanceFrame (A/B builds)
#endif
// Attribution builds only (tools/mkvar.sh -DRB_FAN_EXP=...; results are wrong): 1 presimulates no
// branch (every fan-out invalid), 2 stores no branch cell.  Always 0 in the product.
#ifndef RB_FAN_EXP
#define RB_FAN_EXP 0
#endif

// kSpec / kSparse / kNet: the fan-out select, sparse saving and the
// network-fed bookkeeping (desync detection, peers' connect-status reports)
// are compiled in only where the batch uses them (fewer live scalars: no SGPR
// spills on the plain path)
// kAsync (plain path with the LDS snapshot ring only): lane-asynchronous
// ticks.  Every loop iteration a session executes exactly one AdvanceFrame:
// a resimulated frame of its current rollback ([SaveGameState], its
// synchronized_inputs, AdvanceFrame), or, once its rollback is done, the rest
// of the tick (set_last_confirmed_frame, add_local_input, SaveGameState of
// the current frame) and the tick's new frame.  A session starting a tick
// first runs the tick's opening (poll, PredictionThreshold, the rollback
// decision, LoadGameState) in the same iteration.  A wave then iterates max
// over its sessions of the frames each executes in the launch, instead of the
// sum over ticks of its deepest rollback (every per-frame step of the
// rollback, the InputQueue reads included, rides in the same iteration): one
// session's rollback no longer holds up the other 31.  Each session's own
// operations run in the reference's order, except that the tick's final
// SaveGameState moves behind set_last_confirmed_frame and add_local_input,
// which touch neither the state nor the cells.
#ifndef RB_P2P_ONE_WAVES
#define RB_P2P_ONE_WAVES 4  // waves per SIMD the one-tick kernels (kOne) are compiled for
#endif
#ifndef RB_P2P_SHORT_WAVES
#define RB_P2P_SHORT_WAVES 4  // waves per SIMD the short-launch kernels (kQ, one-tick) are compiled for (A/B builds)
#endif
#ifndef RB_P2P_WAVES_PER_EU
#define RB_P2P_WAVES_PER_EU 1  // >1: ask the compiler for that many waves per SIMD (VGPR cap; A/B builds)
#endif
// RB_SPEC_Q: the in-kernel fan-out of a batch with more than two waves per SIMD keeps its cells in HBM
// and only the input ring in LDS (kQ), capped at RB_SPEC_Q_WAVES waves per SIMD, instead of the LDS
// snapshot ring's two workgroups per CU
#ifndef RB_SPEC_Q
#define RB_SPEC_Q 0
#endif
#ifndef RB_SPEC_Q_WAVES
#define RB_SPEC_Q_WAVES 3
#endif
// kMtf (fan-out batches only): the candidates come from the queues' move-to-front lists, for an
// alphabet larger than K; otherwise (ex_game at K = 16) they are the alphabet itself, and the lists
// are neither kept nor read (no registers held for them).
// RB_P2P_PHASE (A/B builds, tools/p2p_phase.py): one-tick launches record, per wave, the
// constant-rate clock (100 MHz) at entry, once the state loads are in, after the poll and
// threshold decision, after the rollback and saves, after the tick's own frame, and at the end.
// Measured at 65,536 sessions (p50 / p90 us): state loads 1.28 / 1.52, poll + threshold 1.44 /
// 1.60, rollback + saves 2.40 / 3.16, the tick's frame 0.84 / 1.00, epilogue 0.76 / 0.92; first
// entry to last end 8.6 of the launch's 10.4.  Fetching the likely rollback cell with the first
// deliveries (one round trip fewer) cut the rollback phase to 2.16 but not the launch (A/B,
// dropped); so did the LDS input ring (11.7-12.5 against 10.4-11.0 us one-tick, but 5.0 against
// 5.6 us per tick in 8-tick launches).
#ifndef RB_P2P_PHASE
#define RB_P2P_PHASE 0
#endif
#if RB_P2P_PHASE
__device__ uint64_t rb_p2p_phase[8 * 4096];
#define RB_PH(i)                                                    \
  do {                                                              \
    if (p.T == 1) ph[i] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#else
#define RB_PH(i) \
  do {           \
  } while (0)
#endif
template <class G, bool kSpec, bool kSparse, bool kNet, bool kLdsC, bool kAsync, bool kWire = false, bool kMtf = false,
          bool kQ = false, bool kOne = false>
// kQ (the input ring alone in LDS, 32 KiB per 256 threads) is capped at 128 VGPRs: with the cells in
// HBM four workgroups fit a CU, so batches of more than two waves per SIMD run four resident instead
// of the LDS-cell kernel's two (kernels.hpp launch_p2p_as_m).
// The launches that keep the cells in HBM on the plain / sparse path (kQ, and the one-tick launches
// of live play) are capped at 128 VGPRs the same way: four waves per SIMD once a batch has them.
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(kOne ? RB_P2P_ONE_WAVES : (kQ && kSpec) ? RB_SPEC_Q_WAVES : (kQ || (!kLdsC && !kSpec && !kNet)) ? RB_P2P_SHORT_WAVES : RB_P2P_WAVES_PER_EU)))
p2p_kernel(const P2PParams p) {
  static_assert(!kAsync || (kLdsC && !kSpec && !kNet), "lane-asynchronous ticks: plain or sparse path, LDS cells");
  static_assert(!kWire || (!kSpec && !kSparse && !kNet && !kAsync), "packet-fed ticks: the plain lock-step path");
  using InRec = typename G::InRec;
  using CS = typename G::CS;
  constexpr int NW = G::NWL;
  constexpr int L = G::kLanes;
  constexpr int P = G::kPlayers, IB = G::kInputBytes;
  constexpr bool kSplit = L > 1;  // lane h of the group owns player h
  constexpr int PPL = kSplit ? 1 : P;
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned s = g / L;
  const int lane = static_cast<int>(g % L);
  const bool lead = lane == 0;
  // kOne: the launches of one tick (live play), the tick count a compile-time 1, so the tick loop
  // and the next tick's prefetch compile away (kernels.hpp launch_p2p_as_m)
  static_assert(!kOne || (!kLdsC && !kAsync && !kQ), "one-tick launches keep the cells in HBM");
  const int T = kOne ? 1 : p.T;
  if (p.launch_clock) launch_clock_put(p.launch_clock, g / 64u, 0u);
  if (s >= static_cast<unsigned>(p.S)) return;  // whole lane groups leave together
#if RB_P2P_PHASE
  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
#endif
  RB_PH(0);
  // A session that hit a reference assert stays stopped (the reference
  // process would have aborted): it reports RB_PANIC from then on and its
  // state, cells and queues stay as the panic left them.  (Checked once the
  // session's state loads are issued, so they do not wait for this one.)
  if constexpr (RB_P2P_EXP & 32) return;  // (attribution builds only: the launch floor)
  const int32_t status0 = p.status[s];  // (stored back only when the tick changes it)
  const bool panicked = status0 == kP2PStatusPanic;
  const unsigned Spad = static_cast<unsigned>(p.Spad), Gpad = Spad * L;
  const unsigned slot_words = static_cast<unsigned>(NW) * Gpad;
  const int W = p.W;
  CS* __restrict__ csa = reinterpret_cast<CS*>(p.cs);
  constexpr bool kLdsQ = p2p_lds_queue_in<G, kLdsC || kQ>();  // (kQ: the input ring alone, see kLdsQMinTicks)
  const RingIO<IB> hbm{reinterpret_cast<uint8_t*>(p.ring), P, p.Spad};
  extern __shared__ uint8_t lds_queue[];
  const auto ring = [&]() __attribute__((always_inline)) {
    if constexpr (kLdsQ) return LdsRing{lds_queue + threadIdx.x, blockDim.x};
    else return hbm;
  }();
  // the in-kernel fan-out (the batch's branches are this kernel's own unless fan_generic)
  constexpr bool kInFan = kSpec && inlane_fan<G>();
  const bool in_fan = kInFan && !p.fan_generic;
  // The next tick's deliveries are prefetched, except by the P2P launches of
  // the two-launch fan-out (fanout_kernel), which are always of one tick (the
  // fan-out runs between ticks): there they would only hold registers.
  constexpr bool kPrefetch = !kSpec || kInFan;
  static_assert(!kLdsC || (kLdsQ && (!kSpec || kInFan) && !kNet),
                "the LDS snapshot ring needs the LDS queue; fanout_kernel and desync detection read HBM cells mid-launch");
  const unsigned bd = blockDim.x, tid = threadIdx.x, sl = tid / L, bps = bd / L;
  uint32_t* const lds_cell = reinterpret_cast<uint32_t*>(lds_queue + kQueueLen * bd);  // [W][NW][bd]
  int32_t* const lds_tag = reinterpret_cast<int32_t*>(lds_cell + static_cast<unsigned>(W) * NW * bd);  // [W][bps]
  CS* const lds_cs = reinterpret_cast<CS*>(lds_tag + static_cast<unsigned>(W) * bps);  // [W][bps]
  auto qrow = [&](int field, int h) __attribute__((always_inline)) { return p.qs + static_cast<size_t>(QS_PLAYER0 + field * 4 + h) * Spad + s; };
  auto player_of = [&](int j) __attribute__((always_inline)) { return kSplit ? lane : j; };

  int32_t cur = p.qs[QS_CUR * Spad + s];
  // cur % W, kept alongside cur (every SaveGameState is of the current frame):
  // a division by the runtime W costs a dozen VALU instructions
  unsigned cur_slot = static_cast<unsigned>(cur % p.W);
  // the packed bookkeeping (decoded below, once every load of the launch's entry is issued)
  const uint32_t sc_pk = static_cast<uint32_t>(p.qs[QS_SAVED_CONF * Spad + s]);
  int32_t last_saved = kNullFrame, last_conf = kNullFrame;
  DevQueue q[PPL];
  uint32_t qpk[PPL][4];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int h = player_of(j);
    if (h < P) {
#pragma unroll
      for (int i = 0; i < 4; ++i) qpk[j][i] = static_cast<uint32_t>(*qrow(QF_LA_CONN + i, h));
      if constexpr (IB > 1) q[j].pred_val = static_cast<uint32_t>(*qrow(QF_PRED_VAL, h));
      q[j].bad = false;
      // the fan-out's candidate list, for an alphabet larger than K
      q[j].mtf = kSpec && kMtf;
      q[j].mcanon = kSpec && kMtf && InputCanon<G>::value && in_fan;  // the in-kernel fan-out: classes
      if constexpr (kSpec && kMtf) {
        q[j].mlo = static_cast<uint32_t>(*qrow(QF_MTF0, h)) | static_cast<uint64_t>(static_cast<uint32_t>(*qrow(QF_MTF0 + 1, h))) << 32;
        q[j].mhi = static_cast<uint32_t>(*qrow(QF_MTF0 + 2, h)) | static_cast<uint64_t>(static_cast<uint32_t>(*qrow(QF_MTF0 + 3, h))) << 32;
        q[j].mn = *qrow(QF_MTF_N, h);
      }
    } else {  // padding lane of a 4-lane group (P = 3): no player
      q[j] = DevQueue{kNullFrame, kNullFrame, kNullFrame, kNullFrame, INT32_MAX, 0u, false, 0};
#pragma unroll
      for (int i = 0; i < 4; ++i) qpk[j][i] = 0u;
    }
  }
  // disconnect_player between launches: P2PSession::disconnect_frame, consumed
  // by the next advance_frame's check_simulation_consistency (:281-288)
  int32_t disc_frame = p.qs[QS_DISC_FRAME * Spad + s];
  const int32_t disc_frame0 = disc_frame;
  bool any_disc = false;  // (after the decode below)
  // confirmed_frame (:487-498) skips disconnected players
  auto conn_of = [&](int j) __attribute__((always_inline)) { return q[j].disc ? INT32_MAX : q[j].conn_last; };
  uint32_t w[NW];
  load_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);
  // the fan-out's branch metadata (written between launches), with the state loads
  [[maybe_unused]] int32_t sm_valid = 0, sm_end = 0, sm_base = 0, sm_player = 0;
  [[maybe_unused]] uint32_t sm_cand[4] = {0u, 0u, 0u, 0u};
  if constexpr (kSpec) {
    sm_valid = p.spec_meta[SM_VALID * Spad + s];
    sm_end = p.spec_meta[SM_END * Spad + s];
    sm_base = p.spec_meta[SM_BASE * Spad + s];
    sm_player = p.spec_meta[SM_PLAYER * Spad + s];
#pragma unroll
    for (int q = 0; q < 4; ++q) sm_cand[q] = static_cast<uint32_t>(p.spec_meta[(SM_CAND + q) * Spad + s]);
  }
  // per-player fan-out: this lane's player's first unconfirmed frame when its branches were made
  // (row SM_CAND + lane: the candidate rows are free there, the candidates being the whole alphabet)
  [[maybe_unused]] int32_t sm_pbase = 0;
  if constexpr (kInFan && !kMtf) sm_pbase = static_cast<int32_t>(sm_cand[min(lane, 3)]);
  // ---- the per-tick delivery tensors, loaded one tick ahead: at the top of
  // tick t, before its snapshot stores, come the delivered watermark and the
  // local inputs of tick t+1; right after the poll, the first kPre remote
  // frames tick t+1 will add (their frame numbers are known once the poll
  // has moved the connection status).  Every lane loads (clamped, always
  // valid addresses) and uses what its players need: a branch around a load
  // would make the compiler wait for it at the join.
  constexpr int kPre = 4;
  const int first_local = p.local_mask ? __builtin_ctz(p.local_mask) : 0;
  auto load_upto = [&](int t, int j) __attribute__((always_inline)) -> int32_t {
    if constexpr (kWire) return kNullFrame;  // (no delivery tensors: packets)
    const int h = min(player_of(j), P - 1);
    return p.upto[static_cast<int64_t>(t) * p.upto_stride + static_cast<int64_t>(h) * p.S + s];
  };
  auto load_local = [&](int t, int j) __attribute__((always_inline)) -> uint32_t {
    if (!p.local_mask) return 0u;  // launch-uniform
    int h = player_of(j);
    h = (h < P && ((p.local_mask >> h) & 1u)) ? h : first_local;
    const uint8_t* src = p.local_in + static_cast<int64_t>(t) * p.local_stride + (static_cast<size_t>(h) * p.S + s) * IB;
    return IB == 4 ? *reinterpret_cast<const uint32_t*>(src) : *src;
  };
  auto remote_start = [&](int j) __attribute__((always_inline)) {
    return q[j].conn_last == kNullFrame ? p.remote_delay : q[j].conn_last + 1;
  };
  // remote_in[frame][P][S]: a per-lane base and a 32-bit frame stride (P * S * IB < 2^32),
  // so an address is one 32x32->64 multiply-add
  const uint32_t rstride = static_cast<uint32_t>(P) * static_cast<uint32_t>(p.S) * IB;
  const uint8_t* rbase[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j)
    rbase[j] = kWire ? nullptr : p.remote_in + (static_cast<size_t>(min(player_of(j), P - 1)) * p.S + s) * IB;
  auto load_remote = [&](int j, int32_t f) __attribute__((always_inline)) -> uint32_t {
    if constexpr (kWire) return 0u;
    f = max(0, min(f, p.remote_frames - 1));
    const uint8_t* src = rbase[j] + static_cast<uint64_t>(static_cast<uint32_t>(f)) * rstride;
    return IB == 4 ? *reinterpret_cast<const uint32_t*>(src) : *src;
  };
  // the first tick's watermark and local inputs (addresses known at entry: with the state loads)
  int32_t up[PPL];
  uint32_t lin[PPL], rv[PPL][kPre];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    up[j] = load_upto(0, j);
    lin[j] = load_local(0, j);
  }
  // kWire: a tick's packet (length, start frame, first 32 bytes)
  struct PkHead {
    int32_t n, start;
    uint32_t w0[8];
  };
  auto wire_fetch = [&](int h, int t) __attribute__((always_inline)) -> PkHead {
    PkHead r{0, 0, {}};
    const size_t idx = (static_cast<size_t>(t) * P + static_cast<size_t>(h)) * static_cast<size_t>(p.S) + s;
    r.n = p.pk_len[idx];
    r.start = p.pk_start[idx];
    const uint8_t* pk = p.packets + static_cast<int64_t>(idx) * p.packet_stride;
    const uint4 a = reinterpret_cast<const uint4*>(pk)[0], b = reinterpret_cast<const uint4*>(pk)[1];
    r.w0[0] = a.x, r.w0[1] = a.y, r.w0[2] = a.z, r.w0[3] = a.w, r.w0[4] = b.x, r.w0[5] = b.y, r.w0[6] = b.z, r.w0[7] = b.w;
    return r;
  };
  // kWire: the first tick's packet heads, with the state loads (their addresses depend on nothing
  // loaded), so the poll's decode waits one round trip less; each later tick's come one tick
  // ahead (pre_n, with the other deliveries)
  [[maybe_unused]] PkHead pre0[PPL];
  if constexpr (kWire) {
#pragma unroll
    for (int j = 0; j < PPL; ++j) pre0[j] = wire_fetch(min(player_of(j), P - 1), 0);
  }
  // ---- the packed bookkeeping decoded (q_unpack); a row with a value past its 16-bit deltas reads
  // its absolute rows (a branch taken only then, after every entry load above is in flight)
  if (sc_pk == kQsEscWord) {
    last_saved = p.qs[QS_ABS_SAVED * Spad + s];
    last_conf = p.qs[QS_ABS_CONF * Spad + s];
  } else {
    last_saved = fd_dec(sc_pk, cur);
    last_conf = fd_dec(sc_pk >> 16, cur);
  }
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int h = player_of(j);
    if (h >= P) continue;
    int32_t ab[7] = {0, 0, 0, 0, 0, 0, 0};
    if (qpk[j][3] & kQmEsc) {
#pragma unroll
      for (int i = 0; i < 7; ++i) ab[i] = *qrow(QF_ABS0 + i, h);
    }
    const QFields f = q_unpack(qpk[j], cur, ab);
    q[j].last_added = f.la;
    q[j].conn_last = f.conn;
    q[j].pred_frame = f.pred;
    q[j].first_inc = f.fi;
    q[j].last_req = f.req;
    q[j].tail = f.tail;
    q[j].len = f.len;
    q[j].disc = f.disc;
    if constexpr (IB == 1) q[j].pred_val = f.pv;
  }
#pragma unroll
  for (int j = 0; j < PPL; ++j) any_disc |= q[j].disc;
  any_disc = group_min<L>(any_disc ? 0 : 1) == 0;
  if (panicked) return;
#if RB_P2P_PHASE
  settle(static_cast<uint32_t>(cur));
  settle(w[0]);
  settle(static_cast<uint32_t>(q[0].last_req));
  settle(static_cast<uint32_t>(up[0]));
#endif
  RB_PH(1);
  // LDS queue: the HBM frames this launch can read.  Reads are of frames
  // >= cur - W (adjust_gamestate checks that before it advances) up to the
  // last added one, or of the last added frame itself (predictions and the
  // delay replication); every later frame is added inside the launch.  (The
  // fan-out's candidates come from the queue's move-to-front list, not from
  // these frames: fan_candidates.)
  const int32_t la0 = q[0].last_added;  // (the LDS queue's fill: after the first deliveries' loads, below)

  if constexpr (kLdsC) {  // the snapshot ring of this launch's sessions into LDS
#pragma unroll
    for (int k = 0; k < kLdsCellsMaxW; ++k) {
      const unsigned kk = static_cast<unsigned>(min(k, W - 1));
      uint32_t cw[NW];
      load_words<NW>(p.snap + kk * slot_words, static_cast<int>(Gpad), static_cast<int>(g), cw);
      const int32_t tg = p.tag[kk * Spad + s];
      const CS cv = csa[kk * Spad + s];
      if (k < W) {
#pragma unroll
        for (int n = 0; n < NW; ++n) lds_cell[(kk * NW + n) * bd + tid] = cw[n];
        if (lead) {
          lds_tag[kk * bps + sl] = tg;
          lds_cs[kk * bps + sl] = cv;
        }
      }
    }
  }

  int32_t status = kP2PStatusOk, load_frame = kNullFrame, nadv = 0, nsave = 0;
  uint32_t nonce = 0;
  uint32_t tot_adv = 0, tot_save = 0, tot_load = 0, tot_sel = 0;  // requests the game executed in this launch
  // exec = false: bookkeeping only.  When advance_frame returns
  // Err(PredictionThreshold) the reference drops the request Vec it built
  // (p2p_session.rs:320 `?`): the sync layer has rolled back, saved and
  // re-predicted, but the game never loads, saves or advances.  A dry run
  // reproduces that bookkeeping without touching the game state or the cells.
  bool exec = true;
  auto next_frame = [&]() __attribute__((always_inline)) {  // SyncLayer::advance_frame
    cur += 1;
    cur_slot = cur_slot + 1 == static_cast<unsigned>(W) ? 0u : cur_slot + 1;
  };
  // SaveGameState{cell, frame = cur}: game checksum, cell.save (sync_layer.rs:118-125)
  auto store_cell = [&](int32_t f, unsigned slot) __attribute__((always_inline)) {
    CsCtx ctx{0ull, s, nonce++};
    CS c{};
    if constexpr (!(RB_P2P_EXP & 2)) c = G::checksum(w, f, lane, ctx);
    if constexpr (kLdsC) {
#pragma unroll
      for (int n = 0; n < NW; ++n) lds_cell[(slot * NW + n) * bd + tid] = w[n];
      // the checksum and frame are the session's in every lane of its group, so every lane stores
      // them (same value, same address) and no lead-lane branch splits the save (A/B,
      // profiles/r05_ab_alllane.log: 3.44 -> 3.40 us per tick in 50-tick launches, 5.32 -> 5.26 at 131,072)
      lds_cs[slot * bps + sl] = c;
      lds_tag[slot * bps + sl] = f;
    } else {
      store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), w);
      csa[slot * Spad + s] = c;
      p.tag[slot * Spad + s] = f;
    }
  };
  auto save = [&](int32_t f) __attribute__((always_inline)) {
    last_saved = f;
    ++nsave;
    if (!exec) return;
    ++tot_save;
    store_cell(f, cur_slot);  // f == cur
  };
  // SyncLayer::synchronized_inputs (sync_layer.rs:187-200) for this lane's
  // players: a disconnected player past its last frame is (zeroed, Disconnected)
  // and its queue is not asked
  auto sync_inputs = [&](int32_t f, uint32_t& dmask) __attribute__((always_inline)) -> InRec {
    uint64_t rec = 0;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int h = player_of(j);
      if (h >= P) continue;
      if (q[j].disc && q[j].conn_last < f) {
        dmask |= 1u << h;
      } else {
        rec |= static_cast<uint64_t>(q_input<!kSparse>(q[j], ring, h, s, f)) << (8 * IB * h);
        if constexpr (G::kUsesStatus) dmask |= (q[j].pred_frame >= 0 ? 1u : 0u) << (8 + h);  // InputStatus::Predicted
      }
    }
    return static_cast<InRec>(rec);
  };
  auto advance = [&](int32_t f) __attribute__((always_inline)) {  // AdvanceFrame{inputs}
    uint32_t dmask = 0u;
    const InRec in = sync_inputs(f, dmask);
    ++nadv;
    if (exec) {
      if constexpr (RB_P2P_EXP & 1) w[0] += static_cast<uint32_t>(in);  // attribution builds only
      else advance_frame<G>(w, in, lane, dmask, &p.counters[1]);
      ++tot_adv;
    }
  };
  // P2PSession::adjust_gamestate (p2p_session.rs:621-673)
  // its opening: the load_frame asserts, LoadGameState, reset_prediction; the
  // number of frames to resimulate (-1 after a panic)
  auto adjust_begin = [&](int32_t first_incorrect) __attribute__((always_inline)) -> int32_t {
    const int32_t to_load = kSparse ? last_saved : first_incorrect;
    const int32_t count = cur - to_load;
    const unsigned slot = static_cast<unsigned>(max(to_load, 0) % W);
    // (HBM cells: the cell's words are loaded with its tag, before the checks, so the
    // LoadGameState costs one global round trip instead of two)
    [[maybe_unused]] uint32_t cw[NW];
    if constexpr (!kLdsC) load_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), cw);
    const int32_t tag = kLdsC ? lds_tag[slot * bps + sl] : p.tag[slot * Spad + s];
    if (to_load < 0 || to_load > first_incorrect || count <= 0 || count > W || tag != to_load) {
      status = kP2PStatusPanic;  // a reference assert (sync_layer.rs:141-148) would fire
      return -1;
    }
    if (exec) {  // LoadGameState
      if constexpr (kLdsC) {
#pragma unroll
        for (int n = 0; n < NW; ++n) w[n] = lds_cell[(slot * NW + n) * bd + tid];
      } else {
#pragma unroll
        for (int n = 0; n < NW; ++n) w[n] = cw[n];
      }
      ++tot_load;
    }
    load_frame = to_load;
    cur = to_load;
    cur_slot = slot;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {  // SyncLayer::reset_prediction
      q[j].pred_frame = kNullFrame;
      q[j].first_inc = kNullFrame;
      q[j].last_req = kNullFrame;
    }
    return count;
  };
  auto adjust = [&](int32_t first_incorrect, int32_t min_confirmed) __attribute__((always_inline)) {
    const int32_t count = adjust_begin(first_incorrect);
    for (int32_t i = 0; i < count; ++i) {
      if (kSparse ? cur == min_confirmed : i > 0) save(cur);
      advance(cur);
      next_frame();
    }
  };
  // Speculative select: when the only misprediction is the speculated
  // player's, starting exactly at the branch base, and every input it
  // confirmed since is one value k held, branch k (fanout_kernel, previous
  // tick) already holds what adjust_gamestate would recompute: the states of
  // frames base+1 .. cur-1 and of frame cur, built from the same inputs (k
  // confirmed then k predicted for the speculated player, the reference's
  // predictions for the others, confirmed local inputs).  The sync layer's
  // bookkeeping runs as in adjust (dry), the cells and the state are copied.
  // The per-player select (fan_per_player's branches): the rollback starts at their base B, and
  // every remote player's inputs since its own base hold one class (newly confirmed ones, then the
  // repeat-last prediction; or the prediction alone when none arrived): each lane takes its player's
  // branch of that class (a local player: its one chain) for every cell adjust would save and for
  // the state, and each cell's checksum is rebuilt from the players' fletcher parts.
  // A rollback from F > B (the oldest-unconfirmed player did not mispredict; a later one did) selects
  // too when every lane's branch word at F equals the cell of F the reference loads: the trajectories
  // then agree from F on, whatever the cells of frames B .. F hold (a PredictionThreshold tick can
  // leave cells computed with predictions the sync layer has since dropped, p2p_session.rs:320).
  auto select_per_player = [&](int32_t first_incorrect, int32_t min_confirmed) __attribute__((always_inline)) -> bool {
    if constexpr (kInFan && !kMtf) {
      const int32_t B = sm_base;
      if (first_incorrect < B || first_incorrect >= cur || B + W <= cur) return false;
      const int32_t F = first_incorrect;
      constexpr auto AC = AlphabetClasses<G>::value;
      uint32_t acp[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) acp[qq] = AC.packed[qq];
      const bool my_remote = lane < P && !((p.local_mask >> lane) & 1u);
      bool ok = true;
      int32_t kk = 0;
      if (my_remote) {
        const int32_t la = q[0].last_added;
        const int32_t pb = sm_pbase;  // this player's first unconfirmed frame at the branches' making
        // the class held from pb on: the first newly confirmed input, else the prediction
        const uint32_t c0 = InputCanon<G>::apply(la >= pb ? ring.get(pb, lane, s) : (la == kNullFrame ? 0u : ring.get(la, lane, s))) & 0xFFu;
        for (int32_t f = pb + 1; f <= la && f < cur; ++f) ok &= (InputCanon<G>::apply(ring.get(f, lane, s)) & 0xFFu) == c0;
        kk = cand_find(acp, c0, AC.n);
        ok &= kk >= 0;
      }
      const unsigned Gs = Spad * static_cast<unsigned>(L) * static_cast<unsigned>(kSpecBranches + 1);
      // (fan_per_player's columns: class kk of lane l's player at kk * Spad * L + s * L + l; with FanShare
      // a remote player's cells up to frame P0, where its classes still agree, in the lane's own
      // column 16 * Spad * L + s * L + l, which a local player's chain uses for all of its cells)
      const unsigned col = (my_remote ? static_cast<unsigned>(kk >= 0 ? kk : 0) : static_cast<unsigned>(kSpecBranches)) *
                               (Spad * static_cast<unsigned>(L)) + s * L + static_cast<unsigned>(lane);
      const unsigned ocol = static_cast<unsigned>(kSpecBranches) * (Spad * static_cast<unsigned>(L)) + s * L +
                            static_cast<unsigned>(lane);
      const int32_t P0 = FanShare<G>::value && AC.n == 9 ? min(max(B, sm_pbase), cur) : B;
      auto col_of = [&](int32_t f) __attribute__((always_inline)) { return f <= P0 ? ocol : col; };
      const bool has = lane < P;
      if (F > B && ok && has) {  // the branch at F must be the cell the reference loads
        const unsigned fslot = static_cast<unsigned>(F % W);
        uint32_t bw[NW], cw[NW];
        load_words<NW>(p.spec_cells + static_cast<size_t>(fslot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(col_of(F)), bw);
        if constexpr (kLdsC) {
#pragma unroll
          for (int n = 0; n < NW; ++n) cw[n] = lds_cell[(fslot * NW + n) * bd + tid];
        } else {
          load_words<NW>(p.snap + fslot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), cw);
        }
#pragma unroll
        for (int n = 0; n < NW; ++n) ok &= bw[n] == cw[n];
      }
      ok = group_min<L>(ok ? 1 : 0) == 1;
      if (!ok) return false;
      exec = false;  // the sync layer's side of adjust_gamestate
      adjust(first_incorrect, min_confirmed);
      exec = true;
      if (status == kP2PStatusPanic) return true;
      for (int32_t f = F + 1; f < cur; ++f) {  // the cells adjust would have saved
        const unsigned slot = static_cast<unsigned>(f % W);
        uint32_t cw[NW] = {};
        if (has) load_words<NW>(p.spec_cells + static_cast<size_t>(slot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(col_of(f)), cw);
        if (has) {
          if constexpr (kLdsC) {
#pragma unroll
            for (int n = 0; n < NW; ++n) lds_cell[(slot * NW + n) * bd + tid] = cw[n];
          } else {
            store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), cw);
          }
        }
        Fl16 a{0u, 0u};
        if (has) a = G::fan_partial(cw, lane);
        a.s1 = group_sum<L>(a.s1);
        a.s2 = group_sum<L>(a.s2);
        const CS c = G::fan_finish(a, f);
        if (lead) {
          if constexpr (kLdsC) {
            lds_cs[slot * bps + sl] = c;
            lds_tag[slot * bps + sl] = f;
          } else {
            csa[slot * Spad + s] = c;
            p.tag[slot * Spad + s] = f;
          }
        }
        ++tot_save;
      }
      if (has) load_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(col), w);
      ++tot_sel;
      return true;
    } else {
      return false;
    }
  };
  auto try_select = [&](int32_t first_incorrect, int32_t min_confirmed) __attribute__((always_inline)) -> bool {
    if (kLdsC && !in_fan) return false;  // (not launched: fanout_kernel's branches need HBM cells)
    if (any_disc || disc_frame != kNullFrame) return false;  // the branches assumed everybody connected
    if (!(sm_valid & 1) || sm_end != cur) return false;
    if constexpr (kInFan && !kMtf) {
      if (sm_valid & (1 << 16)) return select_per_player(first_incorrect, min_confirmed);
    }
    const int32_t base = sm_base;
    const int rs = sm_player;
    if (first_incorrect != base || base + W <= cur) return false;
    // every mispredicting player must be the speculated one; its confirmed run from base must be one value
    bool ok = true;
    uint32_t k = 0;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int h = player_of(j);
      if (h >= P) continue;
      if (h != rs) {
        ok &= q[j].first_inc == kNullFrame;
      } else {
        k = ring.get(base, h, s);
        for (int32_t f = base + 1; f <= q[j].last_added && f < cur; ++f) ok &= ring.get(f, h, s) == k;
      }
    }
    // the lane that owns the speculated player found the held value k; its branch is the candidate
    // slot holding k (none: no branch presimulated it); share it with the group
    // (the in-kernel fan-out's branches are the candidates' classes, sm_valid >> 8 of them)
    int32_t kk = in_fan ? cand_find(sm_cand, InputCanon<G>::apply(k) & 0xFFu, sm_valid >> 8) : cand_find(sm_cand, k, p.fan_k);
    kk = (kSplit ? lane == rs : true) ? kk : -1;
    kk = -group_min<L>(-kk);  // max over the group
    ok = group_min<L>(ok ? 1 : 0) == 1;
    if (!ok || kk < 0 || kk >= kSpecBranches) return false;
    exec = false;  // the sync layer's side of adjust_gamestate
    adjust(first_incorrect, min_confirmed);
    exec = true;
    if (status == kP2PStatusPanic) return true;
    if (in_fan) {
      // the in-kernel fan-out's branch kk, written by lane (rs + kk) % L (which alone reads
      // it back and hands the words to the speculated player's lane); every other lane keeps its own
      // cells and state (no misprediction of its player), and each cell's checksum is rebuilt from the
      // players' fletcher parts
      if constexpr (kInFan) {
        const unsigned Gs = Spad * static_cast<unsigned>(kSpecBranches + L);
        const int owner = (rs + kk) % static_cast<int>(L);  // (fan_inlane's deal of branches to lanes)
        // (fan_inlane's columns: branch kk in plane kk / L, the owner lane's column there)
        const unsigned col = static_cast<unsigned>(kk / static_cast<int>(L)) * (Spad * static_cast<unsigned>(L)) + s * L +
                             static_cast<unsigned>(owner);
        const unsigned ocol = Spad * kSpecBranches + s * L + static_cast<unsigned>(lane);  // this lane's player, once
        const bool other = lane < P && lane != rs;
        const int src = static_cast<int>(__lane_id()) - lane + owner;
        for (int32_t f = base + 1; f < cur; ++f) {  // the cells adjust would have saved
          const unsigned slot = static_cast<unsigned>(f % W);
          uint32_t bw[NW], cw[NW] = {};
          if (lane == owner) load_words<NW>(p.spec_cells + static_cast<size_t>(slot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(col), bw);
#pragma unroll
          for (int n = 0; n < NW; ++n) bw[n] = static_cast<uint32_t>(__shfl(static_cast<int>(bw[n]), src, 64));
          if (other) load_words<NW>(p.spec_cells + static_cast<size_t>(slot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(ocol), cw);
          if (lane == rs || other) {
            if (lane == rs) {
#pragma unroll
              for (int n = 0; n < NW; ++n) cw[n] = bw[n];
            }
            if constexpr (kLdsC) {
#pragma unroll
              for (int n = 0; n < NW; ++n) lds_cell[(slot * NW + n) * bd + tid] = cw[n];
            } else {
              store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), cw);
            }
          }
          Fl16 a{0u, 0u};
          if (lane < P) a = G::fan_partial(cw, lane);  // (the padding lane of P = 3 holds no player)
          a.s1 = group_sum<L>(a.s1);
          a.s2 = group_sum<L>(a.s2);
          const CS c = G::fan_finish(a, f);
          if (lead) {
            if constexpr (kLdsC) {
              lds_cs[slot * bps + sl] = c;
              lds_tag[slot * bps + sl] = f;
            } else {
              csa[slot * Spad + s] = c;
              p.tag[slot * Spad + s] = f;
            }
          }
          ++tot_save;
        }
        uint32_t bw[NW];
        if (lane == owner) load_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(col), bw);
#pragma unroll
        for (int n = 0; n < NW; ++n) bw[n] = static_cast<uint32_t>(__shfl(static_cast<int>(bw[n]), src, 64));
        if (lane == rs) {
#pragma unroll
          for (int n = 0; n < NW; ++n) w[n] = bw[n];
        } else if (other) {
          load_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(ocol), w);
        }
      }
    } else if constexpr (!kLdsC) {
      // fanout_kernel's branch kk, this lane: column (s * 16 + kk) * L + lane of planes Spad * 16 * L wide
      const unsigned Gs = Gpad * kSpecBranches;
      const unsigned col = (s * kSpecBranches + static_cast<unsigned>(kk)) * L + lane;
      const CS* __restrict__ scs = reinterpret_cast<const CS*>(p.spec_cs);
      for (int32_t f = base + 1; f < cur; ++f) {  // the cells adjust would have saved
        const unsigned slot = static_cast<unsigned>(f % W);
        uint32_t cw[NW];
        load_words<NW>(p.spec_cells + static_cast<size_t>(slot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(col), cw);
        store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), cw);
        if (lead) {
          csa[slot * Spad + s] = scs[(slot * Spad + s) * kSpecBranches + kk];
          p.tag[slot * Spad + s] = f;
        }
        ++tot_save;
      }
      load_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(col), w);
    }
    ++tot_sel;
    return true;
  };
  // advance_frame (p2p_session.rs:253-303) up to the local inputs: frame-0
  // save, rollback, save / sparse check, set_last_confirmed_frame.
  // the frame-0 save, confirmed_frame (:487-498) and check_simulation_consistency
  auto rollback_open = [&](int32_t& confirmed, int32_t& first_inc) __attribute__((always_inline)) {
    load_frame = kNullFrame;
    nadv = nsave = 0;
    if (cur == 0) save(cur);
    confirmed = INT32_MAX;
    first_inc = INT32_MAX;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      confirmed = min(confirmed, conn_of(j));
      if (q[j].first_inc != kNullFrame) first_inc = min(first_inc, q[j].first_inc);
    }
    confirmed = group_min<L>(confirmed);
    first_inc = group_min<L>(first_inc);
    if (disc_frame != kNullFrame) first_inc = min(first_inc, disc_frame);  // session-uniform
  };
  // set_last_confirmed_frame (sync_layer.rs:220-244)
  auto set_last_confirmed = [&](int32_t confirmed) __attribute__((always_inline)) {
    last_conf = kSparse ? min(confirmed, last_saved) : confirmed;
    if (last_conf > 0) {
#pragma unroll
      for (int j = 0; j < PPL; ++j) q_discard(q[j], last_conf - 1);
    }
  };
  auto rollback_and_save = [&]() __attribute__((always_inline)) {
    int32_t confirmed, first_inc;
    rollback_open(confirmed, first_inc);
    if (first_inc != INT32_MAX) {
      if (!(kSpec && exec && try_select(first_inc, confirmed))) adjust(first_inc, confirmed);
      disc_frame = kNullFrame;
    }
    if (status == kP2PStatusPanic) return;
    if constexpr (kSparse) {  // check_last_saved_state (:778-802)
      if (cur - last_saved >= W) {
        if (confirmed >= cur) save(cur);
        else adjust(last_saved, confirmed);
      }
    } else {
      save(cur);
    }
    set_last_confirmed(confirmed);
    // an InputQueue panic in this tick's resimulation or discard (DevQueue::bad); the advance
    // of the new frame cannot raise one (its frame is above every tail).  Only peers' reports
    // reach those states: without them a queue's tail never passes a frame a rollback reads
    // (rollbacks start above the discarded frames) and only a disconnected player's queue
    // takes the delete-all branch, after which it is read only past its last frame.
    if constexpr (kNet) {
      bool bad = false;
#pragma unroll
      for (int j = 0; j < PPL; ++j) bad |= q[j].bad;
      status = group_min<L>(bad ? 0 : 1) == 0 ? kP2PStatusPanic : status;
    }
  };

  // desync detection after set_last_confirmed_frame (p2p_session.rs:313-316):
  // the lead lane runs it, the group learns whether it panicked
  [[maybe_unused]] CellSnap send_cells{};
  auto run_desync = [&]() __attribute__((always_inline)) -> bool {
    if constexpr (!kNet) {
      return true;
    } else {
      if (p.ds.interval <= 0) return true;
      bool ok = true;
      if (lead) ok = desync_step(p.ds, send_cells, s, Spad, cur, last_saved, W, P, p.local_mask);
      return group_min<L>(ok ? 1 : 0) == 1;
    }
  };
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int32_t f = remote_start(j);
#pragma unroll
    for (int k = 0; k < kPre; ++k) rv[j][k] = load_remote(j, f + k);
  }
  // LDS queue: the HBM frames this launch can read, loaded in the same round trip as the first
  // deliveries above.  Reads are of frames >= cur - W (adjust_gamestate checks that before it
  // advances) up to the last added one, or of the last added frame itself (predictions and the
  // delay replication); every later frame is added inside the launch.  (The fan-out's candidates
  // come from the queue's move-to-front list, not from these frames: fan_candidates.)
  if constexpr (kLdsQ) {
    const int h = player_of(0);
    // (and a packet's reference input, frame start - 1 >= last received - 2 * max_prediction)
    const int32_t back = kWire ? 2 * W + 1 : 0;
    if (h < P && la0 != kNullFrame) {
      const int32_t lo = max(max(0, la0 - (kQueueLen - 1)), min(cur - W, la0) - back);
      constexpr int kFill = 16;  // loads in flight per round trip
      for (int32_t f0 = lo; f0 <= la0; f0 += kFill) {
        uint32_t v[kFill];
#pragma unroll
        for (int k = 0; k < kFill; ++k) v[k] = hbm.get(min(f0 + k, la0), h, s);
#pragma unroll
        for (int k = 0; k < kFill; ++k)
          if (f0 + k <= la0) ring.put(f0 + k, h, s, v[k]);
      }
    }
  }


  // ---- kWire: UdpProtocol::on_input (protocol.rs:616-689) for the endpoint
  // of remote handle h, fused into the poll.  The packet is the XOR delta of
  // its inputs against the input before its start frame, bitfield-RLE coded
  // (network/compression.rs, wire.hip); that reference input is the queue's
  // ring entry of frame start - 1 (recv_inputs holds what the queue holds:
  // remote inputs enter it at their own frame).  A structurally invalid packet
  // adds nothing and panics the session, as the reference's decode().expect
  // does; a first pass validates, the second adds every input past the last
  // received frame.  The first 32 bytes come in as 8 words (a byte window
  // shifted as it is consumed), later bytes one load each.
  [[maybe_unused]] auto wire_poll = [&](int j, int h, int t) __attribute__((always_inline)) -> int32_t {
    if constexpr (!kWire) {
      return kWireNothing;
    } else {
      const size_t idx = (static_cast<size_t>(t) * P + static_cast<size_t>(h)) * static_cast<size_t>(p.S) + s;
      const PkHead hd = kPrefetch ? pre0[j] : (t == 0 ? pre0[j] : wire_fetch(h, t));  // (tick t's heads)
      const int32_t n = hd.n, start = hd.start;
      const uint8_t* pk = p.packets + static_cast<int64_t>(idx) * p.packet_stride;
      uint32_t w0[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) w0[i] = hd.w0[i];
      if (q[j].disc || n <= 0) return kWireNothing;  // a disconnected player's endpoint no longer runs
      if (n > p.packet_stride) return kWirePanic;    // the row does not hold that many bytes
      const int32_t last = q[j].conn_last;
      if (last != kNullFrame && last + 1 < start) return kWireGap;  // assert! (protocol.rs:639-642)
      if (last != kNullFrame && (start - 1 < last - 2 * W || start - 1 < kNullFrame)) return kWireNothing;
      const uint32_t ref = (last != kNullFrame && start - 1 != kNullFrame) ? ring.get(start - 1, h, s) : 0u;
      // The two packet shapes a tick's delta of a few inputs takes: one literal run of every byte, or
      // (inputs equal to the reference) one compressed run.  Both are valid by their header alone, so
      // their inputs are added in one pass, without the general parse below.
      {
        const uint32_t h0 = w0[0] & 0xFFu;
        const bool lit = !(h0 & 0x81u) && static_cast<int32_t>(h0 >> 1) == n - 1 && n <= 32 && (n - 1) % IB == 0;
        const bool run = (h0 & 0x81u) == 1u && n == 1 && (h0 >> 2) % IB == 0;
        if (lit || run) {
          const int32_t nb = lit ? n - 1 : static_cast<int32_t>(h0 >> 2);
          const uint32_t fill = (h0 & 2u) ? 0xFFu : 0u;
          uint32_t win[8];
#pragma unroll
          for (int i = 0; i < 7; ++i) win[i] = __builtin_amdgcn_alignbyte(w0[i + 1], w0[i], 1);  // skip the header
          win[7] = w0[7] >> 8;
          uint32_t acc = 0;
          for (int32_t k = 0; k < nb; ++k) {
            const uint32_t x = lit ? (win[0] & 0xFFu) : fill;
            if (lit) {
#pragma unroll
              for (int i = 0; i < 7; ++i) win[i] = __builtin_amdgcn_alignbyte(win[i + 1], win[i], 1);
              win[7] >>= 8;
            }
            const int i = k % IB;
            acc |= (((ref >> (8 * i)) ^ x) & 0xFFu) << (8 * i);
            if (i == IB - 1) {
              const int32_t f = start + k / IB;
              if (f > last) {  // protocol.rs:661-663
                q_add<InputCanon<G>>(q[j], ring, h, s, f, acc);
                q[j].conn_last = f;
              }
              acc = 0;
            }
          }
          return start + nb / IB - 1 > last ? kWireOk : kWireNothing;
        }
      }
      // pass 0 validates (and counts the bytes the inputs take), pass 1 adds the inputs
      int32_t nbytes = 0;
      for (int pass = 0; pass < 2; ++pass) {
        uint32_t win[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) win[i] = w0[i];
        int32_t pos = 0, k = 0;
        uint32_t acc = 0;
        auto next = [&]() __attribute__((always_inline)) -> uint32_t {
          const uint32_t b = pos < 32 ? (win[0] & 0xFFu) : pk[pos];
#pragma unroll
          for (int i = 0; i < 7; ++i) win[i] = __builtin_amdgcn_alignbyte(win[i + 1], win[i], 1);
          win[7] >>= 8;
          ++pos;
          return b;
        };
        auto emit = [&](uint32_t x) __attribute__((always_inline)) {
          const int i = k % IB;
          acc |= (((ref >> (8 * i)) ^ x) & 0xFFu) << (8 * i);
          if (i == IB - 1) {
            const int32_t f = start + k / IB;
            if (f > last) {  // protocol.rs:661-663: inputs already received are skipped
              q_add<InputCanon<G>>(q[j], ring, h, s, f, acc);  // add_remote_input (frame delay 0)
              q[j].conn_last = f;
            }
            acc = 0;
          }
          ++k;
        };
        bool ok = true;
        while (pos < n) {
          uint32_t hdr = 0;
          int shift = 0;
          bool done = false;
          while (pos < n && shift < 35) {  // LEB128
            const uint32_t b = next();
            hdr |= (b & 0x7Fu) << shift;
            shift += 7;
            if (!(b & 0x80u)) {
              done = true;
              break;
            }
          }
          if (!done) {
            ok = false;
            break;
          }
          if (hdr & 1u) {  // a run of 0x00 / 0xFF bytes
            const uint32_t len = hdr >> 2;
            if (len > (1u << 16)) {
              ok = false;
              break;
            }
            if (pass == 0) {
              k += static_cast<int32_t>(len);
            } else {
              const uint32_t x = (hdr & 2u) ? 0xFFu : 0u;
              for (uint32_t i = 0; i < len; ++i) emit(x);
            }
          } else {  // literal bytes
            const uint32_t len = hdr >> 1;
            if (len > static_cast<uint32_t>(n - pos)) {
              ok = false;
              break;
            }
            for (uint32_t i = 0; i < len; ++i) {
              const uint32_t x = next();
              if (pass == 1) emit(x);
              else ++k;
            }
          }
        }
        if (pass == 0) {
          if (!ok || k % IB != 0) return kWirePanic;  // compression.rs:47: whole inputs only
          nbytes = k;
        }
      }
      return start + nbytes / IB - 1 > last ? kWireOk : kWireNothing;
    }
  };

  // One tick of the batch for this session (advance_frame and the requests it
  // returns); false when the session stops on a reference panic.
  int32_t up_n[PPL];
  uint32_t lin_n[PPL], rv_n[PPL][kPre];
  [[maybe_unused]] PkHead pre_n[PPL];  // kWire: the next tick's packet heads
  [[maybe_unused]] int32_t pk_ds[PPL];  // kWire: the last tick's decode status of each endpoint this lane serves
#pragma unroll
  for (int j = 0; j < PPL; ++j) pk_ds[j] = kWireNothing;
  uint32_t n_thr = 0;                             // PredictionThreshold ticks of this session in the launch
  // The tick's opening, through the PredictionThreshold decision: 0 = the
  // session stopped on a panic, 1 = the tick is over (Err(PredictionThreshold)),
  // 2 = rollback_and_save, add_local_input and the new frame follow.
  // (the next tick's deliveries are prefetched unless kPrefetch is false, above)
  auto tick_begin = [&](int t) __attribute__((always_inline)) -> int {
    const int tn = t + 1 < T ? t + 1 : t;

    // A one-tick launch has no next tick to prefetch for (measured: 10.40 -> 9.96 us per one-tick launch
    // at 65,536 sessions, 94.5 -> 91.6 at 1,048,576; profiles/r06_ab_short_waves.log).  The packet-fed
    // fused launches (kWire with the LDS ring) prefetch without the branch: with it their ticks ran
    // 4.88 -> 5.26 us, while the plain fused ticks run faster with it (3.37 -> 3.11 us; sparse and the
    // C4 fan-out neutral; profiles/r06_ab_prefetch_branch.log).
    const bool pre_next = (kWire && kLdsC) || T > 1;
    if constexpr (kPrefetch) {
      if (pre_next) {
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          up_n[j] = load_upto(tn, j);
          lin_n[j] = load_local(tn, j);
          if constexpr (kWire) pre_n[j] = wire_fetch(min(player_of(j), P - 1), tn);
        }
      }
    }
    status = kP2PStatusOk;
    load_frame = kNullFrame;
    nadv = nsave = 0;
    // ---- poll_remote_clients: Event::Input in frame order (handle_event, :838-852)
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int h = player_of(j);
      if constexpr (kWire) {
        if (h < P && !((p.local_mask >> h) & 1u)) {
          const int32_t ds = wire_poll(j, h, t);
          pk_ds[j] = ds;  // (stored once per endpoint, at the end of the launch)
          // the reference panics: "decoding failed" (protocol.rs:656) or the gap assert (:639-642)
          if (ds == kWirePanic || ds == kWireGap) status = kP2PStatusPanic;
        }
        continue;
      }
      if (h < P && !((p.local_mask >> h) & 1u) && !q[j].disc) {  // handle_event ignores a disconnected player (:852)
        const int32_t end = min(up[j], p.remote_frames - 1);
        int32_t f = remote_start(j);
#pragma unroll
        for (int k = 0; k < kPre; ++k, ++f) {
          if (f > end) break;
          q_add<InputCanon<G>>(q[j], ring, h, s, f, rv[j][k]);  // add_remote_input (frame delay 0)
          q[j].conn_last = f;
        }
        for (; f <= end; ++f) {  // more than kPre frames delivered in one tick
          q_add<InputCanon<G>>(q[j], ring, h, s, f, load_remote(j, f));
          q[j].conn_last = f;
        }
      }
    }
    if constexpr (kPrefetch) {
      if (pre_next) {
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const int32_t f = remote_start(j);
#pragma unroll
          for (int k = 0; k < kPre; ++k) rv_n[j][k] = load_remote(j, f + k);
        }
      }
    }
    {  // input_queue.rs:181 assert!(self.length <= INPUT_QUEUE_LENGTH) fired during the poll.  No
      // branch here: the panic status is picked up by the panic check after the threshold decision
      // (a branch at this point would make the waitcnt pass wait for the loads in flight).
      bool ovf = kWire && status == kP2PStatusPanic;  // (a malformed packet, decoded by its player's lane)
#pragma unroll
      for (int j = 0; j < PPL; ++j) ovf |= q_overflow(q[j]);
      status = group_min<L>(ovf ? 0 : 1) == 0 ? kP2PStatusPanic : status;
    }
    if constexpr (kNet) {
      // ---- update_player_disconnects (p2p_session.rs:274-275, 707-742), before the
      // confirmed frame is taken.  Every lane of the group runs the handle loop on the
      // gathered connection flags (the same values in every lane), then keeps its own
      // handles' results.  Each remote handle is its own endpoint: an endpoint runs
      // until its player is disconnected.
      if (p.peer.on) {
        bool dsc[P];
        int32_t lastf[P];
#pragma unroll
        for (int h = 0; h < P; ++h) {
          if constexpr (kSplit) {
            const int src = static_cast<int>(__lane_id()) - lane + h;
            dsc[h] = __shfl(q[0].disc ? 1 : 0, src, 64) != 0;
            lastf[h] = __shfl(q[0].conn_last, src, 64);
          } else {
            dsc[h] = q[h].disc;
            lastf[h] = q[h].conn_last;
          }
        }
        auto at = [&](int e, int i) { return (static_cast<size_t>(e) * 4 + static_cast<size_t>(i)) * Spad + s; };
#pragma unroll
        for (int h = 0; h < P; ++h) {
          bool queue_connected = true;
          int32_t queue_min = INT32_MAX;
#pragma unroll
          for (int e = 0; e < P; ++e) {
            if (((p.local_mask >> e) & 1u) || dsc[e]) continue;  // !endpoint.is_running()
            queue_connected = queue_connected && p.peer.disc[at(e, h)] == 0;
            queue_min = min(queue_min, p.peer.last[at(e, h)]);
          }
          const bool local_connected = !dsc[h];
          if (local_connected) queue_min = min(queue_min, lastf[h]);
          if (!queue_connected && (local_connected || lastf[h] > queue_min) && !((p.local_mask >> h) & 1u)) {
            dsc[h] = true;  // disconnect_player_at_frame(h, queue_min) (:555-581)
            if (cur > queue_min) disc_frame = queue_min + 1;
          }
        }
        any_disc = false;
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const int h = player_of(j);
          if (h < P) q[j].disc = dsc[h];
        }
#pragma unroll
        for (int h = 0; h < P; ++h) any_disc |= dsc[h];
      }
      // ---- the cells check_checksum_send_interval will read, before this tick's saves
      if (p.ds.interval > 0) {
        int32_t confirmed = INT32_MAX;
#pragma unroll
        for (int j = 0; j < PPL; ++j) confirmed = min(confirmed, conn_of(j));
        confirmed = group_min<L>(confirmed);  // confirmed_frame (:487-498)
        if (lead && cur % p.ds.interval == 0) send_cells = snap_send_cells(csa, p.tag, s, Spad, W, cur, confirmed, last_saved);
      }
    }
    // ---- PredictionThreshold (sync_layer.rs:163-167) is decided by bookkeeping
    // alone: without sparse saving from the confirmed frame, with it by a dry run.
    bool threshold;
    if constexpr (!kSparse) {
      int32_t confirmed = INT32_MAX;
#pragma unroll
      for (int j = 0; j < PPL; ++j) confirmed = min(confirmed, conn_of(j));
      confirmed = group_min<L>(confirmed);
      threshold = cur >= W && cur - confirmed >= W;
      if (threshold) {  // the dropped request list: bookkeeping only
        exec = false;
        rollback_and_save();
        exec = true;
      }
    } else {
      // With sparse saving the decision needs the frames rollback_and_save leaves behind.  They follow
      // from a handful of frame numbers: the rollback loads last_saved (sparse) and saves exactly the
      // confirmed frame when it passes it; check_last_saved_state (:778-802) then saves the current
      // frame or rolls back again from last_saved; last_confirmed = min(confirmed, last_saved).  So the
      // outcome and every assert the two loads would fire (load_frame, sync_layer.rs:141-148) are
      // decided here, and the bookkeeping-only dry run of rollback_and_save (a second pass over every
      // resimulated frame's input queues) runs only when that decision is PredictionThreshold or a
      // panic, whose state the dry run must leave; or with network reports on (kNet), whose queue
      // asserts are not decided here.  Measured: skipping the dry run takes the sparse tick from 9.55
      // to 5.99 us (profiles/r06_ab_sparse_dry.log).
      bool need_dry = kNet || (RB_P2P_EXP & 128);
      if constexpr (!kNet) {
        int32_t C = INT32_MAX, FI = INT32_MAX;
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          C = min(C, conn_of(j));
          if (q[j].first_inc != kNullFrame) FI = min(FI, q[j].first_inc);
        }
        C = group_min<L>(C);  // confirmed_frame (:487-498)
        FI = group_min<L>(FI);
        if (disc_frame != kNullFrame) FI = min(FI, disc_frame);
        const int32_t c = cur;
        int32_t ls = c == 0 ? 0 : last_saved;  // (the frame-0 save, :270-272)
        bool pan = false;
        auto adj = [&](int32_t fi) __attribute__((always_inline)) {  // adjust_gamestate(fi, C), sparse
          const int32_t to_load = ls, count = c - to_load;
          const unsigned slot = static_cast<unsigned>(max(to_load, 0) % W);
          const int32_t tag = kLdsC ? lds_tag[slot * bps + sl] : p.tag[slot * Spad + s];
          pan |= to_load < 0 || to_load > fi || count <= 0 || count > W || tag != to_load;
          if (to_load <= C && C < c) ls = C;  // the save of the confirmed frame on the way
        };
        if (FI != INT32_MAX) adj(FI);
        if (c - ls >= W) {
          if (C >= c) ls = c;
          else adj(ls);
        }
        const int32_t lc = min(C, ls);
        need_dry = pan || (c >= W && c - lc >= W);
      }
      if (need_dry) {
        const int32_t cur0 = cur, ls0 = last_saved, df0 = disc_frame;
        const unsigned cs0 = cur_slot;
        DevQueue q0[PPL];
#pragma unroll
        for (int j = 0; j < PPL; ++j) q0[j] = q[j];
        exec = false;
        if constexpr (!(RB_P2P_EXP & 128)) rollback_and_save();  // (attribution builds: 128 skips the dry run)
        exec = true;
        threshold = status != kP2PStatusPanic && cur >= W && cur - last_conf >= W && !(RB_P2P_EXP & 128);
        if (!threshold && status != kP2PStatusPanic) {
          cur = cur0;
          cur_slot = cs0;
          last_saved = ls0;
          disc_frame = df0;
#pragma unroll
          for (int j = 0; j < PPL; ++j) q[j] = q0[j];
        }
      } else {
        threshold = false;
      }
    }
    if (status == kP2PStatusPanic) return 0;
    if (threshold) {
      status = kP2PStatusThreshold;  // Err(PredictionThreshold): the game does not move this tick
      load_frame = kNullFrame;       // and the user never sees the dropped requests
      nadv = nsave = 0;
      ++n_thr;  // (added to the batch counter once, at the end of the launch)
      if (!run_desync()) {  // desync detection ran before add_local_input failed (:313-316, :334)
        status = kP2PStatusPanic;
        return 0;
      }
      return 1;
    }
    return 2;
  };
  // ---- local inputs: SyncLayer::add_local_input (sync_layer.rs:159-174)
  auto add_local = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int h = player_of(j);
      if (h >= P || !((p.local_mask >> h) & 1u)) continue;
      q[j].conn_last = q_add<InputCanon<G>>(q[j], ring, h, s, cur + p.delay, lin[j]);  // local_connect_status[h].last_frame
    }
  };
  // ---- the in-kernel fan-out (kInFan, see inlane_fan), after the tick: the
  // speculated player (the remote handle with the oldest last added input,
  // ties: the lowest handle), its first unconfirmed frame `base`, and the K
  // candidates' branches from the saved cell of `base` up to the current
  // frame, each saving its cells like adjust_gamestate would.  Every lane of
  // the session runs 16 / L of the branches, kFanGroup at a time.
  [[maybe_unused]] uint32_t tot_branch = 0;
  // ---- the per-player form (RB_P2P_FLAG_FANOUT_PER_PLAYER; whole alphabet only): every remote
  // player is speculated.  B = the oldest first unconfirmed frame over the remote players; each
  // remote player's own lane presimulates the nb input classes of that player from the cell of B
  // (confirmed inputs up to its own last added frame, then the class held), each local player's
  // lane its player once with its confirmed inputs.  A later tick whose rollback starts at B and
  // in which every remote player's newly confirmed inputs hold one class (or none arrived) then
  // selects, player by player (try_select).  Columns: class k of lane l's player k * Spad * L + s * L
  // + l, a local player's chain Spad * L * 16 + s * L + l (planes Spad * L * 17 wide).
  auto fan_per_player = [&]() __attribute__((always_inline)) {
    if constexpr (kInFan && !kMtf) {
      const int lane_base = static_cast<int>(__lane_id()) - lane;
      int32_t B = INT32_MAX;
      int nrem = 0;
#pragma unroll
      for (int h = 0; h < P; ++h) {
        const int32_t la = __shfl(q[0].last_added, lane_base + h, 64);
        if ((p.local_mask >> h) & 1u) continue;
        B = min(B, (la == kNullFrame ? -1 : la) + 1);
        ++nrem;
      }
      const bool my_remote = lane < P && !((p.local_mask >> lane) & 1u);
      const int32_t la_own = q[0].last_added;
      sm_pbase = (la_own == kNullFrame ? -1 : la_own) + 1;
      const unsigned bslot = static_cast<unsigned>(B >= 0 && B != INT32_MAX ? B % W : 0);
      const int32_t btag = kLdsC ? lds_tag[bslot * bps + sl] : p.tag[bslot * Spad + s];
      const bool valid = !(RB_FAN_EXP & 1) && !any_disc && nrem > 0 && B >= 0 && B < cur && B + W > cur && btag == B;
      constexpr auto AC = AlphabetClasses<G>::value;
      constexpr int nb = AC.n;
      uint32_t acp[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) acp[qq] = AC.packed[qq];
      sm_valid = valid ? (1 | (nb << 8) | (1 << 16)) : 0;
      sm_base = B;
      sm_end = cur;
      sm_player = -1;
      if (!valid) return;  // session-uniform
      uint32_t ow[NW];  // this lane's player's words of the cell of B
      if constexpr (kLdsC) {
#pragma unroll
        for (int n = 0; n < NW; ++n) ow[n] = lds_cell[(bslot * NW + n) * bd + tid];
      } else {
        load_words<NW>(p.snap + bslot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), ow);
      }
      const int h_own = min(lane, P - 1);
      const bool own_local = (p.local_mask >> h_own) & 1u;
      const uint32_t pred_own = la_own == kNullFrame ? 0u : ring.get(la_own, h_own, s);
      uint32_t vin[kFanPre];
      fan_prefetch(ring, h_own, s, B, cur, own_local, la_own, pred_own, vin);
      const uint64_t vpk = fan_pack(vin);
      const unsigned Gs = Spad * static_cast<unsigned>(L) * static_cast<unsigned>(kSpecBranches + 1);
      // class k of this lane's player at column k * Spad * L + s * L + lane: one chain slot of the whole
      // wave stores 64 consecutive words per plane (with the columns (s * L + lane) * 16 + k of round 5 a
      // store wrote 4 bytes of every 64-byte line: the per-player C4 tick spent 21 of its 61 us storing)
      const unsigned bcol = s * static_cast<unsigned>(L) + static_cast<unsigned>(lane);
      const unsigned ocol = Spad * static_cast<unsigned>(L) * kSpecBranches + s * L + static_cast<unsigned>(lane);
      const int nsl = my_remote ? nb : (lane < P ? 1 : 0);  // this lane's chains
      bool inr = false;
      if constexpr (G::kHasRangePath && RB_FAN_INRANGE) inr = __all(G::in_range(ow));
      auto adv = [&](uint32_t (&x)[NW], InRec in) __attribute__((always_inline)) {
        if constexpr (G::kHasRangePath) {
          if (inr) {
            G::template advance<true>(x, in, h_own, 0u, &p.counters[1]);
            return;
          }
        }
        advance_frame<G>(x, in, h_own, 0u, &p.counters[1]);
      };
      auto group = [&](auto ng_tag, int b0) __attribute__((always_inline)) {
        constexpr int NG = decltype(ng_tag)::value;
        uint32_t wb[NG][NW];
        uint32_t rep[NG];
        bool on[NG];
        unsigned col[NG];
#pragma unroll
        for (int b = 0; b < NG; ++b) {
          const int k = b0 + b;
          on[b] = k < nsl;
          rep[b] = cand_at(acp, k & (kSpecBranches - 1));
          col[b] = my_remote ? static_cast<unsigned>(k & (kSpecBranches - 1)) * (Spad * static_cast<unsigned>(L)) + bcol : ocol;
#pragma unroll
          for (int n = 0; n < NW; ++n) wb[b][n] = ow[n];
        }
        unsigned fsl = bslot;  // f % W, kept alongside f (no integer division per frame)
        for (int32_t f = B; f < cur; ++f, fsl = fsl + 1 == static_cast<unsigned>(W) ? 0u : fsl + 1) {
          if (f > B && !(RB_FAN_EXP & 2)) {  // SaveGameState of frame f in every chain
            const unsigned slot = fsl;
#pragma unroll
            for (int b = 0; b < NG; ++b)
              if (on[b]) store_words<NW>(p.spec_cells + static_cast<size_t>(slot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(col[b]), wb[b]);
          }
          // the player's input of frame f: confirmed up to its last added frame, then the chain's class
          // (a remote player) or its repeat-last prediction (a local player's inputs are all confirmed)
          const int j = f - B;
          uint32_t v;
          if (j < kFanPre) v = fan_input(vpk, j);
          else if (own_local || (la_own != kNullFrame && f <= la_own)) v = ring.get(f, h_own, s);
          else v = pred_own;
          const bool held = my_remote && !(la_own != kNullFrame && f <= la_own);
#pragma unroll
          for (int b = 0; b < NG; ++b)
            adv(wb[b], static_cast<InRec>(static_cast<uint64_t>(held ? rep[b] : v) << (8 * h_own)));
        }
#pragma unroll
        for (int b = 0; b < NG; ++b)
          if (on[b]) store_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(col[b]), wb[b]);
      };
      if constexpr (FanShare<G>::value && nb == 9) {
        // A remote player's classes agree until its first unconfirmed frame pb: the frames up to it
        // are run once, their cells stored in the lane's own column (the one a local player's chain
        // uses; select_per_player reads frames up to P0 there).  From P0 on the nine classes are
        // three turn groups (no turn, left, right) of three thrusts each: per group and frame one
        // rotation step and one sine / cosine serve its three classes (ExGame::fan_turn / fan_thrust,
        // fan_move per class), where every class ran the whole AdvanceFrame before.
        if (my_remote) {
          const int32_t P0 = min(max(B, sm_pbase), cur);
          uint32_t x[NW];
#pragma unroll
          for (int n = 0; n < NW; ++n) x[n] = ow[n];
          unsigned fsl = bslot;
          for (int32_t f = B; f < P0; ++f, fsl = fsl + 1 == static_cast<unsigned>(W) ? 0u : fsl + 1) {
            if (f > B && !(RB_FAN_EXP & 2))
              store_words<NW>(p.spec_cells + static_cast<size_t>(fsl) * NW * Gs, static_cast<int>(Gs), static_cast<int>(ocol), x);
            const int j = f - B;
            const uint32_t v = j < kFanPre ? fan_input(vpk, j) : ring.get(f, h_own, s);  // confirmed (f <= la_own)
            adv(x, static_cast<InRec>(static_cast<uint64_t>(v) << (8 * h_own)));
          }
          if (P0 > B && P0 < cur && !(RB_FAN_EXP & 2))  // the cell of frame P0, common to every class
            store_words<NW>(p.spec_cells + static_cast<size_t>(fsl) * NW * Gs, static_cast<int>(Gs), static_cast<int>(ocol), x);
          constexpr auto ACs = AlphabetClasses<G>::value;
          constexpr uint32_t kSlots = static_cast<uint32_t>(class_slot(ACs, 0)) | static_cast<uint32_t>(class_slot(ACs, 1)) << 4 |
                                      static_cast<uint32_t>(class_slot(ACs, 2)) << 8 | static_cast<uint32_t>(class_slot(ACs, 4)) << 12 |
                                      static_cast<uint32_t>(class_slot(ACs, 5)) << 16 | static_cast<uint32_t>(class_slot(ACs, 6)) << 20 |
                                      static_cast<uint32_t>(class_slot(ACs, 8)) << 24 | static_cast<uint32_t>(class_slot(ACs, 9)) << 28;
          constexpr uint32_t kSlot10 = static_cast<uint32_t>(class_slot(ACs, 10));
#pragma unroll 1
          for (int tg = 0; tg < 3; ++tg) {  // turn groups: class bits 2-3 = 0, 4 (left), 8 (right); one at a time
            const uint32_t turn = static_cast<uint32_t>(tg) * 4u;
            uint32_t wb[3][NW];
            unsigned cc[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {  // thrust: class bits 0-1 = 0, 1 (up), 2 (down)
              const int q = tg * 3 + c;  // the class slots of (turn, thrust) in the AlphabetClasses order
              cc[c] = q < 8 ? (kSlots >> (4 * q)) & 15u : kSlot10;
#pragma unroll
              for (int n = 0; n < NW; ++n) wb[c][n] = x[n];
            }
            float rot = __uint_as_float(x[4]);
            SinCos th{0.0f, 0.0f};
            if (tg == 0) th = inr ? G::template fan_thrust<true>(rot, &p.counters[1]) : G::template fan_thrust<false>(rot, &p.counters[1]);
            unsigned fs2 = fsl;
            for (int32_t f = P0; f < cur; ++f, fs2 = fs2 + 1 == static_cast<unsigned>(W) ? 0u : fs2 + 1) {
              if (f > P0 && !(RB_FAN_EXP & 2)) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                  store_words<NW>(p.spec_cells + static_cast<size_t>(fs2) * NW * Gs, static_cast<int>(Gs),
                                  static_cast<int>(cc[c] * (Spad * static_cast<unsigned>(L)) + bcol), wb[c]);
              }
              if (tg != 0) th = inr ? G::template fan_thrust<true>(rot, &p.counters[1]) : G::template fan_thrust<false>(rot, &p.counters[1]);
#pragma unroll
              for (int c = 0; c < 3; ++c) G::fan_move(wb[c], th.c, th.s, static_cast<uint32_t>(c));
              rot = inr ? G::template fan_turn<true>(rot, turn) : G::template fan_turn<false>(rot, turn);
#pragma unroll
              for (int c = 0; c < 3; ++c) wb[c][4] = __float_as_uint(rot);
            }
#pragma unroll
            for (int c = 0; c < 3; ++c)
              store_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(cc[c] * (Spad * static_cast<unsigned>(L)) + bcol), wb[c]);
          }
        } else if (lane < P) {
          group(std::integral_constant<int, 1>{}, 0);  // a local player's one chain
        }
      } else {
        int ns = 0;  // the chain slots the wave runs: the most any of its lanes needs
#pragma unroll
        for (int sb = 0; sb < kSpecBranches; ++sb) ns += __any(sb < nsl) ? 1 : 0;
        for (int b0 = 0; b0 < ns; b0 += kFanGroup) {
          const int ng = min(kFanGroup, ns - b0);
          if (ng == 1) group(std::integral_constant<int, 1>{}, b0);
          else if (ng == 2 || kFanGroup == 2) group(std::integral_constant<int, 2>{}, b0);
          else if (ng == 3 || kFanGroup == 3) group(std::integral_constant<int, 3>{}, b0);
          else group(std::integral_constant<int, (kFanGroup >= 4 ? 4 : 3)>{}, b0);
        }
      }
      tot_branch += static_cast<uint32_t>(cur - B) * static_cast<uint32_t>(nb * nrem);
    }
  };
  auto fan_inlane = [&]() __attribute__((always_inline)) {
    if constexpr (kInFan && !kMtf) {
      if (p.spec_per_player) {
        fan_per_player();
        return;
      }
    }
    if constexpr (kInFan) {
      const int lane_base = static_cast<int>(__lane_id()) - lane;
      int rs = -1;
      int32_t la_rs = INT32_MAX;
#pragma unroll
      for (int h = 0; h < P; ++h) {
        const int32_t la = __shfl(q[0].last_added, lane_base + h, 64);
        if ((p.local_mask >> h) & 1u) continue;
        const int32_t key = la == kNullFrame ? -1 : la;
        if (key < la_rs) {
          la_rs = key;
          rs = h;
        }
      }
      const int32_t base = la_rs + 1;
      const unsigned bslot = static_cast<unsigned>(base >= 0 ? base % W : 0);
      const int32_t btag = kLdsC ? lds_tag[bslot * bps + sl] : p.tag[bslot * Spad + s];
      const bool valid = !(RB_FAN_EXP & 1) && !any_disc && rs >= 0 && base < cur && base + W > cur && base >= 0 && btag == base;
      // the speculated player's candidates as distinct classes (InputCanon): one branch per class.
      // A whole alphabet of at most K values gives a compile-time set; otherwise the queue's
      // move-to-front list, which for this fan-out already holds distinct classes (mcanon).
      uint32_t cand[4];
      int nb;
      if constexpr (!kMtf) {  // the whole alphabet (at most K values)
        constexpr auto AC = AlphabetClasses<G>::value;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) cand[qq] = AC.packed[qq];
        nb = AC.n;
      } else {  // the speculated player's candidate list, from its lane
        const int src = lane_base + max(rs, 0);
        const uint64_t mlo = static_cast<uint32_t>(__shfl(static_cast<int>(q[0].mlo), src, 64)) |
                             static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(q[0].mlo >> 32), src, 64))) << 32;
        const uint64_t mhi = static_cast<uint32_t>(__shfl(static_cast<int>(q[0].mhi), src, 64)) |
                             static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(q[0].mhi >> 32), src, 64))) << 32;
        fan_candidates(mlo, mhi, __shfl(q[0].mn, src, 64), InputAlphabet<G>::value, p.fan_k, cand, canon_reps<G>());
        // distinct classes in a prefix, unused slots 0xFF after it: the branch count is the index
        // of the first 0xFF byte (the lowest zero byte of the complement, exact)
        const uint64_t xl = ~(static_cast<uint64_t>(cand[1]) << 32 | cand[0]);
        const uint64_t xh = ~(static_cast<uint64_t>(cand[3]) << 32 | cand[2]);
        const uint64_t zl = (xl - 0x0101010101010101ull) & ~xl & 0x8080808080808080ull;
        const uint64_t zh = (xh - 0x0101010101010101ull) & ~xh & 0x8080808080808080ull;
        nb = min(p.fan_k, zl ? static_cast<int>(__builtin_ctzll(zl) >> 3)
                             : (zh ? 8 + static_cast<int>(__builtin_ctzll(zh) >> 3) : kSpecBranches));
      }
      sm_valid = valid ? (1 | (nb << 8)) : 0;  // (the branch count rides along)
      sm_base = base;
      sm_end = cur;
      sm_player = rs;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) sm_cand[qq] = cand[qq];
      if (!valid) return;  // session-uniform
      // the speculated player's words of the base cell (its lane's column), and this lane's own
      uint32_t bw[NW], ow[NW];
      if constexpr (kLdsC) {
#pragma unroll
        for (int n = 0; n < NW; ++n) {
          bw[n] = lds_cell[(bslot * NW + n) * bd + tid - static_cast<unsigned>(lane) + static_cast<unsigned>(rs)];
          ow[n] = lds_cell[(bslot * NW + n) * bd + tid];
        }
      } else {
        load_words<NW>(p.snap + bslot * slot_words, static_cast<int>(Gpad), static_cast<int>(g) - lane + rs, bw);
        load_words<NW>(p.snap + bslot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), ow);
      }
      // The chains: the nb branches and, in every other player's lane, that player simulated once
      // from the base cell with the inputs a rollback would give it (confirmed, or the repeat-last
      // prediction): not always the main trajectory's, which keeps the effect of predictions a
      // PredictionThreshold tick dropped the rollback of (p2p_session.rs:320); into column
      // Spad * 16 + s * L + lane.  Chain slots are dealt round-robin starting at the speculated
      // player's lane, which simulates no player of its own: branch k runs in lane (rs + k) % L,
      // slot k / L, and each other player's chain takes the wave's last slot, which no other
      // player's lane needs for a branch.  So the wave runs ceil((nb + P - 1) / L) slots or fewer
      // (ex_game's 9 classes at P = 4: 3, where branches by k % L plus the other players' chains
      // took 4).
      const int h_own = min(lane, P - 1);  // (the padding lane of P = 3 reads a real row, unused)
      const bool other = lane < P && lane != rs;
      const bool own_local = (p.local_mask >> h_own) & 1u;
      const int32_t la_own = q[0].last_added;
      const uint32_t pred_own = la_own == kNullFrame ? 0u : ring.get(la_own, h_own, s);
      uint32_t vin[kFanPre];
      fan_prefetch(ring, h_own, s, base, cur, own_local, la_own, pred_own, vin);
      const uint64_t vpk = fan_pack(vin);
      const unsigned Gs = Spad * static_cast<unsigned>(kSpecBranches + L);  // branch columns, then the others'
      const unsigned ocol = Spad * kSpecBranches + s * L + static_cast<unsigned>(lane);
      const int r = (lane - rs) & static_cast<int>(L - 1);  // this lane's place in the deal
      const int nbr = nb > r ? (nb - r + static_cast<int>(L) - 1) / static_cast<int>(L) : 0;  // its branch slots
      // (an other player's lane has nbr < the wave's slot count: its own chain needs one more)
      const int nslots = nbr + (other ? 1 : 0);
      // every chain of the wave starts in range (games.hpp in_range: e.g. ex_game rotations in [+0, 6.5),
      // which stay there for any number of frames): the AdvanceFrames skip the out-of-range library paths
      bool inr = false;
      if constexpr (G::kHasRangePath && RB_FAN_INRANGE) inr = __all(G::in_range(bw) && G::in_range(ow));
      auto adv = [&](uint32_t (&x)[NW], InRec in, int pl) __attribute__((always_inline)) {
        if constexpr (G::kHasRangePath) {
          if (inr) {
            G::template advance<true>(x, in, pl, 0u, &p.counters[1]);
            return;
          }
        }
        advance_frame<G>(x, in, pl, 0u, &p.counters[1]);
      };
      // One group of a lane's chain slots b0 .. b0 + NG - 1, advanced together (independent chains:
      // instruction-level parallelism); last: the group ends with the wave's last slot.
      auto group = [&](auto ng_tag, int b0, bool last) __attribute__((always_inline)) {
        constexpr int NG = decltype(ng_tag)::value;
        uint32_t wb[NG][NW];
        InRec in[NG];
        bool on[NG], own[NG];
        unsigned col[NG];
        bool any_own = false;
#pragma unroll
        for (int b = 0; b < NG; ++b) {
          const int sb = b0 + b;
          const int k = sb * static_cast<int>(L) + r;
          on[b] = k < nb;
          own[b] = b == NG - 1 && last && other;
          any_own |= own[b];
          in[b] = static_cast<InRec>(static_cast<uint64_t>(cand_at(cand, k & (kSpecBranches - 1))) << (8 * rs));
          // branch k in plane k / L (this lane's column there): a chain slot of the wave stores 64
          // consecutive words per plane (round 5's columns s * 16 + k filled 16 of every 64 bytes)
          col[b] = own[b] ? ocol
                          : static_cast<unsigned>((k & (kSpecBranches - 1)) / static_cast<int>(L)) * (Spad * static_cast<unsigned>(L)) +
                                s * L + static_cast<unsigned>(lane);
#pragma unroll
          for (int n = 0; n < NW; ++n) wb[b][n] = own[b] ? ow[n] : bw[n];
        }
        unsigned fsl = bslot;  // f % W, kept alongside f (no integer division per frame)
        for (int32_t f = base; f < cur; ++f, fsl = fsl + 1 == static_cast<unsigned>(W) ? 0u : fsl + 1) {
          if (f > base && !(RB_FAN_EXP & 2)) {  // SaveGameState of frame f in every chain
            const unsigned slot = fsl;
#pragma unroll
            for (int b = 0; b < NG; ++b)
              if (on[b] || own[b])
                store_words<NW>(p.spec_cells + static_cast<size_t>(slot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(col[b]), wb[b]);
          }
          uint32_t v = 0;  // the other player's input of frame f
          if (any_own) {
            const int j = f - base;
            if (j < kFanPre) v = fan_input(vpk, j);
            else if (own_local || (la_own != kNullFrame && f <= la_own)) v = ring.get(f, h_own, s);  // Confirmed
            else v = pred_own;  // repeat-last prediction (blank before the first input)
          }
          const InRec vo = static_cast<InRec>(static_cast<uint64_t>(v) << (8 * h_own));
#pragma unroll
          for (int b = 0; b < NG; ++b) adv(wb[b], own[b] ? vo : in[b], own[b] ? h_own : rs);
        }
#pragma unroll
        for (int b = 0; b < NG; ++b)
          if (on[b] || own[b]) store_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(col[b]), wb[b]);
      };
      // the slots the wave runs: the most any of its lanes needs
      constexpr int kMaxSlots = (kSpecBranches + P - 1 + static_cast<int>(L) - 1) / static_cast<int>(L);
      int ns = 0;
#pragma unroll
      for (int sb = 0; sb < kMaxSlots; ++sb) ns += __any(sb < nslots) ? 1 : 0;
#pragma unroll
      for (int b0 = 0; b0 < kMaxSlots; b0 += kFanGroup) {
        const int ng = min(kFanGroup, ns - b0);
        if (ng <= 0) break;
        const bool last = b0 + ng == ns;
        if (ng == 1) group(std::integral_constant<int, 1>{}, b0, last);
        else if (ng == 2 || kFanGroup == 2) group(std::integral_constant<int, 2>{}, b0, last);
        else if (ng == 3 || kFanGroup == 3) group(std::integral_constant<int, 3>{}, b0, last);
        else group(std::integral_constant<int, (kFanGroup >= 4 ? 4 : 3)>{}, b0, last);
      }
      tot_branch += static_cast<uint32_t>(cur - base) * static_cast<uint32_t>(nb);
    }
  };
  auto tick_rotate = [&]() __attribute__((always_inline)) {  // the prefetched deliveries become the next tick's
    if constexpr (kPrefetch) {
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        up[j] = up_n[j];
        lin[j] = lin_n[j];
#pragma unroll
        for (int k = 0; k < kPre; ++k) rv[j][k] = rv_n[j][k];
        if constexpr (kWire) pre0[j] = pre_n[j];
      }
    }
  };
  auto tick = [&](int t) __attribute__((always_inline)) -> bool {
    const int r = tick_begin(t);
    RB_PH(2);
    if (r == 0) return false;
    if (r == 2) {
      rollback_and_save();
      RB_PH(3);
      if (status == kP2PStatusPanic) return false;
      if (!run_desync()) {
        status = kP2PStatusPanic;
        return false;
      }
      add_local();
      advance(cur);
      next_frame();
#if RB_P2P_PHASE
      settle(w[0]);
#endif
      RB_PH(4);
    }
    if (in_fan) fan_inlane();
    tick_rotate();
    return true;
  };
#if RB_P2P_PRIO
  const uint32_t wslot = wave_turn_key() & 3u;  // (kernels.hpp prio_turn: two-level turns, measured
                                                // better than the rotation at 4 waves per SIMD here)
#endif
  if constexpr (!kAsync) {
    for (int t = 0; t < T; ++t) {
#if RB_P2P_PRIO
      if (T > 1) prio_turn(wslot);
#endif
      if (!tick(t)) break;
    }
  } else {
    // lane-asynchronous ticks (see kAsync above): one AdvanceFrame per session per iteration
    int t = 0, count = 0, i = 0;
    int32_t confirmed = 0;
    bool inres = false, stopped = false;
    [[maybe_unused]] bool checked = false;  // kSparse: check_last_saved_state already ran this tick
    [[maybe_unused]] uint32_t iters = 0;
    while (inres || (!stopped && t < p.T)) {
#if RB_P2P_PRIO
      prio_turn(wslot);
#endif
      if constexpr (RB_P2P_EXP & 4) ++iters;
      if (!inres) {  // the next tick's opening, up to its rollback's LoadGameState
        const int r = tick_begin(t);
        if (r == 0) {
          stopped = true;
        } else if (r == 1) {
          tick_rotate();
          ++t;
        } else {
          int32_t first_inc;
          rollback_open(confirmed, first_inc);
          count = 0;
          if (first_inc != INT32_MAX) {
            count = adjust_begin(first_inc);
            disc_frame = kNullFrame;
          }
          if (status == kP2PStatusPanic) stopped = true;
          else inres = true, i = 0, checked = false;
        }
      }
      if constexpr (kSparse) {
        // check_last_saved_state (p2p_session.rs:778-802), once the first rollback is done: a save of
        // the current frame, or a second rollback from the last saved frame (its frames follow)
        if (inres && i >= count && !checked) {
          checked = true;
          if (cur - last_saved >= W) {
            if (confirmed >= cur) {
              save(cur);
            } else {
              count = adjust_begin(last_saved);
              i = 0;
              if (status == kP2PStatusPanic) stopped = true, inres = false;
            }
          }
        }
      }
      if (inres) {
        bool save_now, finish = false;
        if (i < count) {  // resimulated frame i of adjust_gamestate (sparse: the frame min_confirmed is saved)
          save_now = kSparse ? cur == confirmed : i > 0;
          ++i;
        } else {  // the rest of advance_frame, add_local_input, then the tick's new frame
          set_last_confirmed(confirmed);
          add_local();
          save_now = !kSparse;  // rollback_and_save's SaveGameState of the current frame (not with sparse saving)
          finish = true;
          inres = false;
        }
        if (save_now) save(cur);
        advance(cur);
        next_frame();
        if (finish) {
          tick_rotate();
          ++t;
        }
      }
    }
    if constexpr (RB_P2P_EXP & 4) {  // attribution builds: loop iterations of the wave (max over its lanes)
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) iters = max(iters, static_cast<uint32_t>(__shfl_xor(static_cast<int>(iters), m, 64)));
      if (__lane_id() == 0) atomicAdd(&p.counters[1], iters);  // reported as the unexpected-path count
    }
  }

  // ---- LDS queue: the frames added in this launch back to the HBM ring
  if constexpr (kLdsQ) {
    const int h = player_of(0);
    const int32_t la = q[0].last_added;
    if (h < P && la != kNullFrame) {
      for (int32_t f = max(la0 == kNullFrame ? 0 : la0 + 1, la - (kQueueLen - 1)); f <= la; ++f) hbm.put(f, h, s, ring.get(f, h, s));
    }
  }
  // ---- write back
  if constexpr (kLdsC) {  // the snapshot ring
    for (int k = 0; k < W; ++k) {
      const unsigned kk = static_cast<unsigned>(k);
      uint32_t cw[NW];
#pragma unroll
      for (int n = 0; n < NW; ++n) cw[n] = lds_cell[(kk * NW + n) * bd + tid];
      store_words<NW>(p.snap + kk * slot_words, static_cast<int>(Gpad), static_cast<int>(g), cw);
      if (lead) {
        csa[kk * Spad + s] = lds_cs[kk * bps + sl];
        p.tag[kk * Spad + s] = lds_tag[kk * bps + sl];
      }
    }
  }
  store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int h = player_of(j);
    if (h >= P) continue;
    const QFields f{q[j].last_added, q[j].conn_last, q[j].pred_frame, q[j].first_inc, q[j].last_req,
                    q[j].tail,       q[j].len,       q[j].disc,       q[j].pred_val};
    const QPacked pk = q_pack(f, cur);
#pragma unroll
    for (int i = 0; i < 4; ++i) *qrow(QF_LA_CONN + i, h) = static_cast<int32_t>(pk.w[i]);
    if constexpr (IB > 1) *qrow(QF_PRED_VAL, h) = static_cast<int32_t>(q[j].pred_val);
    if (pk.esc) {
      const int32_t ab[7] = {f.la, f.conn, f.pred, f.fi, f.req, f.tail, f.len};
#pragma unroll
      for (int i = 0; i < 7; ++i) *qrow(QF_ABS0 + i, h) = ab[i];
    }
    if constexpr (kSpec && kMtf) {
      {
        *qrow(QF_MTF0, h) = static_cast<int32_t>(q[j].mlo);
        *qrow(QF_MTF0 + 1, h) = static_cast<int32_t>(q[j].mlo >> 32);
        *qrow(QF_MTF0 + 2, h) = static_cast<int32_t>(q[j].mhi);
        *qrow(QF_MTF0 + 3, h) = static_cast<int32_t>(q[j].mhi >> 32);
        *qrow(QF_MTF_N, h) = q[j].mn;
      }
    }
  }
  if constexpr (kWire) {  // the last tick's decode status and the newest frame received per endpoint (the ack)
    if (p.pk_status) {
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const int h = player_of(j);
        if (h < P && !((p.local_mask >> h) & 1u)) p.pk_status[static_cast<size_t>(h) * p.S + s] = pk_ds[j];
      }
    }
    if (p.acks) {
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const int h = player_of(j);
        if (h < P && !((p.local_mask >> h) & 1u)) p.acks[static_cast<size_t>(h) * p.S + s] = q[j].conn_last;
      }
    }
  }
  // The work counters by return-less atomics at the L2 (a load, add and store would put one more
  // memory round trip at the end of every wave: one-tick launches at 1,048,576 sessions, eight waves
  // per SIMD slot in turn, 140 -> 111 us without the counter traffic, attribution build 64).  Only
  // their sums are ever read (rb_p2p_totals, the adaptive fan-out's measurement), so a wave whose
  // lanes are all here adds its sessions' counts up first (cross-lane sums) and its first lane adds
  // them to the wave's first session's column: one atomic per counter and wave instead of one per
  // counter and session.  A wave with lanes gone (a panicked session, the padding past S) adds per
  // session as before.
  [[maybe_unused]] bool wave_summed = false;
  if constexpr (!(RB_P2P_EXP & 64)) {
    if (__ballot(1) == ~0ull) {
      uint32_t c[4] = {lead ? tot_adv : 0u, lead ? tot_save : 0u, lead ? tot_load : 0u, lead ? tot_sel : 0u};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) c[i] += static_cast<uint32_t>(__shfl_xor(static_cast<int>(c[i]), o, 64));
      if ((g & 63u) == 0) {
        const unsigned s0 = s;  // the wave's first session
        atomicAdd(&p.stats[ST_ADV * Spad + s0], static_cast<unsigned long long>(c[0]));
        atomicAdd(&p.stats[ST_SAVE * Spad + s0], static_cast<unsigned long long>(c[1]));
        if (c[2]) atomicAdd(&p.stats[ST_LOAD * Spad + s0], static_cast<unsigned long long>(c[2]));
        if (c[3]) atomicAdd(&p.stats[ST_SELECT * Spad + s0], static_cast<unsigned long long>(c[3]));
      }
      wave_summed = true;
    }
  }
  if (lead) {
    p.qs[QS_CUR * Spad + s] = cur;
    const bool sesc = !(fd_fits(last_saved, cur) && fd_fits(last_conf, cur));
    p.qs[QS_SAVED_CONF * Spad + s] = static_cast<int32_t>(sesc ? kQsEscWord : fd_enc(last_saved, cur) | fd_enc(last_conf, cur) << 16);
    if (sesc) {
      p.qs[QS_ABS_SAVED * Spad + s] = last_saved;
      p.qs[QS_ABS_CONF * Spad + s] = last_conf;
    }
    if (disc_frame != disc_frame0) p.qs[QS_DISC_FRAME * Spad + s] = disc_frame;
    if (status != status0) p.status[s] = status;
    if (status == kP2PStatusPanic) atomicAdd(&p.counters[2], 1u);
    if (n_thr) atomicAdd(&p.counters[0], n_thr);
    if constexpr (!(RB_P2P_EXP & 64)) {  // (attribution builds: 64 drops the trace and work-counter traffic)
      p.trace[s] = static_cast<int32_t>(trace_pack(load_frame, nadv, nsave, cur));
      if (!wave_summed) {
        atomicAdd(&p.stats[ST_ADV * Spad + s], static_cast<unsigned long long>(tot_adv));
        atomicAdd(&p.stats[ST_SAVE * Spad + s], static_cast<unsigned long long>(tot_save));
        if (tot_load) atomicAdd(&p.stats[ST_LOAD * Spad + s], static_cast<unsigned long long>(tot_load));
        if (tot_sel) atomicAdd(&p.stats[ST_SELECT * Spad + s], static_cast<unsigned long long>(tot_sel));
      }
    }
    if constexpr (kInFan) {
      if (in_fan) {  // the branches' metadata for the next launch's first tick
        if (tot_branch) atomicAdd(&p.stats[ST_BRANCH * Spad + s], static_cast<unsigned long long>(tot_branch));
        p.spec_meta[SM_BASE * Spad + s] = sm_base;
        p.spec_meta[SM_END * Spad + s] = sm_end;
        p.spec_meta[SM_PLAYER * Spad + s] = sm_player;
        p.spec_meta[SM_VALID * Spad + s] = sm_valid;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          if (!p.spec_per_player) p.spec_meta[(SM_CAND + qq) * Spad + s] = static_cast<int32_t>(sm_cand[qq]);
      }
    }
  }
  if constexpr (kInFan && !kMtf) {  // per-player fan-out: each lane writes its own player's base row
    if (in_fan && p.spec_per_player) p.spec_meta[(SM_CAND + lane) * Spad + s] = sm_pbase;
  }
  if (p.launch_clock) launch_clock_put(p.launch_clock, g / 64u, 1u);
#if RB_P2P_PHASE
  RB_PH(5);
  if (p.T == 1 && (g & 63u) == 0 && g / 64 < 4096) {
#pragma unroll
    for (int i = 0; i < 6; ++i) rb_p2p_phase[8 * (g / 64) + i] = ph[i];
    rb_p2p_phase[8 * (g / 64) + 6] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF814)) << 32 | __builtin_amdgcn_s_getreg(0xF804);
    rb_p2p_phase[8 * (g / 64) + 7] = static_cast<uint64_t>(tot_load) << 32 | tot_adv;
  }
#endif
}
#if RB_P2P_PHASE
extern "C" int rb_debug_p2p_phase(uint64_t* host_out, int n) {
  return static_cast<int>(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(rb_p2p_phase), sizeof(uint64_t) * 8 * min(n, 4096)));
}
#endif

// ---------------------------------------------------------------------------
// Speculative branch fan-out (BASELINE config 4).  After a
// tick, for every session: take the remote handle with the oldest unconfirmed
// input (the speculated player), its first unconfirmed frame `base`, and
// presimulate kSpecBranches branches from the saved cell of `base` up to the
// current frame: branch k feeds candidate k to the speculated player on every
// frame of the window and, for everybody else, exactly the inputs a rollback
// would use (confirmed inputs, the reference's repeat-last predictions).  Each
// branch saves its cells like adjust_gamestate would.  One lane group (a
// branch) per candidate, one lane per player: 16 x L lanes per session, all
// branches in lock-step.  The next tick's p2p_kernel turns a matching
// misprediction into a select (try_select) instead of a resimulation.
// ---------------------------------------------------------------------------
struct FanParams {
  const int32_t* status;  // [Spad] rb_status of the last advance_frame (panicked sessions are skipped)
  const uint32_t* snap;
  const int32_t* tag;
  const void* ring;
  const int32_t* qs;
  uint32_t* spec_state;
  uint32_t* spec_cells;
  void* spec_cs;
  int32_t* spec_meta;
  unsigned long long* stats;  // [ST_COUNT][Spad], ST_BRANCH column
  uint32_t* counters;
  int32_t S, Spad, W;
  uint32_t local_mask;
  int32_t fan_generic;  // fanout_kernel even for independent players
  int32_t fan_k;        // candidates (branches) per session, <= kSpecBranches
  unsigned long long* launch_clock;  // rb_p2p_launch_clock_arm: this launch's [waves][start, end], or null
};

template <class G>
__global__ void __launch_bounds__(256) fanout_kernel(const FanParams p) {
  using InRec = typename G::InRec;
  using CS = typename G::CS;
  constexpr int NW = G::NWL;
  constexpr int L = G::kLanes;
  constexpr int P = G::kPlayers, IB = G::kInputBytes;
  static_assert(L > 1 || P == 1, "fan-out runs with one lane per player (or a wave per session)");
  constexpr int LS = kSpecBranches * L;  // lanes per session
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned s = g / LS;
  const int r = static_cast<int>(g % LS);
  const int k = r / L, lane = r % L;  // branch = candidate input, player slot
  if (p.launch_clock) launch_clock_put(p.launch_clock, g / 64u, 0u);
  if (s >= static_cast<unsigned>(p.S)) return;
  const unsigned Spad = static_cast<unsigned>(p.Spad), Gpad = Spad * L;
  const unsigned Gs = Gpad * kSpecBranches;  // spec plane width: column = this thread's index g
  const int W = p.W;
  const RingIO<IB> ring{const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(p.ring)), P, p.Spad};
  auto qrow = [&](int field, int h) { return p.qs[static_cast<size_t>(QS_PLAYER0 + field * 4 + h) * Spad + s]; };
  const int32_t cur = p.qs[QS_CUR * Spad + s];
  auto last_added_of = [&](int h) {  // InputQueue::last_added_frame from the packed rows (q_unpack)
    const uint32_t m = static_cast<uint32_t>(qrow(QF_MISC, h));
    return (m & kQmEsc) ? qrow(QF_ABS0, h) : fd_dec(static_cast<uint32_t>(qrow(QF_LA_CONN, h)), cur);
  };
  // the remote handle with the oldest last added input (ties: lowest handle)
  int rs = -1;
  int32_t la_rs = INT32_MAX;
#pragma unroll
  for (int h = 0; h < P; ++h) {
    if ((p.local_mask >> h) & 1u) continue;
    const int32_t la = last_added_of(h);
    const int32_t key = la == kNullFrame ? -1 : la;
    if (key < la_rs) {
      la_rs = key;
      rs = h;
    }
  }
  bool any_disc = false;
#pragma unroll
  for (int h = 0; h < P; ++h) any_disc |= (static_cast<uint32_t>(qrow(QF_MISC, h)) & kQmDisc) != 0;
  const int32_t base = la_rs + 1;  // first unconfirmed frame of the speculated player
  const bool valid = p.status[s] != kP2PStatusPanic && !any_disc && rs >= 0 && base < cur && base + W > cur && base >= 0 &&
                     p.tag[static_cast<unsigned>(base % W) * Spad + s] == base;
  uint32_t cand[4];  // the speculated player's candidates (every lane of the session computes the same)
  {
    const int hr = max(rs, 0);
    const uint64_t mlo = static_cast<uint32_t>(qrow(QF_MTF0, hr)) | static_cast<uint64_t>(static_cast<uint32_t>(qrow(QF_MTF0 + 1, hr))) << 32;
    const uint64_t mhi = static_cast<uint32_t>(qrow(QF_MTF0 + 2, hr)) | static_cast<uint64_t>(static_cast<uint32_t>(qrow(QF_MTF0 + 3, hr))) << 32;
    fan_candidates(mlo, mhi, qrow(QF_MTF_N, hr), InputAlphabet<G>::value, p.fan_k, cand);
  }
  if (k == 0 && lane == 0) {
    p.spec_meta[SM_BASE * Spad + s] = base;
    p.spec_meta[SM_END * Spad + s] = cur;
    p.spec_meta[SM_PLAYER * Spad + s] = rs;
    p.spec_meta[SM_VALID * Spad + s] = valid ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) p.spec_meta[(SM_CAND + q) * Spad + s] = static_cast<int32_t>(cand[q]);
  }
  if (!valid || k >= p.fan_k) {  // session-uniform (branch-uniform): the whole group leaves
    if (p.launch_clock) launch_clock_put(p.launch_clock, g / 64u, 1u);
    return;
  }
  const uint32_t ck = cand_at(cand, k);
  const unsigned gl = s * L + lane;  // this lane's column in the session-major planes
  uint32_t w[NW];
  load_words<NW>(p.snap + static_cast<unsigned>(base % W) * NW * Gpad, static_cast<int>(Gpad), static_cast<int>(gl), w);
  // this lane's player: its inputs over the window, as adjust_gamestate would see them
  const int h = lane;
  const bool active = h < P;
  const bool local = active && ((p.local_mask >> h) & 1u);
  const int32_t la_h = active ? last_added_of(h) : kNullFrame;
  const uint32_t pred = (!active || la_h == kNullFrame) ? 0u : ring.get(la_h, h, s);
  uint32_t vin[kFanPre];
  fan_prefetch(ring, active ? h : 0, s, base, cur, local, la_h, pred, vin);
  const uint64_t vpk = fan_pack(vin);
  CS* __restrict__ cs = reinterpret_cast<CS*>(p.spec_cs);
  uint32_t frames = 0;
  for (int32_t f = base; f < cur; ++f) {
    if (f > base) {  // SaveGameState of frame f (adjust_gamestate saves every frame but the loaded one)
      CsCtx ctx{0ull, s, 0u};
      const CS c = G::checksum(w, f, lane, ctx);
      const unsigned slot = static_cast<unsigned>(f % W);
      store_words<NW>(p.spec_cells + static_cast<size_t>(slot) * NW * Gs, static_cast<int>(Gs), static_cast<int>(g), w);
      if (lane == 0) cs[(slot * Spad + s) * kSpecBranches + k] = c;
    }
    uint32_t v = 0;
    if (active) {
      const int j = f - base;
      if (h == rs) v = ck;
      else if (j < kFanPre) v = fan_input(vpk, j);
      else if (local || (la_h != kNullFrame && f <= la_h)) v = ring.get(f, h, s);  // Confirmed
      else v = pred;  // repeat-last prediction (blank before the first input)
    }
    advance_frame<G>(w, static_cast<InRec>(static_cast<uint64_t>(v) << (8 * IB * (active ? h : 0))), lane, 0u,
                     &p.counters[1]);
    ++frames;
  }
  store_words<NW>(p.spec_state, static_cast<int>(Gs), static_cast<int>(g), w);
  if (k == 0 && lane == 0 && frames)
    atomicAdd(&p.stats[ST_BRANCH * Spad + s], static_cast<unsigned long long>(frames) * p.fan_k);  // (no load round trip)
  if (p.launch_clock) launch_clock_put(p.launch_clock, g / 64u, 1u);
}

}  // namespace rb
