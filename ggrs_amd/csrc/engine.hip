// ggrs_amd/csrc/engine.hip — MI355X batched rollback-resimulation engine.
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
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ggrs_amd.h"
#include "games.hpp"
#include "planner.hpp"

namespace rb {

constexpr int kChunk = 8;  // inputs prefetched per chunk of AdvanceFrames
constexpr int kMaxRepl = 8;

struct KParams {
  uint32_t* snap;
  uint32_t* live;
  void* cs;
  void* fs;
  void* ring;
  void* last_cs;
  void* periodic_cs;
  int32_t* err;
  int32_t* live_frame;
  unsigned long long* frozen;
  uint32_t* counters;  // [0] sessions failed, [1] unexpected-path count
  const void* in_ptr[4];
  int32_t in_mode;  // 0: no new input, 1: one array per player, 2: packed [S][P]
  int32_t S, Spad, W;
  int32_t user_slot, n_repl, repl_src;
  int32_t repl_dst[kMaxRepl];
  int32_t load_slot;  // -1: start from the live state
  int32_t f0, n_steps;
  uint32_t save_modes[kMaxSteps / 16];  // 2 bits per step
  int32_t slot0;                        // f0 % W (snapshot slot of step 0)
  int32_t live_out, periodic_step, display;
  uint32_t disc_mask;
  uint64_t seed;
  uint32_t nonce_base;
  uint32_t debug;  // experiment knobs (rb_config.reserved[0]); 0 in every real run
};

// ---- SoA planes: word k of session s inside a block of NW planes -------------
template <int NW>
__device__ __forceinline__ void load_words(const uint32_t* __restrict__ base, int Spad, int s, uint32_t (&w)[NW]) {
  constexpr int Q4 = NW / 4, R = NW % 4;
#pragma unroll
  for (int j = 0; j < Q4; ++j) {
    const uint4 v = reinterpret_cast<const uint4*>(base + j * 4 * Spad)[s];
    w[4 * j + 0] = v.x;
    w[4 * j + 1] = v.y;
    w[4 * j + 2] = v.z;
    w[4 * j + 3] = v.w;
  }
  const uint32_t* b = base + Q4 * 4 * Spad;
  if constexpr (R >= 2) {
    const uint2 v = reinterpret_cast<const uint2*>(b)[s];
    w[Q4 * 4 + 0] = v.x;
    w[Q4 * 4 + 1] = v.y;
    b += 2 * Spad;
  }
  if constexpr (R & 1) w[NW - 1] = b[s];
}
template <int NW>
__device__ __forceinline__ void store_words(uint32_t* __restrict__ base, int Spad, int s, const uint32_t (&w)[NW]) {
  constexpr int Q4 = NW / 4, R = NW % 4;
#pragma unroll
  for (int j = 0; j < Q4; ++j)
    reinterpret_cast<uint4*>(base + j * 4 * Spad)[s] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
  uint32_t* b = base + Q4 * 4 * Spad;
  if constexpr (R >= 2) {
    reinterpret_cast<uint2*>(b)[s] = make_uint2(w[Q4 * 4], w[Q4 * 4 + 1]);
    b += 2 * Spad;
  }
  if constexpr (R & 1) b[s] = w[NW - 1];
}
// host mirror of the plane layout
inline size_t word_index(int NW, int Spad, int s, int k) {
  const int Q4 = NW / 4, R = NW % 4;
  if (k < Q4 * 4) return static_cast<size_t>(k / 4) * 4 * Spad + static_cast<size_t>(s) * 4 + (k % 4);
  size_t b = static_cast<size_t>(Q4) * 4 * Spad;
  if (R >= 2) {
    if (k < Q4 * 4 + 2) return b + static_cast<size_t>(s) * 2 + (k - Q4 * 4);
    b += 2 * static_cast<size_t>(Spad);
  }
  return b + s;
}

// New inputs of this tick.  kPacked: one [S][P] array; else one [S] array per
// handle.  The host always passes valid pointers (a dummy when there is no new
// input), so the loads are unconditional and issue with the others.
template <class G, bool kPacked>
__device__ __forceinline__ typename G::InRec gather_new_input(const KParams& p, unsigned s) {
  using InRec = typename G::InRec;
  constexpr int P = G::kPlayers, IB = G::kInputBytes;
  if constexpr (kPacked && sizeof(InRec) == P * IB) {
    return reinterpret_cast<const InRec*>(p.in_ptr[0])[s];
  } else {
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      uint64_t x = 0;
      if constexpr (kPacked) {
        const uint8_t* b = reinterpret_cast<const uint8_t*>(p.in_ptr[0]) + (s * P + q) * IB;
#pragma unroll
        for (int i = 0; i < IB; ++i) x |= static_cast<uint64_t>(b[i]) << (8 * i);
      } else if constexpr (IB == 4) {
        x = reinterpret_cast<const uint32_t*>(p.in_ptr[q])[s];
      } else {
        x = reinterpret_cast<const uint8_t*>(p.in_ptr[q])[s];
      }
      v |= x << (8 * IB * q);
    }
    return static_cast<InRec>(v);
  }
}

__host__ __device__ inline U128 to_u128(uint16_t c) { return U128{c, 0}; }
__host__ __device__ inline U128 to_u128(uint64_t c) { return U128{c, 0}; }
__host__ __device__ inline U128 to_u128(U128 c) { return c; }

// snapshot slot of step k: (f0 + k) % W with f0 % W precomputed (k < 2W)
__device__ __forceinline__ unsigned step_slot(const KParams& p, int k) {
  int sl = p.slot0 + k;
  sl = sl >= p.W ? sl - p.W : sl;
  sl = sl >= p.W ? sl - p.W : sl;
  return static_cast<unsigned>(sl);
}

// The fused tick.  Thread g serves lane (g % L) of session g / L; a session's
// state slice stays in that lane's VGPRs for the whole tick.  Phase 1 issues
// every load of the tick (frozen mask, new inputs, the loaded snapshot, the
// inputs of every step, the first-seen checksums) before any store: on CDNA
// vmcnt counts loads and stores in issue order, so a load issued after a
// store would make its consumer wait for the store too.  Phase 2 performs the
// input-queue writes, phase 3 runs the request stream: per step [SAVE:
// checksum (lane-group DPP sum) + snapshot store + first-seen record/compare]
// ADVANCE.
template <class G, bool kPacked>
__global__ void __launch_bounds__(256) tick_kernel(const KParams p) {
  using InRec = typename G::InRec;
  using CS = typename G::CS;
  constexpr int NW = G::NWL;
  constexpr unsigned L = G::kLanes;
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned s = g / L;
  const int lane = static_cast<int>(g % L);
  const bool lead = lane == 0;
  if (s >= static_cast<unsigned>(p.S)) return;
  {
    const unsigned wave0 = __builtin_amdgcn_readfirstlane(s) & ~63u;
    const unsigned long long fw = p.frozen[wave0 >> 6];
    if ((fw >> (s & 63)) & 1ull) return;  // advance_frame keeps returning Err for this session
  }
  if (p.debug & 8u) return;  // launch floor (experiment)
  const unsigned Spad = static_cast<unsigned>(p.Spad);
  const unsigned Gpad = Spad * L;  // lane planes
  InRec* __restrict__ ring = reinterpret_cast<InRec*>(p.ring);
  CS* __restrict__ csa = reinterpret_cast<CS*>(p.cs);
  const CS* __restrict__ fsa = reinterpret_cast<const CS*>(p.fs);
  const unsigned slot_words = static_cast<unsigned>(NW) * Gpad;

  // ---- phase 1: loads
  const bool has_new = p.in_mode != 0 && p.user_slot >= 0;
  const InRec newin = gather_new_input<G, kPacked>(p, s);
  const InRec replv = ring[static_cast<unsigned>(p.repl_src) * Spad + s];
  uint32_t w[NW];
  if (p.load_slot >= 0)
    load_words<NW>(p.snap + static_cast<unsigned>(p.load_slot) * slot_words, static_cast<int>(Gpad), static_cast<int>(g), w);
  else
    load_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);

  InRec in[kChunk];
  CS fsv[kChunk];
  auto prefetch = [&](int base) {
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const int kk = base + k < p.n_steps ? base + k : base;  // clamp: always a valid address
      in[k] = ring[static_cast<unsigned>((p.f0 + kk) & (kQueueLen - 1)) * Spad + s];
      fsv[k] = fsa[step_slot(p, kk) * Spad + s];
    }
  };
  prefetch(0);

  // ---- phase 2: InputQueue::add_input for every handle (input_queue.rs:149-239):
  // delay-fill replication, then the new inputs at frame current + delay.
  if (lead) {
    for (int r = 0; r < p.n_repl; ++r) ring[static_cast<unsigned>(p.repl_dst[r]) * Spad + s] = replv;
    if (has_new) ring[static_cast<unsigned>(p.user_slot) * Spad + s] = newin;
  }
  auto patch = [&](int base) {  // prefetched slots that phase 2 just wrote
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const int slot = (p.f0 + base + k) & (kQueueLen - 1);
      for (int r = 0; r < p.n_repl; ++r)
        if (slot == p.repl_dst[r]) in[k] = replv;
      if (has_new && slot == p.user_slot) in[k] = newin;
    }
  };
  patch(0);

  // ---- phase 3: the request stream
  CsCtx ctx{p.seed, s, p.nonce_base};
  int32_t mismatch = kNullFrame;
  for (int base = 0; base < p.n_steps; base += kChunk) {
    if (base > 0) {
      prefetch(base);
      patch(base);
    }
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const int step = base + k;
      if (step >= p.n_steps) break;
      const int32_t f = p.f0 + step;
      const uint32_t mode = (p.save_modes[step >> 4] >> ((step & 15) * 2)) & 3u;
      if (mode != SAVE_NONE) {  // SaveGameState{cell, f}: checksum, cell.save
        ctx.nonce = p.nonce_base + static_cast<uint32_t>(step);
        const CS c = (p.debug & 4u) ? CS{} : G::checksum(w, f, lane, ctx);
        const unsigned slot = step_slot(p, step);
        if (!(p.debug & 2u))
          store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), w);
        if (lead) csa[slot * Spad + s] = c;
        if (mode == SAVE_RECORD) {
          if (lead) reinterpret_cast<CS*>(p.fs)[slot * Spad + s] = c;
        } else if (mode == SAVE_COMPARE) {
          if (c != fsv[k]) mismatch = f;  // newest mismatching frame wins
        }
      }
      if (p.debug & 1u)
        w[0] += in[k];
      else
        G::advance(w, in[k], lane, p.disc_mask, &p.counters[1]);  // AdvanceFrame{inputs}
      if (step == p.periodic_step) {
        ctx.nonce = p.nonce_base + 128u + static_cast<uint32_t>(step);
        const CS c = G::checksum(w, f + 1, lane, ctx);
        if (lead) reinterpret_cast<CS*>(p.periodic_cs)[s] = c;
      }
    }
  }
  if (p.display) {  // Game::last_checksum after the final AdvanceFrame (ex_game.rs:104-108)
    ctx.nonce = p.nonce_base + 255u;
    const CS c = G::checksum(w, p.f0 + p.n_steps, lane, ctx);
    if (lead) reinterpret_cast<CS*>(p.last_cs)[s] = c;
  }
  if (p.live_out || mismatch != kNullFrame) store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);
  if (mismatch != kNullFrame && lead) {
    p.err[s] = mismatch;
    p.live_frame[s] = p.f0 + p.n_steps;  // the session stops at the end of this tick
    atomicOr(&p.frozen[s >> 6], 1ull << (s & 63));
    atomicAdd(&p.counters[0], 1u);
  }
}

// ---------------------------------------------------------------------------
// Fused steady-state SyncTest ticks (rb_run_ticks).  For current frame c > cd
// the reference's stream is always (sync_test_session.rs:89-132, 178-203)
//   Load(c-cd), Adv, [Save(f) Adv] for f = c-cd+1 .. c-1, Save(c), Adv
// so T consecutive such ticks run in ONE launch with the shape known at
// compile time (CD = check distance): no per-tick launch, no per-step control
// flow, and each wave keeps its sessions across ticks (the slot it loads was
// written by the same lanes one tick earlier, so it is L2-hot).  Every
// request still executes against memory exactly as in tick_kernel: the
// snapshot is loaded from its cell, every save stores the cell, the inputs
// come from the input queue ring.  The host bookkeeping runs per tick as
// usual; only ticks whose lowered program has exactly this shape are fused.
struct RunParams {
  uint32_t* snap;
  void* cs;
  void* fs;
  void* ring;
  void* last_cs;
  void* periodic_cs;
  uint32_t* live;
  int32_t* err;
  int32_t* live_frame;
  unsigned long long* frozen;
  uint32_t* counters;
  const uint8_t* in_base;  // tick t, player q: in_base + t*in_stride + q*S*kInputBytes
  int64_t in_stride;
  int32_t S, Spad, W, delay;
  int32_t c0, T;            // current frame of the first fused tick, tick count
  uint32_t tick0;           // engine tick index of the first fused tick (nonce)
  int32_t live_out_last;    // store the live state after the last tick
  uint64_t seed;
};

template <class G, int CD>
__global__ void __launch_bounds__(256) steady_kernel(const RunParams p) {
  static_assert(CD >= 1, "steady shape needs a rollback");
  using InRec = typename G::InRec;
  using CS = typename G::CS;
  constexpr int NW = G::NWL;
  constexpr unsigned L = G::kLanes;
  constexpr int P = G::kPlayers, IB = G::kInputBytes;
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned s = g / L;
  const int lane = static_cast<int>(g % L);
  const bool lead = lane == 0;
  if (s >= static_cast<unsigned>(p.S)) return;
  {
    const unsigned wave0 = __builtin_amdgcn_readfirstlane(s) & ~63u;
    if ((p.frozen[wave0 >> 6] >> (s & 63)) & 1ull) return;
  }
  const unsigned Spad = static_cast<unsigned>(p.Spad), Gpad = Spad * L;
  const unsigned slot_words = static_cast<unsigned>(NW) * Gpad;
  InRec* __restrict__ ring = reinterpret_cast<InRec*>(p.ring);
  CS* __restrict__ csa = reinterpret_cast<CS*>(p.cs);
  CS* __restrict__ fsa = reinterpret_cast<CS*>(p.fs);
  const int W = p.W;
  auto slot_of = [W](int f) { return static_cast<unsigned>(f % W); };

  for (int t = 0; t < p.T; ++t) {
    const int c = p.c0 + t;
    const int f0 = c - CD;
    // ---- loads of the tick
    const uint8_t* tin = p.in_base + static_cast<int64_t>(t) * p.in_stride;
    uint64_t nv = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      uint64_t x;
      if constexpr (IB == 4)
        x = reinterpret_cast<const uint32_t*>(tin + static_cast<size_t>(q) * p.S * IB)[s];
      else
        x = tin[static_cast<size_t>(q) * p.S + s];
      nv |= x << (8 * IB * q);
    }
    const InRec newin = static_cast<InRec>(nv);
    uint32_t w[NW];
    load_words<NW>(p.snap + slot_of(f0) * slot_words, static_cast<int>(Gpad), static_cast<int>(g), w);
    InRec in[CD + 1];
#pragma unroll
    for (int k = 0; k <= CD; ++k) in[k] = ring[static_cast<unsigned>((f0 + k) & (kQueueLen - 1)) * Spad + s];
    CS fsv[CD > 1 ? CD - 1 : 1];
#pragma unroll
    for (int k = 1; k < CD; ++k) fsv[k - 1] = fsa[slot_of(f0 + k) * Spad + s];
    // ---- InputQueue::add_input for every handle: the new inputs at c + delay
    const unsigned uslot = static_cast<unsigned>((c + p.delay) & (kQueueLen - 1));
    if (lead) ring[uslot * Spad + s] = newin;
    if (p.delay == 0) in[CD] = newin;
    // ---- the request stream
    const uint32_t nonce = ((p.tick0 + static_cast<uint32_t>(t)) & 0xffffffu) << 8;
    CsCtx ctx{p.seed, s, nonce};
    int32_t mismatch = kNullFrame;
#pragma unroll
    for (int k = 0; k <= CD; ++k) {
      const int f = f0 + k;
      if (k > 0) {  // SaveGameState{cell, f}
        ctx.nonce = nonce + static_cast<uint32_t>(k);
        const CS cval = G::checksum(w, f, lane, ctx);
        const unsigned slot = slot_of(f);
        store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), w);
        if (lead) csa[slot * Spad + s] = cval;
        if (k == CD) {
          if (lead) fsa[slot * Spad + s] = cval;  // first save of frame c: first-seen
        } else if (cval != fsv[k - 1]) {
          mismatch = f;  // newest mismatching frame wins
        }
      }
      G::advance(w, in[k], lane, 0u, &p.counters[1]);  // AdvanceFrame{inputs}
      if ((f + 1) % 100 == 0) {  // ex_game periodic_checksum (frame % CHECKSUM_PERIOD == 0)
        ctx.nonce = nonce + 128u + static_cast<uint32_t>(k);
        const CS cval = G::checksum(w, f + 1, lane, ctx);
        if (G::kDisplay && lead) reinterpret_cast<CS*>(p.periodic_cs)[s] = cval;
      }
    }
    if constexpr (G::kDisplay) {  // Game::last_checksum after the final AdvanceFrame
      ctx.nonce = nonce + 255u;
      const CS cval = G::checksum(w, c + 1, lane, ctx);
      if (lead) reinterpret_cast<CS*>(p.last_cs)[s] = cval;
    }
    if (mismatch != kNullFrame) {
      store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);
      if (lead) {
        p.err[s] = mismatch;
        p.live_frame[s] = c + 1;
        atomicOr(&p.frozen[s >> 6], 1ull << (s & 63));
        atomicAdd(&p.counters[0], 1u);
      }
      return;  // advance_frame returns Err for this session from the next tick on
    }
    if (t == p.T - 1 && p.live_out_last) store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);
  }
}

template <class G>
__global__ void report_kernel(const typename G::CS* __restrict__ cs, const int32_t* __restrict__ err, int S,
                              int32_t frame, rb_checksum_report* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const U128 c = to_u128(cs[s]);
  rb_checksum_report r;
  r.checksum_lo = c.lo;
  r.checksum_hi = c.hi;
  r.frame = frame;
  r.mismatch_frame = err[s];
  out[s] = r;
}

__global__ void sincos_kernel(const float* __restrict__ x, float* __restrict__ so, float* __restrict__ co, int64_t n,
                              uint32_t* unexpected) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const SinCos r = sincosf_glibc(x[i], unexpected);
  so[i] = r.s;
  co[i] = r.c;
}

}  // namespace rb

// ============================================================================
// host side
// ============================================================================
namespace rb {
struct GameOps {
  virtual ~GameOps() = default;
  int nw = 0, lanes = 1, players = 0, input_bytes = 0, inrec_bytes = 0, cs_bytes = 0, image_bytes = 0, canon_words = 0;
  bool display = false;
  virtual void word_loc(int k, int* lane, int* word) const = 0;
  virtual void init_words(uint32_t* w) const = 0;
  virtual void image(const uint32_t* w, int32_t frame, uint8_t* out) const = 0;
  virtual U128 cs_at(const void* arr, size_t i) const = 0;
  virtual hipError_t launch_tick(const KParams& p, int block, hipStream_t st) const = 0;
  // fused steady-state ticks; hipErrorNotSupported when CD has no instantiation
  virtual hipError_t launch_steady(const RunParams& p, int cd, int block, hipStream_t st) const = 0;
  bool launch_steady_supported(int cd) const { return cd >= 1 && cd <= 8; }
  virtual hipError_t launch_report(const void* cs, const int32_t* err, int S, int32_t frame, void* out,
                                   hipStream_t st) const = 0;
};

template <class G>
struct GameOpsT final : GameOps {
  GameOpsT() {
    nw = G::NWL;
    lanes = G::kLanes;
    canon_words = G::kCanonWords;
    players = G::kPlayers;
    input_bytes = G::kInputBytes;
    inrec_bytes = sizeof(typename G::InRec);
    cs_bytes = sizeof(typename G::CS);
    image_bytes = G::kImageBytes;
    display = G::kDisplay;
  }
  void word_loc(int k, int* lane, int* word) const override { G::word_loc(k, lane, word); }
  void init_words(uint32_t* w) const override { G::init(w); }
  void image(const uint32_t* w, int32_t frame, uint8_t* out) const override { G::image(w, frame, out); }
  U128 cs_at(const void* arr, size_t i) const override {
    return to_u128(reinterpret_cast<const typename G::CS*>(arr)[i]);
  }
  hipError_t launch_tick(const KParams& p, int block, hipStream_t st) const override {
    const int grid = (p.Spad * G::kLanes + block - 1) / block;
    if (p.in_mode == 2)
      hipLaunchKernelGGL((tick_kernel<G, true>), dim3(grid), dim3(block), 0, st, p);
    else
      hipLaunchKernelGGL((tick_kernel<G, false>), dim3(grid), dim3(block), 0, st, p);
    return hipGetLastError();
  }
  template <int CD>
  static hipError_t steady_cd(const RunParams& p, int block, hipStream_t st) {
    const int grid = (p.Spad * G::kLanes + block - 1) / block;
    hipLaunchKernelGGL((steady_kernel<G, CD>), dim3(grid), dim3(block), 0, st, p);
    return hipGetLastError();
  }
  hipError_t launch_steady(const RunParams& p, int cd, int block, hipStream_t st) const override {
    switch (cd) {
      case 1: return steady_cd<1>(p, block, st);
      case 2: return steady_cd<2>(p, block, st);
      case 3: return steady_cd<3>(p, block, st);
      case 4: return steady_cd<4>(p, block, st);
      case 5: return steady_cd<5>(p, block, st);
      case 6: return steady_cd<6>(p, block, st);
      case 7: return steady_cd<7>(p, block, st);
      case 8: return steady_cd<8>(p, block, st);
      default: return hipErrorNotSupported;
    }
  }
  hipError_t launch_report(const void* cs, const int32_t* err, int S, int32_t frame, void* out,
                           hipStream_t st) const override {
    hipLaunchKernelGGL(report_kernel<G>, dim3((S + 255) / 256), dim3(256), 0, st,
                       reinterpret_cast<const typename G::CS*>(cs), err, S, frame,
                       reinterpret_cast<rb_checksum_report*>(out));
    return hipGetLastError();
  }
};

template <bool kSplit>
inline std::unique_ptr<GameOps> make_ex_game(int players) {
  switch (players) {
    case 1: return std::make_unique<GameOpsT<ExGame<1, kSplit>>>();
    case 2: return std::make_unique<GameOpsT<ExGame<2, kSplit>>>();
    case 3: return std::make_unique<GameOpsT<ExGame<3, kSplit>>>();
    case 4: return std::make_unique<GameOpsT<ExGame<4, kSplit>>>();
    default: return nullptr;
  }
}

inline std::unique_ptr<GameOps> make_game(int game, int players, bool lane_per_session) {
  switch (game) {
    case RB_GAME_EX_GAME: return lane_per_session ? make_ex_game<false>(players) : make_ex_game<true>(players);
    case RB_GAME_STUB: return players == 2 ? std::make_unique<GameOpsT<StubGame>>() : nullptr;
    case RB_GAME_STUB_ENUM: return players == 2 ? std::make_unique<GameOpsT<StubEnumGame>>() : nullptr;
    case RB_GAME_STUB_RANDOM_CS: return players == 2 ? std::make_unique<GameOpsT<StubRandomCsGame>>() : nullptr;
    case RB_GAME_BRAWLER:
      switch (players) {
        case 1: return std::make_unique<GameOpsT<Brawler<1>>>();
        case 2: return std::make_unique<GameOpsT<Brawler<2>>>();
        case 3: return std::make_unique<GameOpsT<Brawler<3>>>();
        case 4: return std::make_unique<GameOpsT<Brawler<4>>>();
        default: return nullptr;
      }
    default: return nullptr;
  }
}

}  // namespace rb

using namespace rb;

struct rb_batch {
  rb_config cfg{};
  std::unique_ptr<GameOps> ops;
  std::unique_ptr<SyncTestPlan> plan;
  int S = 0, Spad = 0, W = 0, P = 0, block = 256;
  bool plan_only = false;
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
  uint32_t* pinned_counters = nullptr;
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
};

namespace {
thread_local std::string g_create_err;

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
  if (b->pinned_counters) (void)hipHostFree(b->pinned_counters);
  for (auto& e : b->stage_ev)
    if (e) (void)hipEventDestroy(e);
  if (b->tick_ev) (void)hipEventDestroy(b->tick_ev);
  for (auto& pr : b->prof_ev) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
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
  if (timed) {
    if (b->prof_used == b->prof_ev.size()) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      HIP_TRY(b, hipEventCreate(&e0));
      HIP_TRY(b, hipEventCreate(&e1));
      b->prof_ev.push_back({e0, e1});
    }
    HIP_TRY(b, hipEventRecord(b->prof_ev[b->prof_used].first, b->stream));
  }
  HIP_TRY(b, b->ops->launch_tick(p, b->block, b->stream));
  if (timed) {
    HIP_TRY(b, hipEventRecord(b->prof_ev[b->prof_used].second, b->stream));
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
  if (!ops) return fail(nullptr, RB_INVALID_REQUEST, "unsupported game / num_players combination");
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
  HIP_CREATE(hipHostMalloc(&b->pinned_counters, 16));
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
    HIP_TRY(b, hipMemcpyAsync(b->pinned_counters, b->counters, 8, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(b, hipEventRecord(b->tick_ev, b->stream));
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
  const bool timed = b->prof;
  if (timed) {
    if (b->prof_used == b->prof_ev.size()) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      HIP_TRY(b, hipEventCreate(&e0));
      HIP_TRY(b, hipEventCreate(&e1));
      b->prof_ev.push_back({e0, e1});
    }
    HIP_TRY(b, hipEventRecord(b->prof_ev[b->prof_used].first, b->stream));
  }
  hipError_t e = b->ops->launch_steady(r, b->cfg.check_distance, b->block, b->stream);
  if (e != hipSuccess) return fail(b, RB_DEVICE_ERROR, std::string("steady_kernel: ") + hipGetErrorString(e));
  if (timed) {
    HIP_TRY(b, hipEventRecord(b->prof_ev[b->prof_used].second, b->stream));
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
  const bool can_fuse = b->ops->launch_steady_supported(b->cfg.check_distance);
  int32_t run_start = -1, run_c0 = 0;
  uint32_t run_tick0 = 0;
  auto flush = [&](int32_t end) -> rb_status {
    if (run_start < 0) return RB_OK;
    rb_status st = launch_steady_run(b, dev_in + static_cast<int64_t>(run_start) * stride, stride, run_c0,
                                     end - run_start, run_tick0);
    run_start = -1;
    return st;
  };
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
    if (can_fuse && is_steady_shape(b, tp)) {
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
  if (tmp) (void)hipFreeAsync(tmp, b->stream);
  if (ticks_done) *ticks_done = done;
  if (result == RB_OK && (b->cfg.flags & RB_FLAG_CHECKED)) {
    HIP_TRY(b, hipMemcpyAsync(b->pinned_counters, b->counters, 8, hipMemcpyDeviceToHost, b->stream));
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
  std::vector<uint32_t> w(b->ops->nw * b->ops->lanes);
  for (int s = 0; s < b->S; ++s) {
    words_of(b, planes, s, w.data());
    if (images) b->ops->image(w.data(), frame, static_cast<uint8_t*>(images) + static_cast<size_t>(s) * b->ops->image_bytes);
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

rb_status rb_debug_sincosf(int32_t device, const float* x, float* so, float* co, int64_t n) {
  rb_batch* b = nullptr;
  if (n <= 0) return RB_OK;
  HIP_TRY(b, hipSetDevice(device));
  float *dx = nullptr, *ds = nullptr, *dc = nullptr;
  uint32_t* du = nullptr;
  const size_t bytes = static_cast<size_t>(n) * 4;
  hipError_t e = hipMalloc(&dx, bytes);
  if (e == hipSuccess) e = hipMalloc(&ds, bytes);
  if (e == hipSuccess) e = hipMalloc(&dc, bytes);
  if (e == hipSuccess) e = hipMalloc(&du, 4);
  if (e == hipSuccess) e = hipMemset(du, 0, 4);
  if (e == hipSuccess) e = hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(sincos_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, nullptr, dx, ds, dc, n, du);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(so, ds, bytes, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(co, dc, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(ds);
  (void)hipFree(dc);
  (void)hipFree(du);
  if (e != hipSuccess) return fail(nullptr, RB_DEVICE_ERROR, std::string("rb_debug_sincosf: ") + hipGetErrorString(e));
  return RB_OK;
}

rb_status rb_profile_enable(rb_batch* b, int32_t on) {
  b->prof = on != 0;
  b->prof_every = on > 1 ? static_cast<uint32_t>(on) : 8u;
  b->prof_tick = 0;
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
