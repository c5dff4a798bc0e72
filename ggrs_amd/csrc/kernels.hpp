// ggrs_amd/csrc/kernels.hpp — device kernels of the batched rollback engine and the
// per-game launcher (GameOpsT).  Included by every ops_*.hip translation unit, each
// of which instantiates the kernels of its own games (so the device code of the
// games compiles in parallel), and by engine.hip for the shared types.
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
#pragma once
#include <hip/hip_ext.h>
#include <algorithm>
#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "../../include/ggrs_amd.h"
#include "games.hpp"
#include "planner.hpp"
#include <type_traits>

namespace rb {

// ---- Issue-priority turns for the waves that share a SIMD (round 4, tools/wave_clock.py).
// At 65,536 sessions the fused kernels run two waves per SIMD, and the SIMD's arbiter issues
// the older wave first whenever both are ready: per-wave clocks showed the first wave of every
// SIMD finishing a 50-tick SyncTest launch in ~130 us and the second in ~200 us, the second
// running alone (one wave: a latency-bound chain) for the last third of the launch.  Taking
// turns at the higher priority (s_setprio), switched on the chip's constant-rate clock every
// 2^RB_PRIO_SHIFT x 10 ns and keyed to the wave's slot on its SIMD (HW_ID bit 0: the two waves
// of a SIMD hold slots 0 and 1), lets both progress at the pair's rate and finish together.
// Quanta measured (SyncTest, 50 ticks): 2^10 205, 2^11 201, 2^12 200 us against 217; checking
// every AdvanceFrame instead of every tick: 212.  Turns by progress instead of the clock (512-thread
// workgroups, the two waves of a SIMD posting their tick counts in LDS) equalised every pair but
// not the launch: what is left is the spread between SIMDs, whose waves take the speed clamp
// (ex_game.rs:300-304) in different numbers of frames (lifetime correlation 0.66).  One-tick launches (T = 1) take no turns:
// 2^7-2^9 quanta checked at the tick's opening and every AdvanceFrame measured no gain.
#ifndef RB_PRIO_SHIFT
#define RB_PRIO_SHIFT 11
#endif
#ifndef RB_STEADY_PRIO
#define RB_STEADY_PRIO 1  // 0: the hardware's oldest-first order (A/B builds)
#endif
#ifndef RB_P2P_PRIO
#define RB_P2P_PRIO 1
#endif
#ifndef RB_PRIO_ROTATE
#define RB_PRIO_ROTATE 1  // 0: two-level turns whatever the waves per SIMD (A/B builds)
#endif
// The turn key: the wave's slot on its SIMD (HW_ID bits 1:0) and, in bit 2, whether the launch
// puts more than two waves on a SIMD (`many`: decided on the host from the device's SIMD count,
// RunParams::many_waves).  Two waves take turns at priority
// 1 over 0; three or four rotate through priorities 0-3 (each leads a quarter of the time).
// Measured at 131,072 sessions (4 waves per SIMD): SyncTest 8.58 us per tick rotating, 8.78 with
// two-level turns, 8.85 without turns; P2P 7.01 / 6.76 / 7.22, so p2p_kernel keeps two levels.
__device__ __forceinline__ uint32_t wave_turn_key(bool many = false) {
  return (__builtin_amdgcn_s_getreg(0xF804) & 3u) | (RB_PRIO_ROTATE && many ? 4u : 0u);  // HW_ID
}
__device__ __forceinline__ void prio_turn(uint32_t key) {
  const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime() >> RB_PRIO_SHIFT);
  if (key & 4u) {
    switch ((c + key) & 3u) {
      case 0: __builtin_amdgcn_s_setprio(0); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      case 2: __builtin_amdgcn_s_setprio(2); break;
      default: __builtin_amdgcn_s_setprio(3); break;
    }
  } else if (((c ^ key) & 1u) != 0u) {
    __builtin_amdgcn_s_setprio(1);
  } else {
    __builtin_amdgcn_s_setprio(0);
  }
}

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
  uint32_t* fail_flag;  // host-mapped word set to 1 when a session fails (checked mode), or null
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
// The same accesses addressed as the array's base (SGPRs) plus a 32-bit per-lane byte offset that
// carries the slot too (global_* saddr form): per access one scalar multiply for the slot and one
// 32-bit add per plane group, where the 64-bit form builds a 64-bit address per plane group and
// slot.  Only for arrays below 4 GiB (the caller checks).  `lane` holds the lane's offset inside a
// slot for plane group 0 (16 * g bytes: launch constants), `slot_off` the slot's byte offset.
template <int NW>
__device__ __forceinline__ void store_words_sa(char* __restrict__ base, uint32_t slot_off, uint32_t Gpad, uint32_t g,
                                               const uint32_t (&w)[NW]) {
  constexpr int Q4 = NW / 4, R = NW % 4;
#pragma unroll
  for (int j = 0; j < Q4; ++j)
    *reinterpret_cast<uint4*>(base + (slot_off + j * 16u * Gpad + 16u * g)) =
        make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
  uint32_t b = slot_off + Q4 * 16u * Gpad;
  if constexpr (R >= 2) {
    *reinterpret_cast<uint2*>(base + (b + 8u * g)) = make_uint2(w[Q4 * 4], w[Q4 * 4 + 1]);
    b += 8u * Gpad;
  }
  if constexpr (R & 1) *reinterpret_cast<uint32_t*>(base + (b + 4u * g)) = w[NW - 1];
}
template <int NW>
__device__ __forceinline__ void load_words_sa(const char* __restrict__ base, uint32_t slot_off, uint32_t Gpad, uint32_t g,
                                              uint32_t (&w)[NW]) {
  constexpr int Q4 = NW / 4, R = NW % 4;
#pragma unroll
  for (int j = 0; j < Q4; ++j) {
    const uint4 v = *reinterpret_cast<const uint4*>(base + (slot_off + j * 16u * Gpad + 16u * g));
    w[4 * j + 0] = v.x;
    w[4 * j + 1] = v.y;
    w[4 * j + 2] = v.z;
    w[4 * j + 3] = v.w;
  }
  uint32_t b = slot_off + Q4 * 16u * Gpad;
  if constexpr (R >= 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(base + (b + 8u * g));
    w[Q4 * 4 + 0] = v.x;
    w[Q4 * 4 + 1] = v.y;
    b += 8u * Gpad;
  }
  if constexpr (R & 1) w[NW - 1] = *reinterpret_cast<const uint32_t*>(base + (b + 4u * g));
}
// steady_kernel's cells and checksums in the saddr form, for games whose per-session state is at
// most 80 B per slot (ex_game: 5 words x up to 4 lanes; the stubs): their whole snapshot ring stays
// below 4 GiB up to 3.3M sessions at W = 16, and larger batches run per-tick launches
// (GameOps::launch_steady_supported).  The brawler's 8 KiB cells keep the 64-bit form.  Measured
// (interleaved A/B, profiles/r05_ab_saddr.log): SyncTest 4.15 -> 4.04 us per tick, the driver's
// 20-tick call 1.211e11 -> 1.250e11 session-frames/s.
template <class G>
constexpr bool steady_saddr() {
  return G::NWL * G::kLanes * 4 <= 80;
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

// G::kHasFast (games.hpp ExGame::advance_prepared_fast), false when not declared
template <class G, class = void>
struct HasFast {
  static constexpr bool value = false;
};
template <class G>
struct HasFast<G, std::void_t<decltype(G::kHasFast)>> {
  static constexpr bool value = G::kHasFast;
};
template <class G, class Pr>
__device__ __forceinline__ void advance_fast(uint32_t (&w)[G::NWL], const Pr& pr, int k, uint32_t& special) {
  if constexpr (HasFast<G>::value) G::advance_prepared_fast(w, pr, k, special);
}
// One AdvanceFrame{inputs} (State::advance, ex_game.rs:259-321) for the
// kernels that run frames one at a time (tick_kernel, p2p_kernel, the fan-out).
// (Round 3 measured a branch-free form with a wave-wide redo here: neutral on
// p2p_kernel, so it was dropped.)
template <class G>
__device__ __forceinline__ void advance_frame(uint32_t (&w)[G::NWL], typename G::InRec in, int lane, uint32_t dmask,
                                              uint32_t* unexpected) {
  G::advance(w, in, lane, dmask, unexpected);
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
        advance_frame<G>(w, in[k], lane, p.disc_mask, &p.counters[1]);  // AdvanceFrame{inputs}
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
    if (p.fail_flag) *p.fail_flag = 1u;  // (every failing lead lane stores the same word)
  }
}

// ---------------------------------------------------------------------------
// Fused steady-state SyncTest ticks (rb_run_ticks).  For current frame c > cd
// the reference's stream is always (sync_test_session.rs:89-132, 178-203)
//   Load(c-cd), Adv, [Save(f) Adv] for f = c-cd+1 .. c-1, Save(c), Adv
// so T consecutive such ticks run in ONE launch with the shape known at
// compile time (CD = check distance): no per-tick launch, no per-step control
// flow, and each wave keeps its sessions across ticks.  Every request still
// executes against memory exactly as in tick_kernel: every save stores the
// cell, its checksum and (frame c) the first-seen record, the new inputs are
// written to the input-queue ring, and each tick's LoadGameState reads its
// cell back from memory.  What a tick needs is fetched a tick ahead, so no
// load sits on the critical path of the 8 serial AdvanceFrames:
//  * the next tick loads cell c+1-CD, which this tick saves at its step 1:
//    the load is issued right after that store (same lane and address, so
//    program order returns the stored bytes) and consumed CD-1 steps later;
//  * inputs and first-seen checksums already known to the launch slide
//    through register windows; the one new input per tick comes from the
//    read-only per-tick input buffer, never from a ring entry this launch
//    wrote.
// The host bookkeeping runs per tick as usual; only ticks whose lowered
// program has exactly this shape are fused.
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
  uint32_t* fail_flag;     // host-mapped word set to 1 when a session fails (checked mode), or null
  const uint8_t* in_base;  // tick t, player q: in_base + t*in_stride + q*S*kInputBytes
  int64_t in_stride;
  int32_t S, Spad, W, delay;
  int32_t c0, T;            // current frame of the first fused tick, tick count
  uint32_t tick0;           // engine tick index of the first fused tick (nonce)
  int32_t live_out_last;    // store the live state after the last tick
  uint64_t seed;
  uint32_t debug;           // experiment knobs (rb_config.reserved[0]); 0 in every real run
  int32_t pipe;             // 1: two ticks in flight per lane where the game allows it (steady_pipe.hpp)
  uint32_t lds_pad;         // dynamic LDS bytes per workgroup the launch reserves (unused: caps workgroups per CU)
  uint32_t many_waves;      // the launch puts more than two waves on a SIMD of this device (prio_turn)
  // rb_launch_clock_arm: when set, every wave stores its start and end on the chip's 100 MHz
  // constant clock (s_memrealtime) at [2 * wave] and [2 * wave + 1]; the host takes the first
  // start and the last end (rb_launch_clock_read).  A kernel time taken by the kernel itself: no
  // host call, event or profiler sits in it.  Plain stores, one lane per wave: no atomics on a
  // shared address (2,048 waves folding into one word serialise at the memory side: +40 us).
  unsigned long long* launch_clock;
};

__device__ __forceinline__ void launch_clock_put(unsigned long long* c, unsigned wave, unsigned which) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  if (__lane_id() == static_cast<unsigned>(__builtin_ctzll(__ballot(1)))) c[2u * wave + which] = t;
}

// An empty asm that reads v: the compiler must complete the load that
// produced v before this point (an s_waitcnt counted within the iteration).
__device__ __forceinline__ void settle(uint32_t v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void settle(uint64_t v) {
  settle(static_cast<uint32_t>(v));
  settle(static_cast<uint32_t>(v >> 32));
}
__device__ __forceinline__ void settle(U128 v) {
  settle(v.lo);
  settle(v.hi);
}
__device__ __forceinline__ void settle(uint16_t v) { settle(static_cast<uint32_t>(v)); }
__device__ __forceinline__ void settle(uint8_t v) { settle(static_cast<uint32_t>(v)); }

// The game's phase-split state for N AdvanceFrames (games.hpp kHasPrep), or nothing.
template <class G, int N, bool = G::kHasPrep>
struct PrepSel {
  struct type {};
};
template <class G, int N>
struct PrepSel<G, N, true> {
  using type = typename G::template Prep<N>;
};
template <class G, int N>
using PrepOf = typename PrepSel<G, N>::type;
template <class G, bool = G::kHasPrep>
struct DecSel {
  struct type {};
};
template <class G>
struct DecSel<G, true> {
  using type = typename G::Dec;
};
template <class G>
using DecOf = typename DecSel<G>::type;
// RB_STEADY_FAST (RB_EXPERIMENTS builds only): the branch-free form with the tick redo, measured
// slower (269 vs 220 us per 50 ticks, round 3); never compiled into the product library.
#if RB_EXPERIMENTS && defined(RB_STEADY_FAST_AB)
#define RB_STEADY_FAST 1
#else
#define RB_STEADY_FAST 0
#endif

// kExp: attribution experiments (RunParams::debug knobs, tools/exp_steady.py);
// instantiated only in builds made with RB_EXPERIMENTS=1, never in the product.
#ifndef RB_STEADY_WAVES_PER_EU
#define RB_STEADY_WAVES_PER_EU 0  // >0: the occupancy the compiler may schedule for (A/B builds)
#endif
// RB_WAVE_CLOCK (A/B builds, tools/wave_clock.py): every wave of the steady kernel records its
// start and end on the chip's constant-rate clock (s_memrealtime, 100 MHz) and where it ran
// (HW_ID, XCC_ID) into rb_wave_clock, read back by rb_debug_wave_clock.
#ifndef RB_WAVE_CLOCK
#define RB_WAVE_CLOCK 0
#endif
#if RB_WAVE_CLOCK
__device__ uint64_t rb_wave_clock[4 * 8192];
#endif
template <class G, int CD, bool kExp>
__global__ void __launch_bounds__(256)
#if RB_STEADY_WAVES_PER_EU > 0
__attribute__((amdgpu_waves_per_eu(1, RB_STEADY_WAVES_PER_EU)))
#endif
steady_kernel(const RunParams p) {
  static_assert(CD >= 1, "steady shape needs a rollback");
  const uint32_t dbg = kExp ? p.debug : 0u;
  using InRec = typename G::InRec;
  using CS = typename G::CS;
  constexpr int NW = G::NWL;
  constexpr unsigned L = G::kLanes;
  constexpr int P = G::kPlayers, IB = G::kInputBytes;
  constexpr int NF = CD > 1 ? CD - 1 : 1;  // first-seen window: frames f0+1 .. f0+CD-1
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned s = g / L;
  const int lane = static_cast<int>(g % L);
  const bool lead = lane == 0;
  if (p.launch_clock) launch_clock_put(p.launch_clock, g / 64u, 0u);
  if (s >= static_cast<unsigned>(p.S)) return;
  {
    const unsigned wave0 = __builtin_amdgcn_readfirstlane(s) & ~63u;
    if ((p.frozen[wave0 >> 6] >> (s & 63)) & 1ull) return;
  }
  const unsigned Spad = static_cast<unsigned>(p.Spad), Gpad = Spad * L;
  const unsigned slot_words = static_cast<unsigned>(NW) * Gpad;
  constexpr bool kSA = steady_saddr<G>();  // (the host launches this kernel only for rings below 4 GiB)
#if RB_WAVE_CLOCK
  const uint64_t wc_start = __builtin_amdgcn_s_memrealtime();
  uint32_t wc_general = 0;  // ticks this wave ran in the general (not in-range) form
  uint32_t wc_clamp = 0;
#endif
  InRec* __restrict__ ring = reinterpret_cast<InRec*>(p.ring);
  CS* __restrict__ csa = reinterpret_cast<CS*>(p.cs);
  CS* __restrict__ fsa = reinterpret_cast<CS*>(p.fs);
  const int W = p.W;
  auto slot_of = [W](int f) { return static_cast<unsigned>(f % W); };
  // slot of frame f0 + k given slot0 = f0 % W, k <= CD < W: no division per step
  auto slot_after = [W](unsigned slot0, int k) {
    const unsigned sl = slot0 + static_cast<unsigned>(k);
    return sl >= static_cast<unsigned>(W) ? sl - static_cast<unsigned>(W) : sl;
  };
  // The new inputs of launch tick tt (the read-only per-tick input buffer).
  auto new_input = [&](int tt) -> InRec {
    const uint8_t* tin = p.in_base + static_cast<int64_t>(tt) * p.in_stride;
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      uint64_t x;
      if constexpr (IB == 4)
        x = reinterpret_cast<const uint32_t*>(tin + static_cast<size_t>(q) * p.S * IB)[s];
      else
        x = tin[static_cast<size_t>(q) * p.S + s];
      v |= x << (8 * IB * q);
    }
    return static_cast<InRec>(v);
  };
  // InputQueue::input(frame) for a confirmed frame: the input added at tick
  // frame - delay.  Inside this launch that is that tick's new input (read
  // from the input buffer, never from a ring entry this launch wrote); older
  // frames come from the ring as written before the launch.  Wave-uniform.
  // Both loads are issued unconditionally and selected: a branch around a
  // load makes the compiler wait for it (and every older store) at the join.
  auto input_of_frame = [&](int fr) -> InRec {
    const int tt = fr - p.delay - p.c0;
    const InRec a = new_input(tt >= 0 ? tt : 0);
    const InRec b = ring[static_cast<unsigned>(fr & (kQueueLen - 1)) * Spad + s];
    return tt >= 0 ? a : b;
  };

  // Prologue: the first tick's snapshot, input window and first-seen window.
  // Later ticks get them from registers (inputs, first-seen values this
  // launch recorded) or from a load issued one tick ahead (the snapshot).
  int f0 = p.c0 - CD;
  uint32_t w[NW];
  load_words<NW>(p.snap + slot_of(f0) * slot_words, static_cast<int>(Gpad), static_cast<int>(g), w);
  InRec win[CD + 1];  // inputs of frames f0 .. f0+CD
#pragma unroll
  for (int k = 0; k <= CD; ++k) win[k] = input_of_frame(f0 + k);
  // the phase-split games read the window decoded (games.hpp ExGame::Dec), each
  // input once, as it enters the window
  [[maybe_unused]] DecOf<G> dec[CD + 1];
  if constexpr (G::kHasPrep) {
#pragma unroll
    for (int k = 0; k <= CD; ++k) dec[k] = G::decode(win[k], lane);
  }
  CS fsw[NF];  // SyncTest first-seen checksums of frames f0+1 .. f0+CD-1
#pragma unroll
  for (int k = 1; k < CD; ++k) fsw[k - 1] = fsa[slot_of(f0 + k) * Spad + s];

  // A load whose value is used after a store waits for that store too (vmcnt
  // retires loads and stores in issue order), so every input load is issued
  // one tick before it is used, ahead of that tick's stores.
  InRec newin = new_input(0);
  unsigned slot0 = slot_of(f0);  // f0 % W, advanced with f0
  [[maybe_unused]] CS pc{};  // Game::periodic_checksum, carried through the launch
  if constexpr (G::kDisplay) pc = reinterpret_cast<const CS*>(p.periodic_cs)[s];
  // Complete the prologue loads before the loop.  The waitcnt pass merges
  // the loop header's state from the preheader and the latch: a load still
  // pending on the preheader path makes it put a conservative vmcnt at the
  // first use inside the loop, which in the steady state then waits for every
  // store of the previous tick.
#pragma unroll
  for (int i = 0; i < NW; ++i) settle(w[i]);
#pragma unroll
  for (int k = 0; k <= CD; ++k) settle(win[k]);
#pragma unroll
  for (int k = 0; k + 1 < CD; ++k) settle(fsw[k]);
  settle(newin);
  if constexpr (G::kDisplay) settle(pc);
#if RB_STEADY_PRIO
  const uint32_t wslot = wave_turn_key(p.many_waves != 0);
#endif
  for (int t = 0; t < p.T; ++t) {
    const int c = p.c0 + t;
    const bool more = t + 1 < p.T;
#if RB_STEADY_PRIO
    if (p.T > 1) prio_turn(wslot);  // (launch-uniform)
#endif
    // ---- the next tick's inputs (read-only sources), before this tick's stores
    const InRec newin_next = new_input(more ? t + 1 : t);
    const InRec next_last = input_of_frame(more ? c + 1 : c);  // frame f0+CD+1 of the next tick
    // ---- InputQueue::add_input for every handle: the new inputs at c + delay
    ring[static_cast<unsigned>((c + p.delay) & (kQueueLen - 1)) * Spad + s] = newin;  // same value from every lane
    // ---- the request stream
    const uint32_t nonce = ((p.tick0 + static_cast<uint32_t>(t)) & 0xffffffu) << 8;
    CsCtx ctx{p.seed, s, nonce};
    int32_t mismatch = kNullFrame;
    CS recorded{};
    // the save of this tick whose frame is a multiple of 100 (ex_game's CHECKSUM_PERIOD), if any:
    // one scalar modulo per tick instead of a divisibility test per save
    [[maybe_unused]] const int kp = G::kDisplay ? (100 - f0 % 100) % 100 : -1;
    uint32_t wn[NW];  // next tick's LoadGameState(c+1-CD), loaded right after this tick saves it
    // The tick's steps, instantiated twice: with the game's out-of-line range
    // checks compiled out when the whole wave's loaded state is in range
    // (G::in_range, decided once per tick), and the general form otherwise.
    // Checksums are whole-session values present in every lane of the group
    // (group_sum), so the checksum stores are issued by every lane: the lanes
    // of a session write the same value to the same address, and no exec-mask
    // branch splits the tick into separately scheduled blocks.
    // kFast (in-range ticks of a game with G::kHasFast): the branch-free AdvanceFrame, whose
    // flagged lanes (operands outside its short division sequence) make the wave redo the tick
    // in the general form below; returns this lane's flag.
    auto steps = [&](auto in_range_tag, auto fast_tag) __attribute__((always_inline)) -> uint32_t {
    constexpr bool kInRange = decltype(in_range_tag)::value;
    constexpr bool kFast = decltype(fast_tag)::value;
    uint32_t special = 0;
    [[maybe_unused]] PrepOf<G, CD + 1> prep;
    if constexpr (G::kHasPrep && !kExp)  // the tick's rotation chain and thrust first (games.hpp)
      G::template prepare<kInRange, CD + 1>(w, dec, prep, &p.counters[1]);
#pragma unroll
    for (int k = 0; k <= CD; ++k) {
      const int f = f0 + k;
      if (k > 0) {  // SaveGameState{cell, f}
        ctx.nonce = nonce + static_cast<uint32_t>(k);
        const CS cval = (dbg & 4u) ? CS{} : G::checksum(w, f, lane, ctx);
        const unsigned slot = slot_after(slot0, k);
        [[maybe_unused]] const uint32_t soff = slot * slot_words * 4u;  // (kSA: the slot's byte offset)
        if constexpr (kSA) {
          if (!(dbg & 2u)) store_words_sa<NW>(reinterpret_cast<char*>(p.snap), soff, Gpad, g, w);
          *reinterpret_cast<CS*>(reinterpret_cast<char*>(csa) + (slot * Spad * static_cast<uint32_t>(sizeof(CS)) +
                                                                 s * static_cast<uint32_t>(sizeof(CS)))) = cval;
        } else {
          if (!(dbg & 2u)) store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), w);
          csa[slot * Spad + s] = cval;
        }
        if (k == CD) {
          fsa[slot * Spad + s] = cval;  // first save of frame c: first-seen
          recorded = cval;
        } else if (cval != fsw[k - 1]) {
          mismatch = f;  // newest mismatching frame wins
        }
        // ex_game periodic_checksum (frame % CHECKSUM_PERIOD == 0, ex_game.rs:104-111): the state an
        // AdvanceFrame reaches at frame f is the one this save checksums, so the value is this one
        if constexpr (G::kDisplay) pc = (k == kp) ? cval : pc;
        // Same lane, same address, program order: this load returns the cell just stored.
        if (k == 1 && more) {
          if constexpr (kSA)
            load_words_sa<NW>(reinterpret_cast<const char*>(p.snap), soff, Gpad, g, wn);
          else
            load_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), wn);
        }
      }
      if (dbg & 1u)
        w[0] += win[k];
      else if constexpr (kFast && !kExp)
        advance_fast<G>(w, prep, k, special);  // AdvanceFrame{inputs}
      else if constexpr (G::kHasPrep && !kExp) {
#if RB_WAVE_CLOCK
        {  // (wave clocks: frames in which some lane of the wave takes the speed clamp)
          const float vx = __uint_as_float(w[2]) * G::kFriction + prep.tx[0][k], vy = __uint_as_float(w[3]) * G::kFriction + prep.ty[0][k];
          wc_clamp += __any(vx * vx + vy * vy > 49.0f) ? 1u : 0u;
        }
#endif
        G::advance_prepared(w, prep, k);  // AdvanceFrame{inputs}
      }
      else
        G::template advance<kInRange>(w, (dbg & 32u) ? static_cast<InRec>(win[k] & static_cast<InRec>(dbg >> 8)) : win[k],
                                      lane, 0u, &p.counters[1]);  // AdvanceFrame{inputs}
    }
    return special;
    };
    if (G::kHasRangePath && __all(G::in_range(w))) {
      if constexpr (HasFast<G>::value && RB_STEADY_FAST && !kExp) {
        // Optimistic: every lane of the wave runs the branch-free tick; if any lane met an
        // operand its division sequence does not cover, the wave runs the tick again from the
        // loaded state in the general form.  The redo re-executes every request of the tick:
        // it stores the same cells, checksums and first-seen record over the first pass's (same
        // lanes, same addresses, program order), re-decides the mismatch and reloads the next
        // tick's cell.
        uint32_t w0[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) w0[i] = w[i];
        if (__any(steps(std::true_type{}, std::true_type{}) != 0u)) {
#pragma unroll
          for (int i = 0; i < NW; ++i) w[i] = w0[i];
          mismatch = kNullFrame;
          steps(std::false_type{}, std::false_type{});
        }
      } else {
        steps(std::true_type{}, std::false_type{});
      }
    } else {
#if RB_WAVE_CLOCK
      ++wc_general;
#endif
      steps(std::false_type{}, std::false_type{});
    }
    if constexpr (G::kDisplay) {
      // Game::last_checksum after the final AdvanceFrame (frame c+1) and the periodic checksum
      // when c+1 is a multiple of 100, as the session leaves the launch: at its last tick, or at
      // the tick it stops.  The display value of every earlier tick is overwritten unobserved.
      if (!more || (mismatch != kNullFrame && !dbg)) {
        ctx.nonce = nonce + 255u;
        const CS cval = G::checksum(w, c + 1, lane, ctx);
        reinterpret_cast<CS*>(p.last_cs)[s] = cval;
        pc = ((c + 1) % 100 == 0) ? cval : pc;
        reinterpret_cast<CS*>(p.periodic_cs)[s] = pc;
      }
    }
    if (mismatch != kNullFrame && !dbg) {  // experiments (debug knobs) change results: never freeze
      store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);
      if (lead) {
        p.err[s] = mismatch;
        p.live_frame[s] = c + 1;
        atomicOr(&p.frozen[s >> 6], 1ull << (s & 63));
        atomicAdd(&p.counters[0], 1u);
        if (p.fail_flag) *p.fail_flag = 1u;
      }
      return;  // advance_frame returns Err for this session from the next tick on
    }
    if (!more) {
      if (p.live_out_last) store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), w);
      if (p.launch_clock) launch_clock_put(p.launch_clock, g / 64u, 1u);
      break;
    }
    // ---- wait here, inside the iteration, for the loads the next tick uses.
    // Left to the loop back-edge, the compiler's wait for them would also
    // cover every store issued after them (it loses the count across the edge).
    settle(static_cast<uint32_t>(newin_next));
    settle(static_cast<uint32_t>(next_last));
#pragma unroll
    for (int i = 0; i < NW; ++i) settle(wn[i]);
    // ---- slide the windows to the next tick (c+1): f0 -> f0+1
#pragma unroll
    for (int k = 0; k < CD; ++k) win[k] = win[k + 1];
    win[CD] = next_last;
    if constexpr (G::kHasPrep) {
#pragma unroll
      for (int k = 0; k < CD; ++k) dec[k] = dec[k + 1];
      dec[CD] = G::decode(next_last, lane);
    }
    newin = newin_next;
#pragma unroll
    for (int k = 0; k + 1 < NF; ++k) fsw[k] = fsw[k + 1];
    if (CD > 1) fsw[NF - 1] = recorded;
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = wn[i];
    f0 += 1;
    slot0 = slot_after(slot0, 1);
  }
#if RB_WAVE_CLOCK
  const uint64_t wc_end = __builtin_amdgcn_s_memrealtime();
  const unsigned wv = g / 64;
  if ((g & 63u) == 0 && wv < 8192) {
    rb_wave_clock[4 * wv + 0] = wc_start;
    rb_wave_clock[4 * wv + 1] = wc_end;
    rb_wave_clock[4 * wv + 2] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF814)) << 32 |  // XCC_ID
                                __builtin_amdgcn_s_getreg(0xF804);                               // HW_ID
    rb_wave_clock[4 * wv + 3] = wc_general | (blockDim.x / 64u) << 16 | static_cast<uint64_t>(wc_clamp) << 40;
  }
#endif
}
#if RB_WAVE_CLOCK
extern "C" int rb_debug_wave_clock(uint64_t* host_out, int n) {
  return static_cast<int>(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(rb_wave_clock), sizeof(uint64_t) * 4 * min(n, 8192)));
}
#endif

}  // namespace rb
#if RB_EXPERIMENTS
#include "steady_pipe.hpp"  // two ticks in flight per lane (measured slower: A/B builds only)
#endif
namespace rb {

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

}  // namespace rb
#include "p2p.hpp"  // P2PSession kernel (uses load_words / store_words above)
namespace rb {

// Kernel timing (rb_profile_enable / rb_p2p_profile_enable): the events a launch
// records itself through hipExtLaunchKernel — the kernel's own start and end,
// with no marker packets of their own around it on the stream; both null when
// the batch is not profiling.
struct LaunchEv {
  hipEvent_t start = nullptr, stop = nullptr;
};
template <class K, class... A>
inline hipError_t rb_launch(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st, const LaunchEv& ev,
                            A... args) {
  if (ev.start || ev.stop) hipExtLaunchKernelGGL(kernel, grid, block, lds, st, ev.start, ev.stop, 0u, args...);
  else hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
  return hipGetLastError();
}

// rb_launch_clock_arm / rb_p2p_launch_clock_arm: `cap` launch slots of [waves][start, end] words on
// the device (launch_clock_put), cleared once when armed, so nothing is added to the launches
// themselves; every launch of the batch takes the next slot until the slots run out.
struct LaunchClock {
  unsigned long long* buf = nullptr;
  size_t waves = 0, cap = 0, used = 0, alloc = 0;
  bool armed = false;
  hipError_t arm(size_t waves_per_launch, size_t launches, hipStream_t st) {
    const size_t words = 2 * waves_per_launch * launches;
    if (words > alloc) {
      if (buf) (void)hipFree(buf);
      buf = nullptr;
      alloc = 0;
      hipError_t e = hipMalloc(&buf, words * sizeof(unsigned long long));
      if (e != hipSuccess) return e;
      alloc = words;
    }
    waves = waves_per_launch;
    cap = launches;
    used = 0;
    armed = true;
    return hipMemsetAsync(buf, 0, words * sizeof(unsigned long long), st);
  }
  unsigned long long* next() { return armed && used < cap ? buf + 2 * waves * used++ : nullptr; }
  // per launch slot used: the first wave start and the last wave end (10 ns ticks); disarms
  hipError_t read(uint64_t* start_end, int32_t out_cap, int32_t* n, hipStream_t st) {
    std::vector<uint64_t> h(2 * waves * used);
    hipError_t e = h.empty() ? hipSuccess : hipMemcpyAsync(h.data(), buf, h.size() * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    int32_t k = 0;
    for (size_t l = 0; l < used && k < out_cap; ++l, ++k) {
      uint64_t lo = ~0ull, hi = 0;
      for (size_t w = 0; w < waves; ++w) {
        const uint64_t a = h[2 * (l * waves + w)], z = h[2 * (l * waves + w) + 1];
        if (a) lo = std::min<uint64_t>(lo, a);
        hi = std::max<uint64_t>(hi, z);
      }
      start_end[2 * k] = lo == ~0ull ? 0 : lo;
      start_end[2 * k + 1] = hi;
    }
    *n = k;
    armed = false;
    used = 0;
    return hipSuccess;
  }
  void release() {
    if (buf) (void)hipFree(buf);
    buf = nullptr;
    alloc = 0;
  }
};

struct GameOps {
  virtual ~GameOps() = default;
  int nw = 0, lanes = 1, players = 0, input_bytes = 0, inrec_bytes = 0, cs_bytes = 0, image_bytes = 0, canon_words = 0;
  bool display = false;
  virtual void word_loc(int k, int* lane, int* word) const = 0;
  virtual void init_words(uint32_t* w) const = 0;
  virtual void image(const uint32_t* w, int32_t frame, uint8_t* out) const = 0;
  virtual U128 cs_at(const void* arr, size_t i) const = 0;
  virtual hipError_t launch_tick(const KParams& p, int block, hipStream_t st, const LaunchEv& ev = {}) const = 0;
  // fused steady-state ticks; hipErrorNotSupported when CD has no instantiation
  virtual hipError_t launch_steady(const RunParams& p, int cd, int block, hipStream_t st,
                                   const LaunchEv& ev = {}) const = 0;
  static constexpr int kMaxFusedCD = 16;  // steady_kernel instantiations: check distances 1..16
  bool steady_saddr = false;              // steady_saddr<G>(): 32-bit offsets into the snapshot ring
  // check distances 1..16, and for steady_saddr games rings below 4 GiB (`limit`)
  bool launch_steady_supported(int cd, size_t ring_bytes, size_t limit = size_t{1} << 32) const {
    return cd >= 1 && cd <= kMaxFusedCD && (!steady_saddr || ring_bytes < std::min(limit, size_t{1} << 32));
  }
  virtual hipError_t launch_report(const void* cs, const int32_t* err, int S, int32_t frame, void* out,
                                   hipStream_t st) const = 0;
  // P2PSession ticks and the speculative fan-out (p2p.hpp); fan-out needs one
  // lane per player (ex_game), hipErrorNotSupported otherwise
  virtual hipError_t launch_p2p(const P2PParams& p, int block, hipStream_t st, const LaunchEv& ev = {}) const = 0;
  virtual hipError_t launch_fanout(const FanParams& p, int block, hipStream_t st) const = 0;
  bool fanout_supported = false;
  bool inlane_fanout = false;  // p2p_kernel runs the fan-out itself (inlane_fan), unless fan_generic
  uint32_t input_alphabet = 0;  // InputAlphabet<G>: the per-player fan-out needs all of it as candidates
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
    fanout_supported = kFanout;
    inlane_fanout = kFanout && inlane_fan<G>();
    input_alphabet = InputAlphabet<G>::value;
    steady_saddr = rb::steady_saddr<G>();
  }
  void word_loc(int k, int* lane, int* word) const override { G::word_loc(k, lane, word); }
  void init_words(uint32_t* w) const override { G::init(w); }
  void image(const uint32_t* w, int32_t frame, uint8_t* out) const override { G::image(w, frame, out); }
  U128 cs_at(const void* arr, size_t i) const override {
    return to_u128(reinterpret_cast<const typename G::CS*>(arr)[i]);
  }
  hipError_t launch_tick(const KParams& p, int block, hipStream_t st, const LaunchEv& ev) const override {
    const int grid = (p.Spad * G::kLanes + block - 1) / block;
    if (p.in_mode == 2) return rb_launch(tick_kernel<G, true>, dim3(grid), dim3(block), 0, st, ev, p);
    return rb_launch(tick_kernel<G, false>, dim3(grid), dim3(block), 0, st, ev, p);
  }
  template <int CD>
  static hipError_t steady_cd(const RunParams& p, int block, hipStream_t st, const LaunchEv& ev) {
    const int grid = (p.Spad * G::kLanes + block - 1) / block;
    if (p.debug) {
#if RB_EXPERIMENTS
      return rb_launch(steady_kernel<G, CD, true>, dim3(grid), dim3(block), 0, st, ev, p);
#else
      return hipErrorNotSupported;  // experiment knobs need a RB_EXPERIMENTS=1 build
#endif
    }
#if RB_EXPERIMENTS
    if constexpr (G::kHasPrep && HasFast<G>::value && CD >= 3 && CD <= 7 && CD % 2 == 1) {  // (an A/B variant)
      if (p.pipe) {
        return rb_launch(steady_pipe_kernel<G, CD>, dim3(grid), dim3(block), 0, st, ev, p);
      }
    }
#endif
    return rb_launch(steady_kernel<G, CD, false>, dim3(grid), dim3(block), p.lds_pad, st, ev, p);
  }
  hipError_t launch_steady(const RunParams& p, int cd, int block, hipStream_t st, const LaunchEv& ev) const override {
    switch (cd) {
      case 1: return steady_cd<1>(p, block, st, ev);
      case 2: return steady_cd<2>(p, block, st, ev);
      case 3: return steady_cd<3>(p, block, st, ev);
      case 4: return steady_cd<4>(p, block, st, ev);
      case 5: return steady_cd<5>(p, block, st, ev);
      case 6: return steady_cd<6>(p, block, st, ev);
      case 7: return steady_cd<7>(p, block, st, ev);
      case 8: return steady_cd<8>(p, block, st, ev);
      case 9: return steady_cd<9>(p, block, st, ev);
      case 10: return steady_cd<10>(p, block, st, ev);
      case 11: return steady_cd<11>(p, block, st, ev);
      case 12: return steady_cd<12>(p, block, st, ev);
      case 13: return steady_cd<13>(p, block, st, ev);
      case 14: return steady_cd<14>(p, block, st, ev);
      case 15: return steady_cd<15>(p, block, st, ev);
      case 16: return steady_cd<16>(p, block, st, ev);
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
  template <bool kSpec, bool kSparse, bool kNet, bool kMtf = false>
  static hipError_t launch_p2p_as_m(const P2PParams& p, int grid, int block, hipStream_t st, const LaunchEv& ev) {
    size_t lds = p2p_lds_bytes<G>(block);  // (the HBM-cell launches below)
    if constexpr ((!kSpec || inlane_fan<G>()) && !kNet && p2p_lds_queue<G>()) {
      // the snapshot ring in LDS (p2p_lds_cell_bytes) for launches of many ticks: it is copied in and
      // written back whole, which short launches (the wire path's one tick per launch) do not repay;
      // with the fan-out only for the in-kernel one (fanout_kernel reads the HBM cells between ticks)
      // ... unless the batch puts more than two waves on a SIMD and the plain or sparse path can keep
      // only the input ring in LDS (kQ below): the LDS cells (79 KiB per 256 threads) fit two
      // workgroups per CU, kQ four (131,072 sessions, lag 1-4: 6.72 -> 5.25 us per tick; at 65,536
      // sessions, two waves per SIMD, the LDS cells stay faster, 3.43 against 3.81)
      constexpr bool kHasQ = (!kSpec || (RB_SPEC_Q && inlane_fan<G>())) && !kNet && G::kLanes > 1;
      if (p2p_lds_cells<G>(p.W, block) && p.T >= kLdsCellsMinTicks && (!kSpec || !p.fan_generic) &&
          !(kHasQ && p.many_waves)) {
        // lane-asynchronous ticks (plain path and sparse saving) unless the batch asked for lock-step
        // ticks; the fan-out runs lock-step ticks
        auto k = (!p.sync_ticks && !kSpec) ? p2p_kernel<G, kSpec, kSparse, kNet, true, !kSpec, false, kMtf>
                                           : p2p_kernel<G, kSpec, kSparse, kNet, true, false, false, kMtf>;
        lds = p2p_lds_bytes<G, true>(block) + p2p_lds_cell_bytes<G>(block, p.W);
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           static_cast<int>(lds));
        if (e != hipSuccess) return e;
        return rb_launch(k, dim3(grid), dim3(block), static_cast<uint32_t>(lds), st, ev, p);
      }
    }
    if constexpr ((!kSpec || (RB_SPEC_Q && inlane_fan<G>())) && !kNet && p2p_lds_queue<G>() && G::kLanes > 1) {
      if (p.T >= kLdsQMinTicks && (!kSpec || (p.many_waves && !p.fan_generic))) {  // the input ring alone in LDS
        auto k = p2p_kernel<G, kSpec, kSparse, kNet, false, false, false, kMtf, true>;
        lds = p2p_lds_bytes<G, true>(block);
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           static_cast<int>(lds));
        if (e != hipSuccess) return e;
        return rb_launch(k, dim3(grid), dim3(block), static_cast<uint32_t>(lds), st, ev, p);
      }
    }
    // live play, one tick per launch: the tick count compiled in (p2p_kernel kOne: 121 -> 99 VGPRs, no
    // SGPR spills; 9.70 -> 9.59 us at 65,536 sessions, packet-fed 11.07 -> 10.45; r06_ab_one_tick.log)
    if constexpr (!kSpec && !kNet) {
      if (p.T == 1)
        return rb_launch(p2p_kernel<G, kSpec, kSparse, kNet, false, false, false, kMtf, false, true>, dim3(grid),
                         dim3(block), static_cast<uint32_t>(lds), st, ev, p);
    }
    return rb_launch(p2p_kernel<G, kSpec, kSparse, kNet, false, false, false, kMtf>, dim3(grid), dim3(block),
                     static_cast<uint32_t>(lds), st, ev, p);
  }
  // the fan-out's candidates: the alphabet itself when it has at most K values, else the queues'
  // move-to-front lists (kMtf); ex_game (16 inputs) builds both, larger alphabets only the lists
  template <bool kSpec, bool kSparse, bool kNet>
  static hipError_t launch_p2p_as(const P2PParams& p, int grid, int block, hipStream_t st, const LaunchEv& ev) {
    if constexpr (kSpec) {
      if constexpr (InputAlphabet<G>::value > static_cast<uint32_t>(kSpecBranches))
        return launch_p2p_as_m<kSpec, kSparse, kNet, true>(p, grid, block, st, ev);
      else if (InputAlphabet<G>::value > static_cast<uint32_t>(p.fan_k))
        return launch_p2p_as_m<kSpec, kSparse, kNet, true>(p, grid, block, st, ev);
    }
    return launch_p2p_as_m<kSpec, kSparse, kNet, false>(p, grid, block, st, ev);
  }
  hipError_t launch_p2p(const P2PParams& p, int block, hipStream_t st, const LaunchEv& ev) const override {
    const int grid = (p.Spad * G::kLanes + block - 1) / block;
    if (p.packets) {  // packet-fed ticks (rb_p2p_run_ticks_packets: the plain path, lock-step ticks)
      size_t lds = p2p_lds_bytes<G>(block);
      if constexpr (p2p_lds_queue<G>()) {
        if (p2p_lds_cells<G>(p.W, block) && p.T >= kLdsCellsMinTicks) {
          auto k = p2p_kernel<G, false, false, false, true, false, true>;
          lds = p2p_lds_bytes<G, true>(block) + p2p_lds_cell_bytes<G>(block, p.W);
          hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(lds));
          if (e != hipSuccess) return e;
          return rb_launch(k, dim3(grid), dim3(block), static_cast<uint32_t>(lds), st, ev, p);
        }
      }
      if (p.T == 1)  // one tick per launch (kOne, above)
        return rb_launch(p2p_kernel<G, false, false, false, false, false, true, false, false, true>, dim3(grid),
                         dim3(block), static_cast<uint32_t>(lds), st, ev, p);
      return rb_launch(p2p_kernel<G, false, false, false, false, false, true>, dim3(grid), dim3(block),
                       static_cast<uint32_t>(lds), st, ev, p);
    }
    if (p.ds.interval > 0 || p.peer.on) {  // desync detection / peers' connect-status reports on
      if (p.sparse)  // sparse saving and the fan-out exclude each other (rb_p2p_create)
        return launch_p2p_as<false, true, true>(p, grid, block, st, ev);
      if (kFanout && p.spec_on && !p.peer.on)  // the fan-out assumes connected queues
        return launch_p2p_as<kFanout, false, true>(p, grid, block, st, ev);
      return launch_p2p_as<false, false, true>(p, grid, block, st, ev);
    }
    if (p.sparse) return launch_p2p_as<false, true, false>(p, grid, block, st, ev);
    if (kFanout && p.spec_on) return launch_p2p_as<kFanout, false, false>(p, grid, block, st, ev);
    return launch_p2p_as<false, false, false>(p, grid, block, st, ev);
  }
  // fan-out: one lane per player (ex_game) or one wave per session (the brawler), 1-byte inputs
  static constexpr bool kFanout = ((G::kLanes > 1 && G::kLanes <= 4) || G::kLanes == 64) && G::kInputBytes == 1;
  hipError_t launch_fanout(const FanParams& p, int block, hipStream_t st) const override {
    if constexpr (kFanout) {
      const int grid = (p.Spad * kSpecBranches * G::kLanes + block - 1) / block;
      hipLaunchKernelGGL(fanout_kernel<G>, dim3(grid), dim3(block), 0, st, p);
      return hipGetLastError();
    } else {
      return hipErrorNotSupported;
    }
  }
};


// per-translation-unit factories (ops_*.hip); nullptr for an unsupported player count
std::unique_ptr<GameOps> make_exgame_ops(int players, bool lane_per_session);
std::unique_ptr<GameOps> make_brawler_ops(int players);
std::unique_ptr<GameOps> make_stub_ops(int game, int players);
// a game registered with rb_register_game_plugin (engine.hip); nullptr if unknown
std::unique_ptr<GameOps> make_plugin_ops(int game, int players);

inline std::unique_ptr<GameOps> make_game(int game, int players, bool lane_per_session) {
  switch (game) {
    case RB_GAME_EX_GAME: return make_exgame_ops(players, lane_per_session);
    case RB_GAME_BRAWLER: return make_brawler_ops(players);
    case RB_GAME_STUB:
    case RB_GAME_STUB_ENUM:
    case RB_GAME_STUB_RANDOM_CS: return make_stub_ops(game, players);
    default: return game >= RB_GAME_PLUGIN_BASE ? make_plugin_ops(game, players) : nullptr;
  }
}

}  // namespace rb
