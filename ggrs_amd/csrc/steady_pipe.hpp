// ggrs_amd/csrc/steady_pipe.hpp — the fused steady-state SyncTest ticks with
// two ticks in flight per lane (included by kernels.hpp after steady_kernel).
//
// The request stream of one steady tick at current frame c (check distance
// CD, sync_test_session.rs:89-132, 178-203) is CD+1 units
//   u0 = LoadGameState(c-CD), AdvanceFrame
//   uk = SaveGameState(c-CD+k) [+ first-seen compare, or record at k = CD], AdvanceFrame
// and each unit's AdvanceFrame depends on the previous one: one tick is a
// serial chain of CD+1 AdvanceFrames.  steady_kernel runs the ticks of a
// launch one after the other, so a lane has exactly one chain in flight and,
// at the two waves per SIMD that 65,536 two-lane sessions give, the SIMD
// spends most cycles waiting on dependent results.
//
// Tick t+1 only needs the cell tick t saves at u1 (its LoadGameState of frame
// c+1-CD).  So here tick t+1 starts while tick t is halfway: with U = CD+1
// units and H = U/2, iteration i runs tick i's units H..CD and tick i+1's
// units 0..H-1 in lock-step pairs (one unit of each per slot), two independent
// chains per lane.  Every request still executes against memory in an order
// the reference's sequential order cannot tell apart:
//  * tick t+1 loads cell c+1-CD after tick t stored it (same lane and address:
//    program order);
//  * each frame tick t+1 saves (c+2-CD .. c) was saved by tick t at the unit
//    one later in tick t's stream, which runs in an earlier slot or earlier in
//    the same slot: the final cell is tick t+1's, as in the reference;
//  * tick t+1's first-seen compare of frame c (its unit CD-1) runs in the next
//    iteration, after tick t recorded it (unit CD);
//  * if tick t reports MismatchedChecksum the session stops after tick t (it
//    is frozen, as the reference's advance_frame keeps returning Err): tick
//    t+1 has then run only units 0..H-1, whose stores rewrite cells tick t
//    wrote in the same tick with the same bytes (the game is deterministic
//    and tick t+1 resimulates from tick t's own cell), and its first store of
//    a new frame (c+1, unit CD) never happens.
// Only deterministic checksums qualify (G::kHasPrep games: ex_game); the
// random-checksum stub keeps steady_kernel.
//
// The units run the branch-free AdvanceFrame (ExGame::advance_prepared_fast)
// on the in-range sincos; a lane whose operands that form does not cover (a
// rotation outside [+0, 6.5), a clamp with a zero or tiny component) flags the
// iteration, and the wave then runs the whole iteration again in the general
// form from the state it started with: the same requests re-executed over the
// same addresses in program order.
#pragma once

#ifndef RB_PIPE_FAST
#define RB_PIPE_FAST 0  // 1: units run ExGame::advance_prepared_fast with the iteration redo (A/B builds)
#endif

namespace rb {

template <class G, int CD>
__global__ void __launch_bounds__(256) steady_pipe_kernel(const RunParams p) {
  static_assert(G::kHasPrep && HasFast<G>::value, "two ticks in flight: phase-split games with a fast AdvanceFrame");
  static_assert(CD >= 3 && CD % 2 == 1, "two ticks in flight: an even number of units per tick");
  using InRec = typename G::InRec;
  using CS = typename G::CS;
  using Dec = typename G::Dec;
  constexpr int NW = G::NWL;
  constexpr unsigned L = G::kLanes;
  constexpr int P = G::kPlayers, IB = G::kInputBytes;
  constexpr int U = CD + 1, H = U / 2;
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
  auto slot_after = [W](unsigned slot0, int k) {
    const unsigned sl = slot0 + static_cast<unsigned>(k);
    return sl >= static_cast<unsigned>(W) ? sl - static_cast<unsigned>(W) : sl;
  };
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
  // InputQueue::input of a confirmed frame (see steady_kernel)
  auto input_of_frame = [&](int fr) -> InRec {
    const int tt = min(fr - p.delay - p.c0, p.T - 1);  // (a clamp for the last iteration's unused prefetch)
    const InRec a = new_input(tt >= 0 ? tt : 0);
    const InRec b = ring[static_cast<unsigned>(fr & (kQueueLen - 1)) * Spad + s];
    return tt >= 0 ? a : b;
  };

  // One tick in flight: its state, its prepared rotation chain and thrusts,
  // the frame its LoadGameState read, the first mismatch it found.
  struct Tick {
    uint32_t w[NW];
    typename G::template Prep<U> prep;
    int32_t f0;
    unsigned slot0;
    int32_t mismatch;
  };
  // Windows, relative to tick A (the older tick in flight, frames f0A ..):
  //   dec[k]  decoded input of frame f0A + k, k = 0 .. U (A reads 0 .. CD, B reads 1 .. U)
  //   fsw[k]  first-seen checksum of frame f0A + 1 + k, k = 0 .. CD-1 (A compares 0 .. CD-2,
  //           B compares 1 .. CD-1; fsw[CD-1] is frame cA, which A records at its last unit)
  Dec dec[U + 1];
  CS fsw[CD];
  Tick A, B;
  [[maybe_unused]] CS pc{};  // Game::periodic_checksum, carried through the launch
  if constexpr (G::kDisplay) pc = reinterpret_cast<const CS*>(p.periodic_cs)[s];

  // ---- prologue: tick 0 of the launch enters as B
  B.f0 = p.c0 - CD;
  B.slot0 = slot_of(B.f0);
  B.mismatch = kNullFrame;
  load_words<NW>(p.snap + B.slot0 * slot_words, static_cast<int>(Gpad), static_cast<int>(g), B.w);
  // dec is kept relative to A = the tick before B, so B's frames are dec[1 ..]
#pragma unroll
  for (int k = 1; k <= U; ++k) dec[k] = G::decode(input_of_frame(B.f0 + k - 1), lane);
  dec[0] = dec[1];  // (A does not exist yet)
  // fsw[k] = frame f0A + 1 + k = B.f0 + k: B compares fsw[1 .. CD-1] (recorded before the launch)
#pragma unroll
  for (int k = 1; k < CD; ++k) fsw[k] = fsa[slot_of(B.f0 + k) * Spad + s];
  fsw[0] = fsw[1];
  InRec newin = new_input(0);  // tick 0's new input (ring store)
  uint32_t wn[NW];             // the next B's LoadGameState, issued after the current B saves it (unit 1)
#pragma unroll
  for (int i = 0; i < NW; ++i) wn[i] = 0u;
#pragma unroll
  for (int i = 0; i < NW; ++i) settle(B.w[i]);
#pragma unroll
  for (int k = 0; k < CD; ++k) settle(fsw[k]);
  settle(newin);

  // Unit k of tick X: [SaveGameState + compare/record], AdvanceFrame.  `fs_k` is
  // the first-seen checksum the save compares with (k < CD).  kLoadNext: issue
  // the next tick's LoadGameState right after this unit's store (k == 1).
  auto unit = [&](Tick& X, int k, CS fs_k, CS& recorded, uint32_t& special, bool load_next, auto fast_tag)
      __attribute__((always_inline)) {
    constexpr bool kFast = decltype(fast_tag)::value;
    const int32_t f = X.f0 + k;
    if (k > 0) {
      CsCtx ctx{p.seed, s, 0u};
      const CS cval = G::checksum(X.w, f, lane, ctx);
      const unsigned slot = slot_after(X.slot0, k);
      store_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), X.w);
      csa[slot * Spad + s] = cval;
      if (k == CD) {
        fsa[slot * Spad + s] = cval;  // first save of frame c: first-seen
        recorded = cval;
      } else if (cval != fs_k) {
        X.mismatch = f;  // newest mismatching frame wins
      }
      if constexpr (G::kDisplay) pc = (f % 100 == 0) ? cval : pc;
      if (k == 1 && load_next)  // same lane, same address, program order: the cell just stored
        load_words<NW>(p.snap + slot * slot_words, static_cast<int>(Gpad), static_cast<int>(g), wn);
    }
    if constexpr (kFast)
      G::advance_prepared_fast(X.w, X.prep, k, special);
    else
      G::advance_prepared(X.w, X.prep, k);
  };

  const int T = p.T;
  // One iteration: A = launch tick it-1 (units H..CD) and B = launch tick it
  // (units 0..H-1).  kA / kB say which of them exist (compile time, so the
  // steady body is one basic block per slot pair and the scheduler can
  // interleave the two chains): the first iteration has only B, the last only
  // A.  Returns false when the lane's session stopped (or the launch ended).
  auto iteration = [&](int it, auto hasA_tag, auto hasB_tag) __attribute__((always_inline)) -> bool {
    constexpr bool kA = decltype(hasA_tag)::value, kB = decltype(hasB_tag)::value;
    // the next iteration's window entries, issued before this iteration's stores
    const InRec newin_next = new_input(min(it + 1, T - 1));
    const InRec next_last = input_of_frame(B.f0 + U);  // frame f0B + U: the next B's last frame
    CS recA{};
    CS unused{};
    uint32_t wA0[NW], wB0[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      wA0[i] = A.w[i];
      wB0[i] = B.w[i];
    }
    const int32_t mA0 = A.mismatch;
    // in_range_tag: B's rotations are all in [+0, 6.5) (prepare's in-range sincos); fast_tag: the
    // branch-free AdvanceFrame (its flags are returned)
    auto slots = [&](auto in_range_tag, auto fast_tag) __attribute__((always_inline)) -> uint32_t {
      constexpr bool kInRange = decltype(in_range_tag)::value;
      constexpr bool kFast = decltype(fast_tag)::value;
      uint32_t special = 0;
      if constexpr (kB) {
        Dec decB[U];  // B's frames f0B .. f0B + CD
#pragma unroll
        for (int k = 0; k < U; ++k) decB[k] = dec[k + 1];
        if constexpr (kFast) special |= G::in_range(B.w) ? 0u : 1u;
        G::template prepare<kInRange, U>(B.w, decB, B.prep, &p.counters[1]);
      }
#pragma unroll
      for (int j = 0; j < H; ++j) {
        if constexpr (kA) unit(A, H + j, H + j < CD ? fsw[H + j - 1] : CS{}, recA, special, false, fast_tag);
        // B's unit 1 always issues the next tick's LoadGameState (an unused load in the last one)
        if constexpr (kB) unit(B, j, j > 0 ? fsw[j] : CS{}, unused, special, true, fast_tag);
      }
      return special;
    };
    if constexpr (!RB_PIPE_FAST) {
      // the general AdvanceFrame (branches around the rare paths), on the in-range sincos when
      // B's whole wave starts in range (A's prep was chosen the same way one iteration earlier)
      if (!kB || __all(G::in_range(B.w)))
        slots(std::true_type{}, std::false_type{});
      else
        slots(std::false_type{}, std::false_type{});
    } else if (__any(slots(std::true_type{}, std::true_type{}) != 0u)) {
      // a lane met an operand outside the fast form: the wave re-runs the iteration exactly
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        A.w[i] = wA0[i];
        B.w[i] = wB0[i];
      }
      A.mismatch = mA0;
      B.mismatch = kNullFrame;
      slots(std::false_type{}, std::false_type{});
    }
    if constexpr (kA) {
      const int32_t cA = A.f0 + CD;
      if constexpr (G::kDisplay) {
        // Game::last_checksum after A's final AdvanceFrame (frame cA+1) and the periodic checksum,
        // as the session leaves the launch (its last tick, or the tick it stops)
        if (!kB || A.mismatch != kNullFrame) {
          CsCtx ctx{p.seed, s, 0u};
          const CS cval = G::checksum(A.w, cA + 1, lane, ctx);
          reinterpret_cast<CS*>(p.last_cs)[s] = cval;
          pc = ((cA + 1) % 100 == 0) ? cval : pc;
          reinterpret_cast<CS*>(p.periodic_cs)[s] = pc;
        }
      }
      if (A.mismatch != kNullFrame) {  // the session stops after tick A: B never happened
        store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), A.w);
        if (lead) {
          p.err[s] = A.mismatch;
          p.live_frame[s] = cA + 1;
          atomicOr(&p.frozen[s >> 6], 1ull << (s & 63));
          atomicAdd(&p.counters[0], 1u);
        }
        return false;
      }
      if constexpr (!kB) {
        if (p.live_out_last) store_words<NW>(p.live, static_cast<int>(Gpad), static_cast<int>(g), A.w);
        return false;
      }
    }
    if constexpr (kB) {
      // ---- B's add_local_input (InputQueue::add_input, frame cB + delay), now that A did not stop
      // the session (B never reads it back: its inputs come from the input buffer)
      ring[static_cast<unsigned>((B.f0 + CD + p.delay) & (kQueueLen - 1)) * Spad + s] = newin;
      // ---- rotate: B becomes A; the next B loads the cell B saved at its unit 1
      settle(static_cast<uint32_t>(newin_next));
      settle(static_cast<uint32_t>(next_last));
#pragma unroll
      for (int i = 0; i < NW; ++i) settle(wn[i]);
#pragma unroll
      for (int k = 0; k < U; ++k) dec[k] = dec[k + 1];
      dec[U] = G::decode(next_last, lane);
      if constexpr (kA) fsw[CD - 1] = recA;  // frame cA, first recorded by A: the new A compares it at unit CD-1
#pragma unroll
      for (int k = 0; k + 1 < CD; ++k) fsw[k] = fsw[k + 1];
      A = B;
      B.f0 = A.f0 + 1;
      B.slot0 = slot_after(A.slot0, 1);
      B.mismatch = kNullFrame;
#pragma unroll
      for (int i = 0; i < NW; ++i) B.w[i] = wn[i];
      newin = newin_next;
    }
    return true;
  };
  if (!iteration(0, std::false_type{}, std::true_type{})) return;
  for (int it = 1; it < T; ++it)
    if (!iteration(it, std::true_type{}, std::true_type{})) return;
  iteration(T, std::true_type{}, std::false_type{});
}

}  // namespace rb
