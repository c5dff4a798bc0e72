/* ===========================================================================
 * ggrs_amd_game.hpp — the device-handler contract for a user's game.
 *
 * The reference's drop-in surface for a game is the `Config` trait (Input:
 * Pod, State: Clone; lib.rs:240-262) plus the user's `handle_requests`, which
 * executes SaveGameState / LoadGameState / AdvanceFrame (ex_game.rs:76-112).
 * In the batched engine the requests are executed on the GPU, so a game is
 * device code: a struct with the members below, compiled against the engine's
 * kernels into a plugin library (ggrs_amd/csrc/plugin.hip; build hook
 * `make -C ggrs_amd/csrc plugin GAME_HEADER=... GAME=... PLUGIN_OUT=...` or
 * ggrs_amd.plugin.build_game_plugin) and registered at run time with
 * rb_register_game_plugin (include/ggrs_amd.h), which returns the game id to
 * put in rb_config.game / rb_p2p_config.game.
 *
 * What the engine does with it (one lane per session, state in registers):
 *   LoadGameState   the cell's words are loaded                 (no user code)
 *   SaveGameState   checksum(words, frame) is stored with the
 *                   words (GameStateCell::save(frame, Some(state), Some(checksum)))
 *   AdvanceFrame    advance(words, inputs, status)
 * The frame counter is not part of `words`: every handler asserts
 * state.frame == cell frame on save (ex_game.rs:89), so the engine supplies it.
 *
 *   struct MyGame {
 *     static constexpr int kPlayers = 2;      // num_players of every session (1..4)
 *     static constexpr int kStateWords = 6;   // u32 words of one session's state
 *     static constexpr int kInputBytes = 1;   // size of one player's Input (1, 2 or 4; kPlayers * kInputBytes <= 8)
 *     using Checksum = uint64_t;              // uint16_t, uint32_t or uint64_t (zero-extended to the u128)
 *     // State::new for one session (host)
 *     static void init(uint32_t* words);
 *     // one AdvanceFrame{inputs}: inputs[p] is player p's Input (little endian, zero-extended),
 *     // status[p] its InputStatus (0 Confirmed, 1 Predicted, 2 Disconnected: input zeroed)
 *     RB_GAME_FN static void advance(uint32_t* words, const uint32_t* inputs, const uint8_t* status);
 *     // the checksum save_game_state stores for the state at `frame`
 *     RB_GAME_FN static Checksum checksum(const uint32_t* words, int32_t frame);
 *   };
 *
 * RB_GAME_FN makes the two functions callable on the device AND the host;
 * that is what lets the CPU oracle (oracle/, test infrastructure) run the
 * same game through its restatement of SyncTestSession / P2PSession for
 * parity tests (oracle/plugin_oracle.cpp).  Write them in plain integer /
 * IEEE C++ (no device intrinsics) so both compilations compute the same bits.
 *
 * The canonical byte image of a session (rb_read_cell, rb_read_live) is
 * le32(frame) || le32(words[0]) || ... || le32(words[kStateWords - 1]).
 * ======================================================================== */
#ifndef GGRS_AMD_GAME_HPP
#define GGRS_AMD_GAME_HPP

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define RB_GAME_FN __host__ __device__ inline
#else
#define RB_GAME_FN inline
#endif

/* ABI of the plugin entry points (rb_plugin_abi); bump when the engine's
 * kernel parameter structs or the layout of the state they point to change
 * (7: the packed P2P bookkeeping rows). */
#define RB_PLUGIN_ABI 7

#endif /* GGRS_AMD_GAME_HPP */
