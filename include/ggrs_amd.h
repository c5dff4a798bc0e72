/* ===========================================================================
 * ggrs_amd.h — C ABI of the MI355X batched rollback-resimulation engine.
 *
 * Drop-in boundary for the GGRS 0.9.4 resimulation path (/root/reference):
 * a batch of S lock-step SyncTestSessions whose request stream
 * (SaveGameState / LoadGameState / AdvanceFrame, lib.rs:170-194) is produced
 * by host-side bookkeeping identical to the reference and executed on the GPU
 * by compiled-in game handlers (the user's `handle_requests`, ex_game.rs:76-84).
 *
 * Plain C types only (no torch, no HIP types in signatures): a Rust `extern
 * "C"` block, a ctypes stub or a C++ wrapper binds it directly; see
 * INTEGRATION.md.  Every entry point names the reference interface it
 * replaces.
 *
 * Threading: one batch = one HIP stream; calls on one batch are not reentrant.
 * Different batches (e.g. one per GPU) may be driven from different threads.
 * No exception or panic crosses the ABI: every call returns rb_status.
 * ======================================================================== */
#ifndef GGRS_AMD_H
#define GGRS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RB_ABI_VERSION 1
#define RB_NULL_FRAME (-1) /* lib.rs:46 NULL_FRAME */
#define RB_INPUT_QUEUE_LENGTH 128 /* input_queue.rs:6 */

/* GGRSError (error.rs:11-36) as status codes, plus engine-side failures. */
typedef enum rb_status {
  RB_OK = 0,
  RB_PREDICTION_THRESHOLD = 1,     /* GGRSError::PredictionThreshold          error.rs:13 */
  RB_INVALID_REQUEST = 2,          /* GGRSError::InvalidRequest{info}         error.rs:15-18 (info: rb_last_error) */
  RB_MISMATCHED_CHECKSUM = 3,      /* GGRSError::MismatchedChecksum{frame}    error.rs:22-25 (per session: rb_mismatches) */
  RB_NOT_SYNCHRONIZED = 4,         /* GGRSError::NotSynchronized              error.rs:27 */
  RB_SPECTATOR_TOO_FAR_BEHIND = 5, /* GGRSError::SpectatorTooFarBehind        error.rs:29 */
  RB_DEVICE_ERROR = 100,           /* HIP runtime failure (no reference analogue) */
  RB_PANIC = 101                   /* a reference assert!/panic! condition was hit (API misuse) */
} rb_status;

/* Compiled-in game handlers (the `Config` trait's State/Input + handle_requests). */
typedef enum rb_game {
  RB_GAME_EX_GAME = 1,        /* examples/ex_game/ex_game.rs: f32 ships, Input{inp:u8}, fletcher16 over the bincode image */
  RB_GAME_STUB = 2,           /* tests/stubs.rs GameStub: i32 state, StubInput{inp:u32}, SipHash-1-3 checksum */
  RB_GAME_STUB_ENUM = 3,      /* tests/stubs_enum.rs GameStubEnum: #[repr(u8)] enum input */
  RB_GAME_STUB_RANDOM_CS = 4, /* tests/stubs.rs RandomChecksumGameStub: random u128 checksums (forces mismatches) */
  RB_GAME_BRAWLER = 5         /* BASELINE config 3: fixed-point 256-entity brawler, 8 KiB state, Input{inp:u8}, fletcher16;
                                 no reference game exists: defined in oracle/ggrs_oracle.hpp */
} rb_game;

/* Games compiled outside the engine (include/ggrs_amd_game.hpp: the `Config`
 * trait + handle_requests of the user's game as device code, built into a
 * plugin library by ggrs_amd/csrc/plugin.hip).  rb_register_game_plugin
 * loads one and returns its game id (RB_GAME_PLUGIN_BASE + k), valid for
 * rb_config.game and rb_p2p_config.game from then on.  Registering the same
 * path twice returns the same id.  RB_INVALID_REQUEST: the library cannot be
 * loaded, lacks the entry points or was built for another plugin ABI. */
#define RB_GAME_PLUGIN_BASE 1000
rb_status rb_register_game_plugin(const char* path, int32_t* game_id);

/* GGRSRequest kinds (lib.rs:170-194) for rb_last_requests. */
typedef enum rb_request_kind { RB_REQ_SAVE = 0, RB_REQ_LOAD = 1, RB_REQ_ADVANCE = 2 } rb_request_kind;

#define RB_FLAG_CHECKED 1u          /* advance_frame reports MismatchedChecksum synchronously, like the reference (default) */
#define RB_FLAG_LANE_PER_SESSION 2u /* ex_game: one lane per session instead of one lane per player; only
                                       libraries built with RB_EXPERIMENTS=1 accept it (the product library
                                       refuses it at create with RB_INVALID_REQUEST) */

/* SessionBuilder fields used by start_synctest_session (builder.rs:32-52). */
typedef struct rb_config {
  int32_t abi_version;    /* = RB_ABI_VERSION */
  int32_t game;           /* rb_game */
  int32_t num_sessions;   /* batch size S (independent sessions in lock-step) */
  int32_t num_players;    /* with_num_players          builder.rs:154-157 (default 2) */
  int32_t max_prediction; /* with_max_prediction_window builder.rs:136-145 (default 8, >0, <= 64 here) */
  int32_t check_distance; /* with_check_distance       builder.rs:202-205 (default 2, < max_prediction) */
  int32_t input_delay;    /* with_input_delay          builder.rs:148-151 (default 0) */
  int32_t device;         /* HIP device ordinal; -1 = plan-only batch (host bookkeeping, no device work) */
  uint64_t seed;          /* RB_GAME_STUB_RANDOM_CS only */
  uint32_t flags;         /* RB_FLAG_* */
  uint32_t block_size;    /* 0 = default; kernel tuning knob */
  uint32_t reserved[6];
} rb_config;

typedef struct rb_batch rb_batch;

/* Checksum report record (mirrors messages.rs:75-79 ChecksumReport{checksum:u128, frame}
 * + the session's desync flag) written to device memory by rb_export_checksum_report. */
typedef struct rb_checksum_report {
  uint64_t checksum_lo;
  uint64_t checksum_hi;
  int32_t frame;
  int32_t mismatch_frame; /* RB_NULL_FRAME when the session is healthy */
} rb_checksum_report;

/* SessionBuilder::new() defaults (builder.rs:13-27, 62-78). */
void rb_config_init(rb_config* cfg);

/* SessionBuilder::start_synctest_session (builder.rs:342-354) for S sessions.
 * Validation errors as in the reference ("Check distance too big.", zero
 * prediction window) -> RB_INVALID_REQUEST; *out = NULL and the message via
 * rb_last_error(NULL). */
rb_status rb_synctest_create(const rb_config* cfg, rb_batch** out);
void rb_destroy(rb_batch* b);

/* Last error message of this batch (or of the failed create when b == NULL). */
const char* rb_last_error(const rb_batch* b);

/* Run this batch on a caller-owned hipStream_t (passed as void*); NULL = the
 * batch's own stream. */
rb_status rb_set_stream(rb_batch* b, void* hip_stream);
/* The hipStream_t the batch runs on (its own one unless rb_set_stream chose
 * another); NULL for a plan-only batch.  Callers order their own streams
 * against it (ggrs_amd/session.py _StreamOrdered). */
void* rb_get_stream(const rb_batch* b);

/* SyncTestSession::add_local_input (sync_test_session.rs:61-74) for every
 * session at once: `inputs` holds S values of the game's Input type
 * (ex_game: u8, stub: u32, enum: u8) for player `handle`; host or device
 * pointer.  Device pointers must stay valid until the next advance has run
 * (stream order).  Overwrites an earlier call for the same handle.
 * handle >= num_players -> RB_INVALID_REQUEST. */
rb_status rb_add_local_input(rb_batch* b, int32_t handle, const void* inputs, int32_t on_device);

/* All players at once, packed [S][num_players] Input values. */
rb_status rb_add_local_inputs_packed(rb_batch* b, const void* inputs, int32_t on_device);

/* SyncTestSession::advance_frame (sync_test_session.rs:85-146) followed by
 * the game's handle_requests on every session, fused into one device launch.
 * Returns RB_INVALID_REQUEST (missing input), RB_PREDICTION_THRESHOLD, or —
 * with RB_FLAG_CHECKED — RB_MISMATCHED_CHECKSUM when at least one session's
 * advance_frame returned Err(MismatchedChecksum) in this call.  A session that
 * failed does not advance (as in the reference, where every retry fails the
 * same way); the others do.  Without RB_FLAG_CHECKED the call is fully
 * asynchronous and mismatches are read with rb_mismatches. */
rb_status rb_advance_frame(rb_batch* b);

/* n_ticks x (add_local_input for every handle + advance_frame) in one call:
 * tick t reads its inputs at inputs + t*tick_stride_bytes, laid out
 * [num_players][num_sessions] Input values (host or device memory).  The host
 * bookkeeping runs tick by tick as in rb_advance_frame; consecutive
 * steady-state ticks (current frame > check_distance, 1 <= check_distance <= 16)
 * execute as ONE fused device launch (for games of at most 80 B of state per
 * cell, e.g. ex_game and the stubs, while the batch's snapshot ring is below
 * 4 GiB: ex_game P=2, W=8 holds 40 B per session per slot, 320 B per session,
 * so up to 13.4M sessions; larger rings run one launch per tick, same results).  A session whose resimulation
 * mismatches stops advancing (as with per-tick calls) while the others run
 * on; with RB_FLAG_CHECKED the call returns RB_MISMATCHED_CHECKSUM if any
 * session has failed by its end.  Bookkeeping errors (RB_INVALID_REQUEST,
 * RB_PREDICTION_THRESHOLD, RB_PANIC) stop the run; *ticks_done = completed ticks. */
rb_status rb_run_ticks(rb_batch* b, int32_t n_ticks, const void* inputs, int64_t tick_stride_bytes,
                       int32_t on_device, int32_t* ticks_done);

/* SyncLayer::current_frame of the batch (sync_layer.rs:110-112). */
int32_t rb_current_frame(const rb_batch* b);
int32_t rb_num_sessions(const rb_batch* b);
/* Bytes of one session's canonical state image (ex_game: the bincode image,
 * 36+20*P; stubs: le32 frame || le32 state) and of one Input value. */
int32_t rb_state_bytes(const rb_batch* b);
int32_t rb_input_bytes(const rb_batch* b);

/* Wait for all work queued on the batch's stream. */
rb_status rb_synchronize(rb_batch* b);

/* Per-session MismatchedChecksum{frame} (RB_NULL_FRAME when healthy) and the
 * count of failed sessions.  Synchronises. */
rb_status rb_mismatches(rb_batch* b, int32_t* frames_out, int32_t* count_out);

/* The (kind, frame) list of the request stream the last rb_advance_frame
 * executed, identical to the Vec<GGRSRequest> the reference returns
 * (AdvanceFrame carries the frame it advances from).  Returns the count. */
int32_t rb_last_requests(const rb_batch* b, int32_t* kinds, int32_t* frames, int32_t cap);

/* GameStateCell::{load, checksum} (sync_layer.rs:28-39) for the cell holding
 * `frame`: images [S][rb_state_bytes], checksums [S][2] (u128 lo, hi).
 * RB_INVALID_REQUEST if no cell holds that frame.  Synchronises. */
rb_status rb_read_cell(rb_batch* b, int32_t frame, void* images, uint64_t* checksums);

/* The game's live state after the last advance (ex_game Game::game_state,
 * images [S][rb_state_bytes]) and its display checksum with its frame
 * (Game::last_checksum, ex_game.rs:104-111; [S] each; RB_NULL_FRAME for games
 * without one).  A failed session reports the state it stopped at.  Synchronises. */
rb_status rb_read_live(rb_batch* b, void* images, uint64_t* display_checksums, int32_t* display_frames);

/* Desync report for the cell holding `frame` into device memory [S]
 * rb_checksum_report (the P2P ChecksumReport payload; multi-GPU allgather
 * input).  Stream-ordered, does not synchronise. */
rb_status rb_export_checksum_report(rb_batch* b, int32_t frame, void* dev_out);

/* The same report in 4 bytes per session, for games whose checksum is 16 bits
 * (ex_game's fletcher16): dev_out[S] uint32 records
 *   bits 0-15   the checksum of the cell holding `frame` (ChecksumReport::checksum)
 *   bits 16-30  frame - mismatch_frame, saturated at 0x7FFF (0 when healthy)
 *   bit  31     the session reports MismatchedChecksum
 * The report frame (ChecksumReport::frame, messages.rs:75-79) is batch-uniform in
 * SyncTest, so it travels once per all-gather instead of once per session: the
 * multi-GPU gather moves 4 B per session instead of 24.  RB_INVALID_REQUEST for a
 * game with a wider checksum (use rb_export_checksum_report).  Stream-ordered. */
rb_status rb_export_compact_report(rb_batch* b, int32_t frame, void* dev_out);

/* Fault injection for tests: XOR `xor_mask` into state word `word` of
 * `session` in the cell holding `frame` (a corrupted snapshot makes the next
 * resimulation diverge, which SyncTest must report). */
rb_status rb_debug_corrupt_cell(rb_batch* b, int32_t session, int32_t frame, int32_t word, uint32_t xor_mask);

/* Device evaluation of the game's sin/cos (the glibc sinf/cosf restatement in
 * device_math.hpp) for n host floats, on `device` — pins it against the host
 * libm in the parity tests. */
rb_status rb_debug_sincosf(int32_t device, const float* x, float* sin_out, float* cos_out, int64_t n);

/* The in-range forms of the same arithmetic the fused steady ticks and the fan-out run
 * (sincosf_glibc<true>, and the rotation step rem_euclid(x +- ROTATION_SPEED, 2 pi),
 * ex_game.rs:282-296, as rem_euclid_near<true> and rem_euclid<true>) for the n floats whose
 * bits are first_bits, first_bits + 1, ... (all in [+0, 6.5)), into device memory dev_out
 * [6][n] (sin, cos, step up, step down, step up, step down).  Synchronises. */
rb_status rb_debug_exgame_inrange(int32_t device, uint32_t first_bits, int64_t n, float* dev_out);

/* Device evaluation of ex_game's speed clamp (ex_game.rs:300-304: v * MAX_SPEED
 * / |v| when |v| > MAX_SPEED) for n host (vx, vy) pairs — pins the short exact
 * sqrt/division sequences of device_math.hpp against host IEEE arithmetic. */
rb_status rb_debug_speed_clamp(int32_t device, const float* vx, const float* vy, float* vx_out, float* vy_out,
                               int64_t n);

/* HIP event timing of the tick kernel on the batch's stream, for bench.py:
 * rb_profile_enable(b, k) brackets every k-th single-tick launch (k <= 1:
 * every 8th) and every fused rb_run_ticks launch with an event pair;
 * rb_profile_take returns the summed milliseconds of the timed launches and
 * the number of ticks they covered, and resets both. */
rb_status rb_profile_enable(rb_batch* b, int32_t on);
rb_status rb_profile_take(rb_batch* b, double* total_ms, int32_t* launches);

/* The kernel's own clock (measurement only, no reference counterpart: bench.py's
 * kernel time).  rb_launch_clock_arm(b, n): the next n fused steady launches
 * (rb_run_ticks) have every wave store its start and end on the chip's 100 MHz
 * constant clock into a slot of their own (cleared here, once: nothing is added
 * to the launches' stream).  rb_launch_clock_read(b, out[2 * cap], cap, &n)
 * waits for the stream, returns per launch the first wave's start and the last
 * wave's end in 10 ns ticks, and disarms.  No host call or event sits between
 * the two readings and a profiler does not change them; the dispatch's own
 * setup and end-of-kernel release fall outside them (bench.py adds the
 * calibrated difference to rocprofv3's dispatch duration). */
rb_status rb_launch_clock_arm(rb_batch* b, int32_t launches);
rb_status rb_launch_clock_read(rb_batch* b, uint64_t* start_end, int32_t cap, int32_t* launches);

/* ===========================================================================
 * P2PSession batches (sessions/p2p_session.rs) — the rollback path.
 *
 * S independent P2P sessions seen from one peer, each with num_players
 * handles: bit h of local_mask set = add_player(PlayerType::Local, h), clear =
 * PlayerType::Remote (builder.rs:90-128).  The network layer is not part of
 * the batch: UdpProtocol's role on this path, turning packets into
 * Event::Input{input, player} in frame order (p2p_session.rs:838-852), is the
 * caller's: per tick and remote handle it passes the newest delivered frame
 * (`remote_upto`) and the inputs by frame (`remote_inputs`).  Mispredicted
 * remote inputs roll sessions back individually (per-session depth), on the
 * device.  rb_p2p_disconnect_player covers disconnects the user issues;
 * peer-reported disconnects arrive through rb_p2p_receive_peer_connect_status
 * (RB_P2P_FLAG_PEER_STATUS, below).  Spectators and time sync are out of scope.
 * ======================================================================== */
typedef struct rb_p2p rb_p2p;

typedef struct rb_p2p_config {
  int32_t abi_version;    /* = RB_ABI_VERSION */
  int32_t game;           /* rb_game: RB_GAME_EX_GAME, RB_GAME_STUB, RB_GAME_STUB_ENUM, RB_GAME_BRAWLER */
  int32_t num_sessions;
  int32_t num_players;    /* with_num_players (builder.rs:154-157) */
  int32_t max_prediction; /* with_max_prediction_window (builder.rs:136-145) */
  int32_t input_delay;    /* with_input_delay (builder.rs:148-151): local handles */
  int32_t device;
  uint32_t local_mask;    /* bit h: handle h is PlayerType::Local; at least one local and one remote */
  int32_t remote_delay;   /* frame of each remote handle's first Event::Input (the peer's input delay) */
  int32_t sparse_saving;  /* with_sparse_saving_mode (builder.rs:159-166) */
  uint32_t flags;         /* RB_FLAG_LANE_PER_SESSION, RB_P2P_FLAG_FANOUT, RB_P2P_FLAG_PEER_STATUS */
  uint32_t block_size;
  int32_t desync_interval; /* with_desync_detection_mode (builder.rs:167-172): DesyncDetection::On{interval}
                              for interval > 0, Off for 0 (the default, builder.rs:15) */
  int32_t fanout_candidates; /* RB_P2P_FLAG_FANOUT: branches per session, 1..16 (default 16) */
  uint32_t fanout_min_select_permille; /* adaptive fan-out (RB_P2P_FLAG_FANOUT without _ALWAYS): the
                              select fraction of rollbacks below which the batch turns it off;
                              0 = the default, 150 */
  uint32_t reserved[1];
} rb_p2p_config;

/* Speculative branch fan-out (BASELINE config 4): after every tick each session
 * presimulates K = fanout_candidates branches (at most 16), one per candidate
 * input of the remote handle with the oldest unconfirmed input, over its
 * unconfirmed frames.  The candidates are the game's whole input alphabet when
 * it has at most K values (ex_game's 4 input bits, K = 16), else the K most
 * likely values: the most recently confirmed distinct inputs of that handle,
 * newest first (the reference's repeat-last prediction, input_queue.rs:126-140,
 * is candidate 0), then the smallest values not taken.  A later misprediction
 * of that handle alone, held at one candidate value, becomes a branch select
 * instead of LoadGameState + resimulation; cells, states, statuses and frames
 * stay identical to the plain rollback.  Candidates that act alike on the
 * player share one branch (ex_game's 16 inputs are 9 trajectories).  ex_game
 * (one lane per player: the fan-out runs inside the P2P tick, so a call of many
 * ticks is one launch) and the brawler (one wave per session: a fan-out launch
 * between one-tick P2P launches); not with sparse saving. */
#define RB_P2P_FLAG_FANOUT 4u

/* The fan-out is adaptive by default: a batch measures, over windows of 64
 * ticks, the fraction of its rollbacks that became selects; below
 * fanout_min_select_permille it stops presimulating for the next 960 ticks (its
 * ticks run as plain P2P ticks), then measures again.  Presimulation only pays
 * through selects: a stream whose held inputs rarely match a candidate (the
 * brawler's 256-value inputs: 3.8% of rollbacks at 20x the plain tick's cost)
 * gets plain rollback.  The measurement is asynchronous (a device reduction into
 * pinned memory, read when it has landed): no call waits for it.  Results are
 * the same either way.  RB_P2P_FLAG_FANOUT_ALWAYS keeps it on. */
#define RB_P2P_FLAG_FANOUT_ALWAYS 16u

/* Per-player speculation (with RB_P2P_FLAG_FANOUT; games whose players move
 * independently and whose whole input alphabet fits the candidates: ex_game at
 * K = 16): every remote player's input classes are presimulated, each in its
 * own lane, from the oldest first unconfirmed frame B over the remote players,
 * instead of the one remote player with that oldest frame.  A rollback from B
 * in which every remote player's newly confirmed inputs hold one class then
 * becomes a select even when several players mispredicted (the plain fan-out
 * needs the speculated player to be the only one).  More chains per tick: the
 * bench reports both forms (bench.py --fanout-mode). */
#define RB_P2P_FLAG_FANOUT_PER_PLAYER 32u

/* Peers' connect-status reports (update_player_disconnects, p2p_session.rs:707-742):
 * every advance_frame combines what the running endpoints last reported about
 * each player (rb_p2p_receive_peer_connect_status) with the session's own
 * view; a player some peer reports disconnected is disconnected here too, at
 * the earliest reported frame, with the resimulation that implies. */
#define RB_P2P_FLAG_PEER_STATUS 8u

/* SessionBuilder::new() defaults for a 2-player session, handle 0 local, handle 1 remote. */
void rb_p2p_config_init(rb_p2p_config* cfg);

/* The adaptive fan-out's state: *active (1: presimulating), the select fraction of
 * rollbacks of the last measured window (-1: none yet), the windows measured and
 * the times it was turned off.  Does not synchronise.  RB_INVALID_REQUEST without
 * the fan-out. */
rb_status rb_p2p_fanout_state(rb_p2p* b, int32_t* active, double* select_fraction, int32_t* windows,
                              int32_t* turned_off);

/* SessionBuilder::start_p2p_session (builder.rs:251-308) for S sessions that
 * start Running (the synchronisation handshake is the network's). */
rb_status rb_p2p_create(const rb_p2p_config* cfg, rb_p2p** out);
void rb_p2p_destroy(rb_p2p* b);
const char* rb_p2p_last_error(const rb_p2p* b);
rb_status rb_p2p_set_stream(rb_p2p* b, void* hip_stream);
void* rb_p2p_get_stream(const rb_p2p* b);  /* as rb_get_stream */

/* n_ticks x [poll_remote_clients + add_local_input for every local handle +
 * advance_frame (p2p_session.rs:253-337) + handle_requests] for every session,
 * in ONE device launch.  Device pointers, stream ordered:
 *   local_inputs  tick t, handle h: local_inputs + t*local_stride_bytes + (h*S + s)*input_bytes
 *                 (entries of remote handles are ignored)
 *   remote_upto   int32 [n_ticks][num_players][S]: newest frame delivered for
 *                 remote handle h before tick t's advance_frame (monotone;
 *                 entries of local handles ignored)
 *   remote_inputs [remote_frames][num_players][S] Input values by frame
 * A session that hits PredictionThreshold (sync_layer.rs:163-167) does not
 * advance that tick (rb_p2p_read_status reports it), exactly as the
 * reference's advance_frame returns Err: its bookkeeping moves, its game does
 * not.  Asynchronous (stream ordered): a session that hits a reference assert
 * stops and reports RB_PANIC through rb_p2p_read_status / rb_p2p_counters. */
rb_status rb_p2p_run_ticks(rb_p2p* b, int32_t n_ticks, const void* local_inputs, int64_t local_stride_bytes,
                           const int32_t* remote_upto, const void* remote_inputs, int32_t remote_frames);

/* rb_p2p_run_ticks with the remote inputs arriving as the peers' input packets
 * (the format of rb_encode_input_packets below): each tick first runs
 * UdpProtocol::on_input (protocol.rs:616-689) for every remote endpoint inside
 * the tick's poll_remote_clients, decoding straight into the InputQueue (one
 * launch does decode and tick; the deliveries never pass through
 * remote_upto / remote_inputs).  Device pointers, stream ordered:
 *   packets       tick t, remote handle h, session s: the packet at
 *                 packets + ((t*num_players + h)*S + s)*packet_stride;
 *                 packet_stride a multiple of 16, at least 32; the packet's
 *                 length and start frame at lengths / start_frames[(t*num_players + h)*S + s]
 *                 (length 0: none; entries of local handles ignored)
 *   decode_status NULL, or int32 [num_players][S]: the last tick's result per
 *                 endpoint (the codes of rb_decode_input_packets)
 *   acks          NULL, or int32 [num_players][S]: after the call, the newest
 *                 frame received per endpoint (RB_NULL_FRAME: none), the ack
 *                 the receiver returns to the sender
 * A malformed packet (or a length above packet_stride) panics its session
 * (the reference's decode().expect, "decoding failed", protocol.rs:656); so
 * does a packet that skips frames never received (status -2: the reference's
 * assert!, protocol.rs:639-642).  Sparse saving, the fan-out, desync
 * detection, peers' connect-status reports and max_prediction >= 64 (a
 * reference input up to 2*max_prediction frames back must still be in the
 * 128-entry input ring): RB_INVALID_REQUEST. */
rb_status rb_p2p_run_ticks_packets(rb_p2p* b, int32_t n_ticks, const void* local_inputs, int64_t local_stride_bytes,
                                   const uint8_t* packets, int64_t packet_stride, const int32_t* lengths,
                                   const int32_t* start_frames, int32_t* decode_status, int32_t* acks);

/* P2PSession::disconnect_player(handle) (p2p_session.rs:430-456, 555-581) in
 * every session whose `session_mask` byte is non-zero (NULL: all sessions),
 * called between rb_p2p_run_ticks calls (stream ordered).  Errors as the
 * reference, RB_INVALID_REQUEST with nothing applied: "Invalid Player Handle."
 * (handle >= num_players), "Local Player cannot be disconnected.", "Player
 * already disconnected." (in any selected session).  From then on the player's
 * deliveries are ignored, it leaves the confirmed frame, every frame after its
 * last one advances with (zeroed, Disconnected), and the next advance_frame
 * resimulates from last_frame + 1 if that frame was already simulated. */
rb_status rb_p2p_disconnect_player(rb_p2p* b, int32_t handle, const uint8_t* session_mask);

/* Per session, the last tick: rb_status of its advance_frame, the LoadGameState
 * frame (RB_NULL_FRAME: no rollback), AdvanceFrame and SaveGameState counts.
 * Any pointer may be NULL.  Synchronises. */
rb_status rb_p2p_read_status(rb_p2p* b, int32_t* status, int32_t* load_frame, int32_t* n_advance, int32_t* n_save);
/* SyncLayer::current_frame and last_confirmed_frame per session.  Synchronises. */
rb_status rb_p2p_read_frames(rb_p2p* b, int32_t* current, int32_t* confirmed);
/* Every session's InputQueue / ConnectionStatus bookkeeping, out[S][P][RB_P2P_QUEUE_FIELDS]:
 * last_added_frame, inputs[tail].frame, length, last_requested_frame, prediction.frame,
 * first_incorrect_frame (input_queue.rs:12-34), ConnectionStatus::last_frame and
 * disconnected (messages.rs:5-18).  For parity tests and debugging.  Synchronises. */
#define RB_P2P_QUEUE_FIELDS 8
rb_status rb_p2p_read_queues(rb_p2p* b, int32_t* out);
/* All cells: frame tags [W][S], images [W][S][rb_p2p_state_bytes], checksums [W][S][2]. */
rb_status rb_p2p_read_cells(rb_p2p* b, int32_t* tags, void* images, uint64_t* checksums);
/* The game state after the last advance, images [S][rb_p2p_state_bytes] (frame word = current frame). */
rb_status rb_p2p_read_live(rb_p2p* b, void* images);
int32_t rb_p2p_state_bytes(const rb_p2p* b);
int32_t rb_p2p_input_bytes(const rb_p2p* b);
/* Counters since create: [0] PredictionThreshold hits, [1] unexpected math paths, [2] panicked sessions. */
rb_status rb_p2p_counters(rb_p2p* b, uint32_t* out3);
/* Work the device executed since create: [0] AdvanceFrame, [1] SaveGameState,
 * [2] LoadGameState (requests dropped with a PredictionThreshold error
 * excluded), [3] rollbacks replaced by a speculative select, [4] branch frames
 * presimulated by the fan-out. */
rb_status rb_p2p_totals(rb_p2p* b, uint64_t* out5);
/* ---- Desync detection (p2p_session.rs:873-928, protocol.rs:27, 710-742) with
 * desync_interval > 0.  In every advance_frame at current % interval == 0 a
 * session records ChecksumReport{checksum, frame = last_saved_frame - 1} of its
 * cell (only when that frame > max_prediction; no such cell is a reference
 * panic -> RB_PANIC), keeps it in its local checksum history (the newest 32
 * frames), and compares the history each remote endpoint received with it:
 * every differing frame is a GGRSEvent::DesyncDetected{frame, local_checksum,
 * remote_checksum, addr}.  The reports travel between peers through the caller
 * (on one node: an all-gather, ggrs_amd/shard.py), like the datagrams
 * UdpProtocol::send_checksum_report sends. */
#define RB_P2P_REPORTS_PER_TAKE 8 /* reports kept per session between two takes (older ones are dropped, like lost datagrams) */
#define RB_P2P_EVENTS_KEPT 16     /* newest DesyncDetected events kept per session */

/* The reports every session sent since the last call, oldest first, into
 * device memory dev_out[RB_P2P_REPORTS_PER_TAKE][S] rb_checksum_report
 * (frame RB_NULL_FRAME: none; mismatch_frame unused, RB_NULL_FRAME).
 * Stream-ordered. */
rb_status rb_p2p_take_checksum_reports(rb_p2p* b, void* dev_out);

/* UdpProtocol::on_checksum_report (protocol.rs:710-722) for the endpoint of
 * remote handle `handle` of every session: dev_in[k * S + s], k < count,
 * rb_checksum_report in the layout rb_p2p_take_checksum_reports writes (the
 * peer's reports for this session), applied in order.  Stream-ordered.
 * RB_INVALID_REQUEST: handle is not a remote handle, or desync detection is off. */
rb_status rb_p2p_receive_checksum_reports(rb_p2p* b, int32_t handle, const void* dev_in, int32_t count);

/* DesyncDetected events per session: counts[S] since create, and the newest
 * RB_P2P_EVENTS_KEPT in order as frames / remote handles (the `addr`) / local /
 * remote checksum low words, each [S][RB_P2P_EVENTS_KEPT] (frame RB_NULL_FRAME,
 * handle -1: none).  Any pointer may be NULL.  Synchronises. */
rb_status rb_p2p_read_desync_events(rb_p2p* b, uint32_t* counts, int32_t* frames, int32_t* handles,
                                    uint64_t* local_checksums, uint64_t* remote_checksums);

/* UdpProtocol::on_input's merge of the peer's connect status (protocol.rs:627-636)
 * for the endpoint of remote handle `endpoint` in every session: the peer
 * reports player i as last_frames[i * S + s] / disconnected[i * S + s] (device
 * memory, [num_players][S] int32 and uint8); the stored status becomes
 * (stored.disconnected || reported, max(stored.last_frame, reported)).
 * Stream-ordered, between ticks.  RB_INVALID_REQUEST without
 * RB_P2P_FLAG_PEER_STATUS or for a local handle. */
rb_status rb_p2p_receive_peer_connect_status(rb_p2p* b, int32_t endpoint, const int32_t* last_frames,
                                             const uint8_t* disconnected);

/* Fault injection for tests (ex_game.rs:211-215 trigger_desync, generalised):
 * XOR `xor_mask` into canonical state word `word` of `session`'s live state
 * and of every cell it holds (checksums unchanged), between ticks. */
rb_status rb_p2p_debug_corrupt(rb_p2p* b, int32_t session, int32_t word, uint32_t xor_mask);

/* HIP event timing of every rb_p2p_run_ticks launch (bench.py): total ms and launches since the last take. */
rb_status rb_p2p_profile_enable(rb_p2p* b, int32_t on);
rb_status rb_p2p_profile_take(rb_p2p* b, double* total_ms, int32_t* launches);
/* rb_launch_clock_arm / _read for P2P batches: every p2p_kernel launch, and
 * with the two-launch fan-out every fanout_kernel launch, takes a slot. */
rb_status rb_p2p_launch_clock_arm(rb_p2p* b, int32_t launches);
rb_status rb_p2p_launch_clock_read(rb_p2p* b, uint64_t* start_end, int32_t cap, int32_t* launches);

/* ===========================================================================
 * Batched input packets (network/compression.rs): one
 * endpoint per (session, remote handle), one packet per endpoint per call.
 * Wire format: XOR delta of every pending input against the reference input,
 * then bitfield RLE (bitfield-rle 0.2 format).  All pointers are device
 * memory; `stream` is a hipStream_t (NULL: the null stream).
 * ======================================================================== */

/* UdpProtocol::on_input (protocol.rs:616-689) for every session's endpoint of
 * remote handle `handle`: packet s is packets + s*packet_stride, lengths[s]
 * bytes (0: none), covering frames start_frames[s]... .  It is decoded against
 * the input before its start frame (remote_inputs, or the zeroed input before
 * the first one), inputs of frames after remote_upto[handle][s] are written to
 * remote_inputs[frame][num_players][num_sessions] (input_bytes each) and
 * remote_upto advances: exactly the delivery tensors rb_p2p_run_ticks reads.
 * status[s]: 0 new inputs, 1 nothing new, -1 malformed (the reference panics:
 * "decoding failed"; also a length above packet_stride), -2 frames missing
 * before start_frame (the reference asserts).  The caller decides what a
 * negative status does to the session (nothing is decoded for it).
 * A packet whose reference input is older than 2*max_prediction frames is
 * ignored (recv_inputs retention, protocol.rs:686-688). */
rb_status rb_decode_input_packets(int32_t device, void* stream, int32_t handle, int32_t num_players,
                                  int32_t num_sessions, int32_t input_bytes, int32_t max_prediction,
                                  const uint8_t* packets, int64_t packet_stride, const int32_t* lengths,
                                  const int32_t* start_frames, void* remote_inputs, int32_t remote_frames,
                                  int32_t* remote_upto, int32_t* status);

/* UdpProtocol::send_pending_output (protocol.rs:468-500) for every session's
 * endpoint: the inputs of handle `handle` for frames acked[s]+1 .. newest[s]
 * (first_frame .. newest[s] before any ack: the sender's input delay) from
 * inputs[frame][num_players][num_sessions], encoded against the input of frame
 * acked[s] (zeroed when acked[s] = RB_NULL_FRAME).  Writes the packet, its
 * length (0: nothing pending, -1: larger than packet_stride) and start frame. */
rb_status rb_encode_input_packets(int32_t device, void* stream, int32_t handle, int32_t num_players,
                                  int32_t num_sessions, int32_t input_bytes, const void* inputs, int32_t frames,
                                  int32_t first_frame, const int32_t* acked, const int32_t* newest, uint8_t* packets,
                                  int64_t packet_stride, int32_t* lengths, int32_t* start_frames);

#ifdef __cplusplus
} /* extern "C" */
#endif
#endif /* GGRS_AMD_H */
