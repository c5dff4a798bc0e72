// ============================================================================
// oracle/ggrs_oracle.hpp — TEST INFRASTRUCTURE ONLY (the parity checker).
//
// CPU restatement of the GGRS 0.9.4 rollback-resimulation path
// (/root/reference, Rust).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this code; the product (ggrs_amd/, libggrs_amd.so)
// never links or calls it.
//
// Every type and function cites the reference file:line it restates.  The
// reference cannot be compiled here (no cargo/rustc, crates not vendored), so
// this restatement is pinned by:
//   * the reference's own known-answer tests, restated in oracle/ref_tests.cpp
//     (tests/test_synctest_session.rs, tests/test_synctest_session_enum.rs,
//      src/input_queue.rs:269-326, src/sync_layer.rs:301-343,
//      src/frame_info.rs:83-102);
//   * published vectors for the third-party arithmetic on the path:
//     fletcher16 (the Wikipedia vectors the example cites at ex_game.rs:41),
//     SipHash (paper vector, + CPython's siphash24 with a zero key) for Rust's
//     std DefaultHasher = SipHash-1-3 with keys (0,0) used by tests/stubs.rs:8-12;
//   * glibc libm sinf/cosf/fmodf are called directly (Rust's f32::sin/cos/%
//     lower to the same libm symbols on x86_64 Linux).
// Numeric state/checksum values of ex_game are not pinned by any reference
// test: for those the oracle is "parity unpinned" beyond the
// restatement itself; see DESIGN.md §Oracle.
//
// Allocation pattern is kept on purpose (heap State with 3 vectors cloned on
// save/load, mutex-guarded shared cells, hash-map checksum history with retain,
// bincode image in a fresh vector on every save AND advance) so the same code
// is the "port" CPU baseline of bench.py.
// ============================================================================
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace orc {

using Frame = int32_t;            // lib.rs:48
constexpr Frame NULL_FRAME = -1;  // lib.rs:46
using PlayerHandle = size_t;      // lib.rs:50
using u128 = unsigned __int128;

// Rust panic!/assert! -> C++ exception, so restated #[should_panic] tests can
// observe them.
struct Panic : std::logic_error {
  using std::logic_error::logic_error;
};
#define ORC_ASSERT(c)                                                          \
  do {                                                                         \
    if (!(c))                                                                  \
      throw ::orc::Panic(std::string("assertion failed: " #c " @ ") +         \
                         __FILE__ + ":" + std::to_string(__LINE__));           \
  } while (0)

// lib.rs:104-112
enum class InputStatus : int32_t { Confirmed = 0, Predicted = 1, Disconnected = 2 };

// error.rs:11-36 (deprecated variants omitted: never produced on this path)
enum class ErrorKind : int32_t {
  Ok = 0,
  PredictionThreshold = 1,
  InvalidRequest = 2,
  MismatchedChecksum = 3,
  NotSynchronized = 4,
  SpectatorTooFarBehind = 5,
};
struct Error {
  ErrorKind kind = ErrorKind::Ok;
  Frame frame = NULL_FRAME;  // MismatchedChecksum{frame}
  std::string info;          // InvalidRequest{info}
  bool is_err() const { return kind != ErrorKind::Ok; }
  static Error ok() { return {}; }
  static Error invalid(std::string i) { return {ErrorKind::InvalidRequest, NULL_FRAME, std::move(i)}; }
};

// ---------------------------------------------------------------------------
// frame_info.rs:27-66  PlayerInput<I>
// ---------------------------------------------------------------------------
template <class I>
struct PlayerInput {
  Frame frame = NULL_FRAME;
  I input{};
  PlayerInput() = default;
  PlayerInput(Frame f, I i) : frame(f), input(i) {}                    // :52-54
  static PlayerInput blank_input(Frame f) { return PlayerInput(f, I{}); }  // :56-61 (zeroed)
  bool equal(const PlayerInput& o, bool input_only) const {            // :63-65
    return (input_only || frame == o.frame) && std::memcmp(&input, &o.input, sizeof(I)) == 0;
  }
};

// frame_info.rs:5-23  GameState<S>
template <class S>
struct GameState {
  Frame frame = NULL_FRAME;
  std::optional<S> data;
  std::optional<u128> checksum;
};

// sync_layer.rs:15-52  GameStateCell = Arc<Mutex<GameState<T>>>
template <class S>
class GameStateCell {
  struct Inner {
    std::mutex m;
    GameState<S> st;
  };
  std::shared_ptr<Inner> p_ = std::make_shared<Inner>();

 public:
  void save(Frame frame, std::optional<S> data, std::optional<u128> checksum) {  // :19-25
    std::lock_guard<std::mutex> g(p_->m);
    ORC_ASSERT(frame != NULL_FRAME);
    p_->st.frame = frame;
    p_->st.data = std::move(data);
    p_->st.checksum = checksum;
  }
  std::optional<S> load() const {  // :28-31 (clone out of the cell)
    std::lock_guard<std::mutex> g(p_->m);
    return p_->st.data;
  }
  Frame frame() const {  // :33-35
    std::lock_guard<std::mutex> g(p_->m);
    return p_->st.frame;
  }
  std::optional<u128> checksum() const {  // :37-39
    std::lock_guard<std::mutex> g(p_->m);
    return p_->st.checksum;
  }
};

// sync_layer.rs:54-76  SavedStates — exactly max_pred cells (the "+2" comment
// at :61-62 only affects Vec capacity).
template <class S>
struct SavedStates {
  std::vector<GameStateCell<S>> states;
  explicit SavedStates(size_t max_pred) {
    states.reserve(max_pred + 2);
    for (size_t i = 0; i < max_pred; ++i) states.emplace_back();
  }
  GameStateCell<S> get_cell(Frame frame) const {  // :71-75
    ORC_ASSERT(frame >= 0);
    return states[static_cast<size_t>(frame) % states.size()];
  }
};

// messages.rs:5-18
struct ConnectionStatus {
  bool disconnected = false;
  Frame last_frame = NULL_FRAME;
};

// lib.rs:170-194  GGRSRequest
enum class RequestKind : int32_t { Save = 0, Load = 1, Advance = 2 };
template <class C>
struct Request {
  RequestKind kind;
  GameStateCell<typename C::State> cell;  // Save/Load
  Frame frame = NULL_FRAME;               // Save/Load; for Advance: frame advanced FROM (trace only)
  std::vector<std::pair<typename C::Input, InputStatus>> inputs;  // Advance
};

// ---------------------------------------------------------------------------
// input_queue.rs  InputQueue<T>
// ---------------------------------------------------------------------------
constexpr size_t INPUT_QUEUE_LENGTH = 128;  // input_queue.rs:6

template <class I>
class InputQueue {
 public:
  // fields: input_queue.rs:10-37 (public for the restated white-box tests)
  size_t head = 0, tail = 0, length = 0;
  bool first_frame = true;
  Frame last_added_frame = NULL_FRAME;
  Frame first_incorrect_frame_ = NULL_FRAME;
  Frame last_requested_frame = NULL_FRAME;
  size_t frame_delay = 0;
  std::vector<PlayerInput<I>> inputs;
  PlayerInput<I> prediction;

  InputQueue()  // :40-53
      : prediction(PlayerInput<I>::blank_input(NULL_FRAME)) {
    inputs.assign(INPUT_QUEUE_LENGTH, PlayerInput<I>::blank_input(NULL_FRAME));
  }

  Frame first_incorrect_frame() const { return first_incorrect_frame_; }  // :55-57
  void set_frame_delay(size_t d) { frame_delay = d; }                     // :59-61

  void reset_prediction() {  // :63-67
    prediction.frame = NULL_FRAME;
    first_incorrect_frame_ = NULL_FRAME;
    last_requested_frame = NULL_FRAME;
  }

  PlayerInput<I> confirmed_input(Frame requested) const {  // :71-80
    size_t offset = static_cast<size_t>(requested) % INPUT_QUEUE_LENGTH;
    if (inputs[offset].frame == requested) return inputs[offset];
    throw Panic("SyncLayer::confirmed_input(): There is no confirmed input for the requested frame");
  }

  void discard_confirmed_frames(Frame frame) {  // :83-101
    if (last_requested_frame != NULL_FRAME) frame = std::min(frame, last_requested_frame);
    if (frame >= last_added_frame) {
      tail = head;
      length = 1;
    } else if (frame <= inputs[tail].frame) {
      // nothing to delete
    } else {
      size_t offset = static_cast<size_t>(frame - inputs[tail].frame);
      // `self.length -= offset` (:99) is checked arithmetic in the reference's test builds
      ORC_ASSERT(offset <= length);
      tail = (tail + offset) % INPUT_QUEUE_LENGTH;
      length -= offset;
    }
  }

  std::pair<I, InputStatus> input(Frame requested) {  // :104-146
    ORC_ASSERT(first_incorrect_frame_ == NULL_FRAME);
    last_requested_frame = requested;
    ORC_ASSERT(requested >= inputs[tail].frame);
    if (prediction.frame < 0) {
      size_t offset = static_cast<size_t>(requested - inputs[tail].frame);
      if (offset < length) {
        offset = (offset + tail) % INPUT_QUEUE_LENGTH;
        ORC_ASSERT(inputs[offset].frame == requested);
        return {inputs[offset].input, InputStatus::Confirmed};
      }
      if (requested == 0 || last_added_frame == NULL_FRAME) {
        prediction = PlayerInput<I>::blank_input(prediction.frame);
      } else {
        size_t prev = head == 0 ? INPUT_QUEUE_LENGTH - 1 : head - 1;
        prediction = inputs[prev];
      }
      prediction.frame += 1;
    }
    ORC_ASSERT(prediction.frame != NULL_FRAME);
    return {prediction.input, InputStatus::Predicted};
  }

  Frame add_input(PlayerInput<I> in) {  // :149-163
    ORC_ASSERT(last_added_frame == NULL_FRAME ||
               in.frame + static_cast<Frame>(frame_delay) == last_added_frame + 1);
    Frame new_frame = advance_queue_head(in.frame);
    if (new_frame != NULL_FRAME) add_input_by_frame(in, new_frame);
    return new_frame;
  }

 private:
  void add_input_by_frame(PlayerInput<I> in, Frame frame_number) {  // :167-204
    size_t prev = head == 0 ? INPUT_QUEUE_LENGTH - 1 : head - 1;
    ORC_ASSERT(last_added_frame == NULL_FRAME || frame_number == last_added_frame + 1);
    ORC_ASSERT(frame_number == 0 || inputs[prev].frame == frame_number - 1);
    inputs[head] = in;
    inputs[head].frame = frame_number;
    head = (head + 1) % INPUT_QUEUE_LENGTH;
    length += 1;
    ORC_ASSERT(length <= INPUT_QUEUE_LENGTH);
    first_frame = false;
    last_added_frame = frame_number;
    if (prediction.frame != NULL_FRAME) {
      ORC_ASSERT(frame_number == prediction.frame);
      if (first_incorrect_frame_ == NULL_FRAME && !prediction.equal(in, true))
        first_incorrect_frame_ = frame_number;
      if (prediction.frame == last_requested_frame && first_incorrect_frame_ == NULL_FRAME)
        prediction.frame = NULL_FRAME;
      else
        prediction.frame += 1;
    }
  }

  Frame advance_queue_head(Frame input_frame) {  // :207-239
    size_t prev = head == 0 ? INPUT_QUEUE_LENGTH - 1 : head - 1;
    Frame expected = first_frame ? 0 : inputs[prev].frame + 1;
    input_frame += static_cast<Frame>(frame_delay);
    if (expected > input_frame) return NULL_FRAME;
    while (expected < input_frame) {
      PlayerInput<I> rep = inputs[prev];  // replicate the entry before head (blank at start)
      add_input_by_frame(rep, expected);
      expected += 1;
    }
    prev = head == 0 ? INPUT_QUEUE_LENGTH - 1 : head - 1;
    ORC_ASSERT(input_frame == 0 || input_frame == inputs[prev].frame + 1);
    return input_frame;
  }
};

// ---------------------------------------------------------------------------
// sync_layer.rs:78-274  SyncLayer<T>
// ---------------------------------------------------------------------------
template <class C>
class SyncLayer {
 public:
  using I = typename C::Input;
  using S = typename C::State;
  size_t num_players, max_prediction;
  SavedStates<S> saved_states;
  Frame last_confirmed_frame = NULL_FRAME, last_saved_frame = NULL_FRAME, current_frame_ = 0;
  std::vector<InputQueue<I>> input_queues;

  SyncLayer(size_t np, size_t mp)  // :93-108
      : num_players(np), max_prediction(mp), saved_states(mp), input_queues(np) {}

  Frame current_frame() const { return current_frame_; }  // :110-112
  void advance_frame() { current_frame_ += 1; }           // :114-116

  Request<C> save_current_state() {  // :118-125
    last_saved_frame = current_frame_;
    Request<C> r{RequestKind::Save, saved_states.get_cell(current_frame_), current_frame_, {}};
    return r;
  }

  void set_frame_delay(PlayerHandle h, size_t d) {  // :127-130
    ORC_ASSERT(h < num_players);
    input_queues[h].set_frame_delay(d);
  }

  void reset_prediction() {  // :132-136
    for (auto& q : input_queues) q.reset_prediction();
  }

  Request<C> load_frame(Frame f) {  // :139-155
    ORC_ASSERT(f != NULL_FRAME && f < current_frame_ &&
               f >= current_frame_ - static_cast<Frame>(max_prediction));
    auto cell = saved_states.get_cell(f);
    ORC_ASSERT(cell.frame() == f);
    current_frame_ = f;
    return Request<C>{RequestKind::Load, cell, f, {}};
  }

  // :159-174
  Error add_local_input(PlayerHandle h, PlayerInput<I> in, Frame* out_frame) {
    Frame frames_ahead = current_frame_ - last_confirmed_frame;
    if (current_frame_ >= static_cast<Frame>(max_prediction) &&
        frames_ahead >= static_cast<Frame>(max_prediction))
      return Error{ErrorKind::PredictionThreshold, NULL_FRAME, ""};
    ORC_ASSERT(in.frame == current_frame_);
    Frame f = input_queues[h].add_input(in);
    if (out_frame) *out_frame = f;
    return Error::ok();
  }

  void add_remote_input(PlayerHandle h, PlayerInput<I> in) {  // :178-184
    input_queues[h].add_input(in);
  }

  std::vector<std::pair<I, InputStatus>> synchronized_inputs(  // :187-200
      const std::vector<ConnectionStatus>& cs) {
    std::vector<std::pair<I, InputStatus>> out;
    for (size_t i = 0; i < cs.size(); ++i) {
      if (cs[i].disconnected && cs[i].last_frame < current_frame_)
        out.push_back({I{}, InputStatus::Disconnected});
      else
        out.push_back(input_queues[i].input(current_frame_));
    }
    return out;
  }

  void set_last_confirmed_frame(Frame frame, bool sparse_saving) {  // :220-244
    Frame first_incorrect = NULL_FRAME;
    for (size_t h = 0; h < num_players; ++h)
      first_incorrect = std::max(first_incorrect, input_queues[h].first_incorrect_frame());
    if (sparse_saving) frame = std::min(frame, last_saved_frame);
    ORC_ASSERT(first_incorrect == NULL_FRAME || first_incorrect >= frame);
    last_confirmed_frame = frame;
    if (last_confirmed_frame > 0)
      for (size_t i = 0; i < num_players; ++i) input_queues[i].discard_confirmed_frames(frame - 1);
  }

  Frame check_simulation_consistency(Frame first_incorrect) const {  // :247-257
    for (size_t h = 0; h < num_players; ++h) {
      Frame inc = input_queues[h].first_incorrect_frame();
      if (inc != NULL_FRAME && (first_incorrect == NULL_FRAME || inc < first_incorrect))
        first_incorrect = inc;
    }
    return first_incorrect;
  }

  std::optional<GameStateCell<S>> saved_state_by_frame(Frame f) const {  // :260-268
    auto cell = saved_states.get_cell(f);
    if (cell.frame() == f) return cell;
    return std::nullopt;
  }
};

// ---------------------------------------------------------------------------
// sessions/sync_test_session.rs  SyncTestSession<T>
// ---------------------------------------------------------------------------
template <class C>
class SyncTestSession {
 public:
  using I = typename C::Input;
  size_t num_players_, max_prediction_, check_distance;
  SyncLayer<C> sync_layer;
  std::vector<ConnectionStatus> dummy_connect_status;
  std::unordered_map<Frame, std::optional<u128>> checksum_history;
  std::map<PlayerHandle, PlayerInput<I>> local_inputs;  // HashMap; iteration order is irrelevant here

  SyncTestSession(size_t np, size_t mp, size_t cd, size_t delay)  // :25-50
      : num_players_(np), max_prediction_(mp), check_distance(cd), sync_layer(np, mp),
        dummy_connect_status(np) {
    for (size_t i = 0; i < np; ++i) sync_layer.set_frame_delay(i, delay);
  }

  Error add_local_input(PlayerHandle h, I input) {  // :61-74
    if (h >= num_players_) return Error::invalid("The player handle you provided is not valid.");
    local_inputs[h] = PlayerInput<I>(sync_layer.current_frame(), input);
    return Error::ok();
  }

  Error advance_frame(std::vector<Request<C>>& requests) {  // :85-146
    requests.clear();
    if (check_distance > 0 && sync_layer.current_frame() > static_cast<Frame>(check_distance)) {
      for (Frame i = 0; i <= static_cast<Frame>(check_distance); ++i) {
        Frame f = sync_layer.current_frame() - i;
        if (!checksums_consistent(f)) return Error{ErrorKind::MismatchedChecksum, f, ""};
      }
      Frame frame_to = sync_layer.current_frame() - static_cast<Frame>(check_distance);
      adjust_gamestate(frame_to, requests);
    }
    if (num_players_ != local_inputs.size())
      return Error::invalid("Missing local input while calling advance_frame().");
    for (auto& kv : local_inputs) {
      Error e = sync_layer.add_local_input(kv.first, kv.second, nullptr);
      if (e.is_err()) return e;
    }
    local_inputs.clear();
    if (check_distance > 0) requests.push_back(sync_layer.save_current_state());
    Request<C> adv{RequestKind::Advance, {}, sync_layer.current_frame(),
                   sync_layer.synchronized_inputs(dummy_connect_status)};
    requests.push_back(std::move(adv));
    sync_layer.advance_frame();
    Frame safe_frame = sync_layer.current_frame() - static_cast<Frame>(check_distance);
    sync_layer.set_last_confirmed_frame(safe_frame, false);
    for (auto& c : dummy_connect_status) c.last_frame = sync_layer.current_frame();
    return Error::ok();
  }

  size_t num_players() const { return num_players_; }
  size_t max_prediction() const { return max_prediction_; }
  Frame current_frame() const { return sync_layer.current_frame(); }

 private:
  bool checksums_consistent(Frame f) {  // :159-176
    Frame oldest = sync_layer.current_frame() - static_cast<Frame>(check_distance);
    for (auto it = checksum_history.begin(); it != checksum_history.end();)
      it = it->first >= oldest ? std::next(it) : checksum_history.erase(it);
    auto cell = sync_layer.saved_state_by_frame(f);
    if (!cell) return true;
    auto found = checksum_history.find(cell->frame());
    if (found != checksum_history.end()) return found->second == cell->checksum();
    checksum_history.emplace(cell->frame(), cell->checksum());
    return true;
  }

  void adjust_gamestate(Frame frame_to, std::vector<Request<C>>& requests) {  // :178-203
    Frame start = sync_layer.current_frame();
    Frame count = start - frame_to;
    requests.push_back(sync_layer.load_frame(frame_to));
    sync_layer.reset_prediction();
    ORC_ASSERT(sync_layer.current_frame() == frame_to);
    for (Frame i = 0; i < count; ++i) {
      auto inputs = sync_layer.synchronized_inputs(dummy_connect_status);
      if (i > 0) requests.push_back(sync_layer.save_current_state());
      Frame from = sync_layer.current_frame();
      sync_layer.advance_frame();
      requests.push_back(Request<C>{RequestKind::Advance, {}, from, std::move(inputs)});
    }
    ORC_ASSERT(sync_layer.current_frame() == start);
  }
};

// ---------------------------------------------------------------------------
// sessions/p2p_session.rs  P2PSession<T> — the rollback path without the
// network layer.  UdpProtocol's job on this path is to turn packets into
// Event::Input{input, player} in frame order (handle_event, :838-852); here the
// caller delivers those inputs directly (deliver_remote_input), and likewise
// the peers' ChecksumReports (on_checksum_report) and connect-status reports
// (receive_peer_connect_status).  Spectators, time sync / wait
// recommendations and the synchronisation handshake (the session starts
// Running) are out of scope.  disconnect_player (a user call
// between advance_frames), desync detection and update_player_disconnects
// are modelled.
// ---------------------------------------------------------------------------
template <class C>
class P2PSession {
 public:
  using I = typename C::Input;
  size_t num_players, max_prediction;
  bool sparse_saving;
  SyncLayer<C> sync_layer;
  std::vector<ConnectionStatus> local_connect_status;
  std::vector<bool> is_local;
  Frame disconnect_frame = NULL_FRAME;
  std::map<PlayerHandle, PlayerInput<I>> local_inputs;

  // Desync detection (p2p_session.rs:154-157, 313-316, 873-928).
  // DesyncDetection::On{interval} with interval > 0; 0 = Off (builder.rs:15
  // DEFAULT_DETECTION_MODE).  Each remote handle is its own endpoint here, so
  // the UdpProtocol side of the exchange (protocol.rs:176-178, 710-742) is
  // one RemoteChecksums per remote handle.
  static constexpr size_t MAX_CHECKSUM_HISTORY_SIZE = 32;  // protocol.rs:27
  uint32_t desync_interval = 0;
  std::unordered_map<Frame, u128> local_checksum_history;  // :157
  struct RemoteChecksums {                                  // UdpProtocol::checksum_history et al.
    std::unordered_map<Frame, u128> checksum_history;       // protocol.rs:177
    Frame last_added_checksum_frame = NULL_FRAME;           // protocol.rs:178
  };
  std::vector<RemoteChecksums> remote_checksums;           // [num_players], remote handles only
  std::vector<std::pair<Frame, u128>> sent_reports;        // ChecksumReport messages sent, in order
  struct DesyncEvent {                                      // GGRSEvent::DesyncDetected (lib.rs:157-166)
    Frame frame;
    u128 local_checksum, remote_checksum;
    PlayerHandle handle;  // stands for `addr`: the remote endpoint
  };
  std::vector<DesyncEvent> events;
  // UdpProtocol::peer_connect_status of each remote handle's endpoint (protocol.rs:158-160):
  // what that peer last reported about every player's connection
  std::vector<std::vector<ConnectionStatus>> peer_connect_status;

  // :160-213 (local players get the input delay; remote queues have none)
  P2PSession(size_t np, size_t mp, bool sparse, size_t delay, std::vector<bool> local)
      : num_players(np), max_prediction(mp), sparse_saving(sparse), sync_layer(np, mp),
        local_connect_status(np), is_local(std::move(local)), remote_checksums(np),
        peer_connect_status(np, std::vector<ConnectionStatus>(np)) {
    for (size_t h = 0; h < np; ++h)
      if (is_local[h]) sync_layer.set_frame_delay(h, delay);
  }

  // UdpProtocol::on_checksum_report (protocol.rs:710-722) of remote handle h's
  // endpoint: a ChecksumReport{checksum, frame} arrived from that peer.
  void on_checksum_report(PlayerHandle h, Frame frame, u128 checksum) {
    ORC_ASSERT(h < num_players && !is_local[h]);
    auto& r = remote_checksums[h];
    if (r.last_added_checksum_frame < frame) {
      if (r.checksum_history.size() > MAX_CHECKSUM_HISTORY_SIZE) {
        const Frame keep_after = r.last_added_checksum_frame - static_cast<Frame>(MAX_CHECKSUM_HISTORY_SIZE);
        for (auto it = r.checksum_history.begin(); it != r.checksum_history.end();)
          it = it->first > keep_after ? std::next(it) : r.checksum_history.erase(it);
      }
      r.last_added_checksum_frame = frame;
      r.checksum_history[frame] = checksum;
    }
  }

  Error add_local_input(PlayerHandle h, I input) {  // :223-240
    if (h >= num_players || !is_local[h])
      return Error::invalid("The player handle you provided is not referring to a local player.");
    local_inputs[h] = PlayerInput<I>(sync_layer.current_frame(), input);
    return Error::ok();
  }

  // handle_event(Event::Input{input, player}) (:838-852)
  void deliver_remote_input(PlayerHandle player, PlayerInput<I> input) {
    ORC_ASSERT(player < num_players);
    if (!local_connect_status[player].disconnected) {
      Frame cur = local_connect_status[player].last_frame;
      ORC_ASSERT(cur == NULL_FRAME || cur + 1 == input.frame);
      local_connect_status[player].last_frame = input.frame;
      sync_layer.add_remote_input(player, input);
    }
  }

  // :430-456 disconnect_player + :555-581 disconnect_player_at_frame (a remote
  // handle maps to its own endpoint: one handle per address in the batch)
  Error disconnect_player(PlayerHandle h) {
    if (h >= num_players) return Error::invalid("Invalid Player Handle.");
    if (is_local[h]) return Error::invalid("Local Player cannot be disconnected.");
    if (local_connect_status[h].disconnected) return Error::invalid("Player already disconnected.");
    disconnect_player_at_frame(h, local_connect_status[h].last_frame);
    return Error::ok();
  }

  // :555-595 disconnect_player_at_frame.  Each remote handle is its own
  // endpoint here, so endpoint.disconnect() (the endpoint stops Running) is
  // the handle's disconnected flag; a local handle is a no-op (:590).
  void disconnect_player_at_frame(PlayerHandle h, Frame last_frame) {
    if (is_local[h]) return;
    local_connect_status[h].disconnected = true;
    if (sync_layer.current_frame() > last_frame) disconnect_frame = last_frame + 1;
  }

  // UdpProtocol::on_input's merge of the peer's connect status (protocol.rs:627-636):
  // the endpoint of remote handle `endpoint` reports player i as (disconnected, last_frame)
  void receive_peer_connect_status(PlayerHandle endpoint, PlayerHandle i, bool disconnected, Frame last_frame) {
    ORC_ASSERT(endpoint < num_players && !is_local[endpoint] && i < num_players);
    auto& c = peer_connect_status[endpoint][i];
    c.disconnected = disconnected || c.disconnected;
    c.last_frame = std::max(c.last_frame, last_frame);
  }

  Frame confirmed_frame() const {  // :487-498
    Frame cf = INT32_MAX;
    for (auto& c : local_connect_status)
      if (!c.disconnected) cf = std::min(cf, c.last_frame);
    ORC_ASSERT(cf < INT32_MAX);
    return cf;
  }
  Frame current_frame() const { return sync_layer.current_frame(); }

  // :253-337 (poll_remote_clients = the deliveries made before this call)
  Error advance_frame(std::vector<Request<C>>& requests) {
    requests.clear();
    if (sync_layer.current_frame() == 0) requests.push_back(sync_layer.save_current_state());
    update_player_disconnects();  // :274-275
    Frame confirmed = confirmed_frame();
    Frame first_incorrect = sync_layer.check_simulation_consistency(disconnect_frame);
    if (first_incorrect != NULL_FRAME) {
      adjust_gamestate(first_incorrect, confirmed, requests);
      disconnect_frame = NULL_FRAME;
    }
    Frame last_saved = sync_layer.last_saved_frame;
    if (sparse_saving)
      check_last_saved_state(last_saved, confirmed, requests);
    else
      requests.push_back(sync_layer.save_current_state());
    sync_layer.set_last_confirmed_frame(confirmed, sparse_saving);
    if (desync_interval) {  // :313-316
      check_checksum_send_interval();
      compare_local_checksums_against_peers();
    }
    for (size_t h = 0; h < num_players; ++h) {  // local_player_handles()
      if (!is_local[h]) continue;
      auto it = local_inputs.find(h);
      if (it == local_inputs.end()) return Error::invalid("Missing local input while calling advance_frame().");
      Frame actual = NULL_FRAME;
      Error e = sync_layer.add_local_input(h, it->second, &actual);
      if (e.is_err()) return e;
      ORC_ASSERT(actual != NULL_FRAME);
      it->second.frame = actual;
      local_connect_status[h].last_frame = actual;
    }
    local_inputs.clear();
    auto inputs = sync_layer.synchronized_inputs(local_connect_status);
    Frame from = sync_layer.current_frame();
    sync_layer.advance_frame();
    requests.push_back(Request<C>{RequestKind::Advance, {}, from, std::move(inputs)});
    return Error::ok();
  }

 private:
  // :707-742.  An endpoint is Running until it is disconnected (the batch has
  // no synchronising or timed-out endpoints: the session starts Running).
  void update_player_disconnects() {
    for (size_t handle = 0; handle < num_players; ++handle) {
      bool queue_connected = true;
      Frame queue_min_confirmed = INT32_MAX;
      for (size_t e = 0; e < num_players; ++e) {  // player_reg.remotes.values()
        if (is_local[e] || local_connect_status[e].disconnected) continue;  // !endpoint.is_running()
        const ConnectionStatus& con = peer_connect_status[e][handle];
        queue_connected = queue_connected && !con.disconnected;
        queue_min_confirmed = std::min(queue_min_confirmed, con.last_frame);
      }
      const bool local_connected = !local_connect_status[handle].disconnected;
      const Frame local_min_confirmed = local_connect_status[handle].last_frame;
      if (local_connected) queue_min_confirmed = std::min(queue_min_confirmed, local_min_confirmed);
      if (!queue_connected && (local_connected || local_min_confirmed > queue_min_confirmed))
        disconnect_player_at_frame(handle, queue_min_confirmed);
    }
  }

  // :900-928.  The report is "sent" to every remote endpoint (sent_reports;
  // the caller forwards it to the peers' on_checksum_report).
  void check_checksum_send_interval() {
    const Frame frame_to_send = sync_layer.last_saved_frame - 1;
    const Frame current = current_frame();
    if (current % static_cast<Frame>(desync_interval) == 0 && frame_to_send > static_cast<Frame>(max_prediction)) {
      auto cell = sync_layer.saved_state_by_frame(frame_to_send);
      if (!cell) throw Panic("cell not found!: frame " + std::to_string(frame_to_send));
      if (auto checksum = cell->checksum()) {
        sent_reports.push_back({frame_to_send, *checksum});
        local_checksum_history[frame_to_send] = *checksum;
      }
    }
    if (local_checksum_history.size() > MAX_CHECKSUM_HISTORY_SIZE) {
      const Frame keep_after = current - static_cast<Frame>(MAX_CHECKSUM_HISTORY_SIZE);
      for (auto it = local_checksum_history.begin(); it != local_checksum_history.end();)
        it = it->first > keep_after ? std::next(it) : local_checksum_history.erase(it);
    }
  }
  // :873-898.  The reference walks HashMaps (unspecified order); here the
  // remote handles ascend and each endpoint's history is walked by frame.
  void compare_local_checksums_against_peers() {
    if (current_frame() % static_cast<Frame>(desync_interval) != 0) return;
    for (size_t h = 0; h < num_players; ++h) {
      if (is_local[h]) continue;
      std::map<Frame, u128> ordered(remote_checksums[h].checksum_history.begin(),
                                    remote_checksums[h].checksum_history.end());
      for (auto& [remote_frame, remote_checksum] : ordered) {
        auto it = local_checksum_history.find(remote_frame);
        if (it != local_checksum_history.end() && it->second != remote_checksum)
          events.push_back({remote_frame, it->second, remote_checksum, h});
      }
    }
  }

  void adjust_gamestate(Frame first_incorrect, Frame min_confirmed, std::vector<Request<C>>& requests) {  // :621-673
    Frame current = sync_layer.current_frame();
    Frame frame_to_load = sparse_saving ? sync_layer.last_saved_frame : first_incorrect;
    ORC_ASSERT(frame_to_load <= first_incorrect);
    Frame count = current - frame_to_load;
    requests.push_back(sync_layer.load_frame(frame_to_load));
    ORC_ASSERT(sync_layer.current_frame() == frame_to_load);
    sync_layer.reset_prediction();
    for (Frame i = 0; i < count; ++i) {
      auto inputs = sync_layer.synchronized_inputs(local_connect_status);
      if (sparse_saving) {
        if (sync_layer.current_frame() == min_confirmed) requests.push_back(sync_layer.save_current_state());
      } else if (i > 0) {
        requests.push_back(sync_layer.save_current_state());
      }
      Frame from = sync_layer.current_frame();
      sync_layer.advance_frame();
      requests.push_back(Request<C>{RequestKind::Advance, {}, from, std::move(inputs)});
    }
    ORC_ASSERT(sync_layer.current_frame() == current);
  }

  void check_last_saved_state(Frame last_saved, Frame confirmed, std::vector<Request<C>>& requests) {  // :778-802
    if (sync_layer.current_frame() - last_saved >= static_cast<Frame>(max_prediction)) {
      if (confirmed >= sync_layer.current_frame())
        requests.push_back(sync_layer.save_current_state());
      else
        adjust_gamestate(last_saved, confirmed, requests);
      ORC_ASSERT(confirmed == NULL_FRAME ||
                 sync_layer.last_saved_frame == std::min(confirmed, sync_layer.current_frame()));
    }
  }
};

// builder.rs:13-27, 136-157, 202-205, 342-354 — the SyncTest subset
struct SessionBuilder {
  size_t num_players = 2;        // DEFAULT_PLAYERS
  size_t max_prediction = 8;     // DEFAULT_MAX_PREDICTION_FRAMES
  size_t input_delay = 0;        // DEFAULT_INPUT_DELAY
  size_t check_dist = 2;         // DEFAULT_CHECK_DISTANCE
  Error with_max_prediction_window(size_t w) {
    if (w == 0) return Error::invalid("Currently, only prediction windows above 0 are supported");
    max_prediction = w;
    return Error::ok();
  }
  SessionBuilder& with_input_delay(size_t d) { input_delay = d; return *this; }
  SessionBuilder& with_num_players(size_t n) { num_players = n; return *this; }
  SessionBuilder& with_check_distance(size_t c) { check_dist = c; return *this; }
  template <class C>
  Error start_synctest_session(std::unique_ptr<SyncTestSession<C>>* out) const {
    if (check_dist >= max_prediction) return Error::invalid("Check distance too big.");
    out->reset(new SyncTestSession<C>(num_players, max_prediction, check_dist, input_delay));
    return Error::ok();
  }
};

// ===========================================================================
// Third-party arithmetic on the path
// ===========================================================================

// ex_game.rs:42-52 — fletcher16 (serial, mod 255)
inline uint16_t fletcher16(const uint8_t* data, size_t n) {
  uint16_t sum1 = 0, sum2 = 0;
  for (size_t i = 0; i < n; ++i) {
    sum1 = static_cast<uint16_t>((sum1 + data[i]) % 255);
    sum2 = static_cast<uint16_t>((sum2 + sum1) % 255);
  }
  return static_cast<uint16_t>((sum2 << 8) | sum1);
}

// SipHash-c-d (Aumasson & Bernstein 2012).  Rust std DefaultHasher::new() is
// SipHasher13 with keys (0,0); Hasher::write_i32 feeds i32::to_ne_bytes (LE).
inline uint64_t siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1, const uint8_t* m, size_t len) {
  auto rotl = [](uint64_t x, int b) { return (x << b) | (x >> (64 - b)); };
  uint64_t v0 = 0x736f6d6570736575ULL ^ k0, v1 = 0x646f72616e646f6dULL ^ k1;
  uint64_t v2 = 0x6c7967656e657261ULL ^ k0, v3 = 0x7465646279746573ULL ^ k1;
  auto round = [&]() {
    v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);
    v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;
    v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;
    v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);
  };
  size_t full = len & ~size_t(7);
  for (size_t i = 0; i < full; i += 8) {
    uint64_t w;
    std::memcpy(&w, m + i, 8);
    v3 ^= w;
    for (int r = 0; r < c_rounds; ++r) round();
    v0 ^= w;
  }
  uint64_t b = static_cast<uint64_t>(len & 0xff) << 56;
  for (size_t i = full; i < len; ++i) b |= static_cast<uint64_t>(m[i]) << (8 * (i - full));
  v3 ^= b;
  for (int r = 0; r < c_rounds; ++r) round();
  v0 ^= b;
  v2 ^= 0xff;
  for (int r = 0; r < d_rounds; ++r) round();
  return v0 ^ v1 ^ v2 ^ v3;
}
inline uint64_t default_hasher_i32_pair(int32_t a, int32_t b) {  // stubs.rs:8-12 on #[derive(Hash)] {i32,i32}
  uint8_t buf[8];
  std::memcpy(buf, &a, 4);
  std::memcpy(buf + 4, &b, 4);
  return siphash(1, 3, 0, 0, buf, 8);
}

// ===========================================================================
// examples/ex_game/ex_game.rs — the reference game (request handler)
// ===========================================================================
namespace exgame {
constexpr uint64_t FPS = 60;                                   // :8
constexpr int32_t CHECKSUM_PERIOD = 100;                       // :9
constexpr float WINDOW_HEIGHT = 800.0f;                        // :13
constexpr float WINDOW_WIDTH = 600.0f;                         // :14
constexpr uint8_t INPUT_UP = 1 << 0, INPUT_DOWN = 1 << 1;      // :16-17
constexpr uint8_t INPUT_LEFT = 1 << 2, INPUT_RIGHT = 1 << 3;   // :18-19
const float MOVEMENT_SPEED = 15.0f / static_cast<float>(FPS);  // :21
const float ROTATION_SPEED = 2.5f / static_cast<float>(FPS);   // :22
constexpr float MAX_SPEED = 7.0f;                              // :23
constexpr float FRICTION = 0.98f;                              // :24
constexpr float PI = 3.14159265358979323846264338327950288f;   // std::f32::consts::PI

struct Input {  // :26-30
  uint8_t inp = 0;
};

// f32::rem_euclid: r = self % rhs; if r < 0 { r + rhs.abs() } else { r }
inline float rem_euclid(float x, float rhs) {
  float r = std::fmod(x, rhs);
  return r < 0.0f ? r + std::fabs(rhs) : r;
}

struct State {  // :224-231
  int32_t frame = 0;
  uint64_t num_players = 0;  // usize
  std::vector<std::pair<float, float>> positions, velocities;
  std::vector<float> rotations;

  static State make(size_t n) {  // :234-257
    State s;
    float r = WINDOW_WIDTH / 4.0f;
    for (int32_t i = 0; i < static_cast<int32_t>(n); ++i) {
      float rot = static_cast<float>(i) / static_cast<float>(n) * 2.0f * PI;
      float x = WINDOW_WIDTH / 2.0f + r * std::cos(rot);
      float y = WINDOW_HEIGHT / 2.0f + r * std::sin(rot);
      s.positions.push_back({x, y});
      s.velocities.push_back({0.0f, 0.0f});
      s.rotations.push_back(std::fmod(rot + PI, 2.0f * PI));
    }
    s.frame = 0;
    s.num_players = n;
    return s;
  }

  void advance(const std::vector<std::pair<Input, InputStatus>>& inputs) {  // :259-321
    frame += 1;
    for (size_t i = 0; i < num_players; ++i) {
      uint8_t input = inputs[i].second == InputStatus::Disconnected ? 4 : inputs[i].first.inp;
      float old_x = positions[i].first, old_y = positions[i].second;
      float old_vx = velocities[i].first, old_vy = velocities[i].second;
      float rot = rotations[i];
      float vel_x = old_vx * FRICTION;
      float vel_y = old_vy * FRICTION;
      if ((input & INPUT_UP) != 0 && (input & INPUT_DOWN) == 0) {
        vel_x += MOVEMENT_SPEED * std::cos(rot);
        vel_y += MOVEMENT_SPEED * std::sin(rot);
      }
      if ((input & INPUT_UP) == 0 && (input & INPUT_DOWN) != 0) {
        vel_x -= MOVEMENT_SPEED * std::cos(rot);
        vel_y -= MOVEMENT_SPEED * std::sin(rot);
      }
      if ((input & INPUT_LEFT) != 0 && (input & INPUT_RIGHT) == 0)
        rot = rem_euclid(rot - ROTATION_SPEED, 2.0f * PI);
      if ((input & INPUT_LEFT) == 0 && (input & INPUT_RIGHT) != 0)
        rot = rem_euclid(rot + ROTATION_SPEED, 2.0f * PI);
      float magnitude = std::sqrt(vel_x * vel_x + vel_y * vel_y);
      if (magnitude > MAX_SPEED) {
        vel_x = (vel_x * MAX_SPEED) / magnitude;
        vel_y = (vel_y * MAX_SPEED) / magnitude;
      }
      float x = old_x + vel_x;
      float y = old_y + vel_y;
      x = std::fmax(x, 0.0f);
      x = std::fmin(x, WINDOW_WIDTH);
      y = std::fmax(y, 0.0f);
      y = std::fmin(y, WINDOW_HEIGHT);
      positions[i] = {x, y};
      velocities[i] = {vel_x, vel_y};
      rotations[i] = rot;
    }
  }
};

// bincode 1.3 `serialize` (fixint, little endian, u64 lengths) of State — the
// byte image fletcher16 runs over at ex_game.rs:90 and :106.  36 + 20·P bytes.
inline std::vector<uint8_t> bincode_serialize(const State& s) {
  std::vector<uint8_t> out;
  auto put = [&out](const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    out.insert(out.end(), b, b + n);
  };
  auto put_u64 = [&put](uint64_t v) { put(&v, 8); };
  put(&s.frame, 4);
  put_u64(s.num_players);
  put_u64(s.positions.size());
  for (auto& p : s.positions) { put(&p.first, 4); put(&p.second, 4); }
  put_u64(s.velocities.size());
  for (auto& v : s.velocities) { put(&v.first, 4); put(&v.second, 4); }
  put_u64(s.rotations.size());
  for (auto& r : s.rotations) put(&r, 4);
  return out;
}

struct Config {
  using Input = exgame::Input;
  using State = exgame::State;
};

// ex_game.rs:55-221 Game (the request handler; rendering/keyboard omitted)
struct Game {
  size_t num_players;
  State game_state;
  std::pair<Frame, uint64_t> last_checksum{NULL_FRAME, 0};
  std::pair<Frame, uint64_t> periodic_checksum{NULL_FRAME, 0};

  explicit Game(size_t n) : num_players(n), game_state(State::make(n)) { ORC_ASSERT(n <= 4); }

  void handle_requests(std::vector<Request<Config>>& reqs) {  // :76-84
    for (auto& r : reqs) {
      switch (r.kind) {
        case RequestKind::Load: load_game_state(r.cell); break;
        case RequestKind::Save: save_game_state(r.cell, r.frame); break;
        case RequestKind::Advance: advance_frame(r.inputs); break;
      }
    }
  }
  void save_game_state(GameStateCell<State>& cell, Frame frame) {  // :88-93
    ORC_ASSERT(game_state.frame == frame);
    auto buffer = bincode_serialize(game_state);
    u128 checksum = fletcher16(buffer.data(), buffer.size());
    cell.save(frame, game_state, checksum);
  }
  void load_game_state(GameStateCell<State>& cell) {  // :96-98
    auto d = cell.load();
    if (!d) throw Panic("No data found.");
    game_state = *d;
  }
  void advance_frame(const std::vector<std::pair<Input, InputStatus>>& inputs) {  // :100-112
    game_state.advance(inputs);
    auto buffer = bincode_serialize(game_state);
    uint64_t checksum = fletcher16(buffer.data(), buffer.size());
    last_checksum = {game_state.frame, checksum};
    if (game_state.frame % CHECKSUM_PERIOD == 0) periodic_checksum = {game_state.frame, checksum};
  }
  void trigger_desync() { game_state.positions[0] = {0.0f, 0.0f}; }  // :211-215
};
}  // namespace exgame

// ===========================================================================
// tests/stubs.rs & tests/stubs_enum.rs — integer stub games
// ===========================================================================
namespace stub {
struct StubInput {  // stubs.rs:19-23
  uint32_t inp = 0;
};
struct StateStub {  // stubs.rs:108-126
  int32_t frame = 0;
  int32_t state = 0;
  void advance_frame(const std::vector<std::pair<StubInput, InputStatus>>& inputs) {
    uint32_t p0 = inputs[0].first.inp, p1 = inputs[1].first.inp;
    if ((p0 + p1) % 2 == 0) state += 2; else state -= 1;
    frame += 1;
  }
};
struct Config {
  using Input = StubInput;
  using State = StateStub;
};
inline uint64_t calculate_hash(const StateStub& s) { return default_hasher_i32_pair(s.frame, s.state); }

struct GameStub {  // stubs.rs:14-65
  StateStub gs;
  void handle_requests(std::vector<Request<Config>>& reqs) {
    for (auto& r : reqs) {
      switch (r.kind) {
        case RequestKind::Load: { auto d = r.cell.load(); if (!d) throw Panic("unwrap on None"); gs = *d; break; }
        case RequestKind::Save: {
          ORC_ASSERT(gs.frame == r.frame);
          r.cell.save(r.frame, gs, static_cast<u128>(calculate_hash(gs)));
          break;
        }
        case RequestKind::Advance: gs.advance_frame(r.inputs); break;
      }
    }
  }
};

// stubs.rs:67-106 — saves a random u128 checksum; rng is a seeded splitmix64
// stream instead of thread_rng (only "differs from the first-seen value" matters).
struct RandomChecksumGameStub {
  StateStub gs;
  uint64_t rng;
  explicit RandomChecksumGameStub(uint64_t seed) : rng(seed) {}
  uint64_t next() {
    uint64_t z = (rng += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  void handle_requests(std::vector<Request<Config>>& reqs) {
    for (auto& r : reqs) {
      switch (r.kind) {
        case RequestKind::Load: { auto d = r.cell.load(); if (!d) throw Panic("No data found."); gs = *d; break; }
        case RequestKind::Save: {
          ORC_ASSERT(gs.frame == r.frame);
          u128 cs = (static_cast<u128>(next()) << 64) | next();
          r.cell.save(r.frame, gs, cs);
          break;
        }
        case RequestKind::Advance: gs.advance_frame(r.inputs); break;
      }
    }
  }
};

// stubs_enum.rs:18-29 (EnumInput), 73-91 (StateStubEnum)
enum class EnumInput : uint8_t { Val1 = 0, Val2 = 1 };
struct StateStubEnum {
  int32_t frame = 0;
  int32_t state = 0;
  // stubs_enum.rs:80-90: `p0_inputs == p1_inputs` compares (EnumInput, InputStatus) tuples
  void advance_frame(const std::vector<std::pair<EnumInput, InputStatus>>& inputs) {
    if (inputs[0].first == inputs[1].first && inputs[0].second == inputs[1].second) state += 2; else state -= 1;
    frame += 1;
  }
};
struct EnumConfig {
  using Input = EnumInput;
  using State = StateStubEnum;
};
struct GameStubEnum {
  StateStubEnum gs;
  void handle_requests(std::vector<Request<EnumConfig>>& reqs) {
    for (auto& r : reqs) {
      switch (r.kind) {
        case RequestKind::Load: { auto d = r.cell.load(); if (!d) throw Panic("unwrap on None"); gs = *d; break; }
        case RequestKind::Save: {
          ORC_ASSERT(gs.frame == r.frame);
          r.cell.save(r.frame, gs, static_cast<u128>(default_hasher_i32_pair(gs.frame, gs.state)));
          break;
        }
        case RequestKind::Advance: gs.advance_frame(r.inputs); break;
      }
    }
  }
};
}  // namespace stub

// ===========================================================================
// BASELINE config 3: the fixed-point 256-entity brawler.  The reference has no
// such game: this is the build's own definition, written
// once here (sequential, entity-index order) and restated on the device
// (ggrs_amd/csrc/games.hpp Brawler, one wavefront per session).  Parity is
// between those two only; the request-stream semantics around it are the
// reference's.  Integer-only, so checksums are bit-exact by construction.
//
// Entity e (8 x i32 = 32 B): x, y (Q16.16, arena [0, 2^20)), vx, vy, hp,
// flags (players: cooldown | attacking << 8; AI: target player), rng
// (xorshift32 state), counter (players: damage taken; AI: frames alive).
// Entities 0..P-1 are the players.  Image = le32 frame || 256 x 8 x le32
// (8196 B); checksum = fletcher16 of the image (as ex_game.rs:90-91).
// ===========================================================================
namespace brawler {
constexpr int N = 256;
constexpr int32_t ARENA = 1 << 20;
constexpr int32_t PLAYER_ACC = 1 << 12, PLAYER_VMAX = 1 << 14;
constexpr int32_t AI_ACC = 1 << 10, AI_VMAX = 1 << 13;
constexpr int32_t CONTACT = 1 << 14;
constexpr int32_t ATTACK_CD = 8, AI_DAMAGE = 25, PLAYER_HP0 = 1000, AI_HP0 = 100;
constexpr uint64_t INIT_KEY = 0x627261776C6572ULL;  // "brawler"
constexpr uint8_t IN_UP = 1, IN_DOWN = 2, IN_LEFT = 4, IN_RIGHT = 8, IN_ATTACK = 16;
enum Word { X = 0, Y, VX, VY, HP, FLAGS, RNG, COUNTER };

struct Input {
  uint8_t inp = 0;
};

inline int32_t clamp(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }
inline int32_t sgn(int32_t v) { return (v > 0) - (v < 0); }
inline int32_t iabs(int32_t v) { return v < 0 ? -v : v; }

inline uint64_t mix64(uint64_t x) {  // splitmix64
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

struct State {
  int32_t frame = 0;
  int32_t num_players = 0;
  std::vector<int32_t> ent;  // [N][8], heap like ex_game's Vecs

  static State make(int32_t P) {
    State s;
    s.num_players = P;
    s.ent.assign(N * 8, 0);
    for (int e = 0; e < N; ++e) {
      const uint64_t h = mix64(INIT_KEY ^ static_cast<uint64_t>(e));
      int32_t* w = &s.ent[e * 8];
      w[X] = static_cast<int32_t>(h & (ARENA - 1));
      w[Y] = static_cast<int32_t>((h >> 20) & (ARENA - 1));
      w[HP] = e < P ? PLAYER_HP0 : AI_HP0;
      w[FLAGS] = e < P ? 0 : e % P;
      w[RNG] = static_cast<int32_t>(static_cast<uint32_t>(h >> 32) | 1u);
    }
    return s;
  }

  void advance(const std::vector<std::pair<Input, InputStatus>>& inputs) {
    frame += 1;
    const int P = num_players;
    // phase 1: players
    for (int e = 0; e < P; ++e) {
      int32_t* w = &ent[e * 8];
      const uint32_t in = inputs[e].second == InputStatus::Disconnected ? 0u : inputs[e].first.inp;
      const int32_t ax = static_cast<int32_t>((in >> 3) & 1) - static_cast<int32_t>((in >> 2) & 1);
      const int32_t ay = static_cast<int32_t>((in >> 1) & 1) - static_cast<int32_t>(in & 1);
      w[VX] = clamp(w[VX] - (w[VX] >> 3) + ax * PLAYER_ACC, -PLAYER_VMAX, PLAYER_VMAX);
      w[VY] = clamp(w[VY] - (w[VY] >> 3) + ay * PLAYER_ACC, -PLAYER_VMAX, PLAYER_VMAX);
      w[X] = clamp(w[X] + w[VX], 0, ARENA - 1);
      w[Y] = clamp(w[Y] + w[VY], 0, ARENA - 1);
      int32_t cd = w[FLAGS] & 0xFF, atk = 0;
      if ((in & IN_ATTACK) && cd == 0) {
        cd = ATTACK_CD;
        atk = 1;
      } else {
        cd = cd > 0 ? cd - 1 : 0;
      }
      w[FLAGS] = cd | (atk << 8);
    }
    // phase 2: AI entities chase their target player (new positions)
    int32_t hits[4] = {0, 0, 0, 0};
    for (int e = P; e < N; ++e) {
      int32_t* w = &ent[e * 8];
      if (w[HP] <= 0) continue;
      const int t = w[FLAGS];
      const int32_t* pw = &ent[t * 8];
      uint32_t r = static_cast<uint32_t>(w[RNG]);
      r ^= r << 13;
      r ^= r >> 17;
      r ^= r << 5;
      w[RNG] = static_cast<int32_t>(r);
      const int32_t jx = static_cast<int32_t>(r & 0xFF) - 128, jy = static_cast<int32_t>((r >> 8) & 0xFF) - 128;
      w[VX] = clamp(w[VX] - (w[VX] >> 2) + sgn(pw[X] - w[X]) * AI_ACC + jx, -AI_VMAX, AI_VMAX);
      w[VY] = clamp(w[VY] - (w[VY] >> 2) + sgn(pw[Y] - w[Y]) * AI_ACC + jy, -AI_VMAX, AI_VMAX);
      w[X] = clamp(w[X] + w[VX], 0, ARENA - 1);
      w[Y] = clamp(w[Y] + w[VY], 0, ARENA - 1);
      w[COUNTER] += 1;
      if (iabs(pw[X] - w[X]) + iabs(pw[Y] - w[Y]) < CONTACT) {
        if ((pw[FLAGS] >> 8) & 1) {
          w[HP] = std::max(w[HP] - AI_DAMAGE, 0);
        } else {
          hits[t] += 1;
        }
      }
    }
    // phase 3: damage to players
    for (int e = 0; e < P; ++e) {
      int32_t* w = &ent[e * 8];
      w[HP] = std::max(w[HP] - hits[e], 0);
      w[COUNTER] += hits[e];
    }
  }
};

inline std::vector<uint8_t> image(const State& s) {
  std::vector<uint8_t> out(4 + s.ent.size() * 4);
  std::memcpy(out.data(), &s.frame, 4);
  std::memcpy(out.data() + 4, s.ent.data(), s.ent.size() * 4);
  return out;
}

struct Config {
  using Input = brawler::Input;
  using State = brawler::State;
};

struct Game {
  State gs;
  explicit Game(int32_t P) : gs(State::make(P)) { ORC_ASSERT(P >= 1 && P <= 4); }
  void handle_requests(std::vector<Request<Config>>& reqs) {
    for (auto& r : reqs) {
      switch (r.kind) {
        case RequestKind::Load: { auto d = r.cell.load(); if (!d) throw Panic("No data found."); gs = *d; break; }
        case RequestKind::Save: {
          ORC_ASSERT(gs.frame == r.frame);
          auto buf = image(gs);
          r.cell.save(r.frame, gs, static_cast<u128>(fletcher16(buf.data(), buf.size())));
          break;
        }
        case RequestKind::Advance: gs.advance(r.inputs); break;
      }
    }
  }
};
}  // namespace brawler

// ===========================================================================
// Synthetic input generator — shared definition with
// ggrs_amd/synth.py (tests check they agree).
// ===========================================================================
inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}
// h = splitmix64(seed ^ (s·2^20 + p·2^16 + f)); a new value (bits 32..) with
// probability 1/8 (h & 7 == 0) or at f == 0, otherwise hold the previous one.
struct SynthInput {
  uint64_t seed;
  uint32_t mask;
  uint64_t hash(uint64_t s, uint64_t p, uint64_t f) const {
    return splitmix64(seed ^ ((s << 20) + (p << 16) + f));
  }
  uint32_t next(uint32_t prev, uint64_t s, uint64_t p, uint64_t f) const {
    uint64_t h = hash(s, p, f);
    if (f == 0 || (h & 7) == 0) return static_cast<uint32_t>(h >> 32) & mask;
    return prev;
  }
};

// ===========================================================================
// network/compression.rs (XOR delta + bitfield RLE) — the input wire format
// that UdpProtocol::on_input decodes (protocol.rs:616-689).
// bitfield-rle 0.2 (Cargo.toml:23) is not vendored: its published format is
// restated (a series of varint-headed sequences; odd header = compressed run
// `len << 2 | bit << 1 | 1` of 0x00 / 0xFF bytes, even header = `len << 1`
// followed by len literal bytes; varints are unsigned LEB128).  Decoding is
// defined by that format.  The encoder's choice of which runs to compress is
// the crate's own heuristic, not pinned by any reference test (the only one,
// compression.rs:81-90, is a round trip): here runs of >= 4 equal 0x00/0xFF
// bytes are compressed — parity unpinned for encoded bytes, pinned for decode
// and for round trips.
// ===========================================================================
namespace wire {
inline void varint_put(std::vector<uint8_t>& out, uint64_t v) {
  while (v >= 0x80) {
    out.push_back(static_cast<uint8_t>(v | 0x80));
    v >>= 7;
  }
  out.push_back(static_cast<uint8_t>(v));
}
// returns false on a truncated or over-long varint
inline bool varint_get(const uint8_t* d, size_t n, size_t& p, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (p >= n) return false;
    const uint8_t b = d[p++];
    v |= static_cast<uint64_t>(b & 0x7F) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}
constexpr size_t kRunMin = 4;
inline std::vector<uint8_t> rle_encode(const std::vector<uint8_t>& bits) {  // bitfield_rle::encode
  std::vector<uint8_t> out;
  size_t i = 0, lit = 0;  // literal segment [lit, i)
  auto flush = [&](size_t end) {
    if (end > lit) {
      varint_put(out, static_cast<uint64_t>(end - lit) << 1);
      out.insert(out.end(), bits.begin() + static_cast<long>(lit), bits.begin() + static_cast<long>(end));
    }
  };
  while (i < bits.size()) {
    const uint8_t b = bits[i];
    size_t j = i;
    if (b == 0x00 || b == 0xFF)
      while (j < bits.size() && bits[j] == b) ++j;
    if (j - i >= kRunMin) {
      flush(i);
      varint_put(out, (static_cast<uint64_t>(j - i) << 2) | (b ? 2u : 0u) | 1u);
      i = lit = j;
    } else {
      i = j > i ? j : i + 1;
    }
  }
  flush(bits.size());
  return out;
}
// bitfield_rle::decode: false on malformed input (the reference's
// `.expect("decoding failed")` panics, protocol.rs:656)
inline bool rle_decode(const uint8_t* d, size_t n, std::vector<uint8_t>& out) {
  out.clear();
  size_t p = 0;
  while (p < n) {
    uint64_t h;
    if (!varint_get(d, n, p, h)) return false;
    if (h & 1) {
      const uint64_t len = h >> 2;
      if (len > (1u << 16)) return false;
      out.insert(out.end(), static_cast<size_t>(len), (h & 2) ? 0xFF : 0x00);
    } else {
      const uint64_t len = h >> 1;
      if (len > n - p) return false;
      out.insert(out.end(), d + p, d + p + len);
      p += static_cast<size_t>(len);
    }
  }
  return true;
}
// compression.rs:3-11 encode = delta_encode (:13-30) then RLE
inline std::vector<uint8_t> encode(const std::vector<uint8_t>& ref, const std::vector<std::vector<uint8_t>>& pending) {
  std::vector<uint8_t> bytes;
  for (auto& in : pending) {
    ORC_ASSERT(in.size() == ref.size());
    for (size_t i = 0; i < ref.size(); ++i) bytes.push_back(ref[i] ^ in[i]);
  }
  return rle_encode(bytes);
}
// compression.rs:32-57 decode = RLE decode then delta_decode
inline bool decode(const std::vector<uint8_t>& ref, const uint8_t* d, size_t n, std::vector<std::vector<uint8_t>>& out) {
  std::vector<uint8_t> buf;
  if (!rle_decode(d, n, buf)) return false;
  ORC_ASSERT(!ref.empty() && buf.size() % ref.size() == 0);
  out.assign(buf.size() / ref.size(), std::vector<uint8_t>(ref.size()));
  for (size_t k = 0; k < out.size(); ++k)
    for (size_t i = 0; i < ref.size(); ++i) out[k][i] = ref[i] ^ buf[ref.size() * k + i];
  return true;
}
}  // namespace wire

}  // namespace orc
