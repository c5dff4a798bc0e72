// ggrs_amd/csrc/planner.hpp — host-side SyncTest bookkeeping for a lock-step
// batch, and its lowering to one device tick program.
//
// In a batch every session shares the frame counters, the input-queue
// head/tail/length, the snapshot ring's frame tags and the request stream:
// all of GGRS's bookkeeping depends only on frame numbers, never on input or
// state values (in SyncTest every input is Confirmed).  So the bookkeeping
// runs ONCE on the host, mirroring the reference call for call, and only the
// per-session values (inputs, states, checksums) live on the device.
//
//   SyncTestPlan::advance   sync_test_session.rs:85-146
//   SyncTestPlan::adjust    sync_test_session.rs:178-203
//   QueueFrames             input_queue.rs:10-239 (frame fields only)
//   SyncTestPlan (layer)    sync_layer.rs:110-274 (frame fields only)
//
// Reference assert!/panic! conditions raise rb::Panic -> RB_PANIC at the ABI.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace rb {

constexpr int32_t kNullFrame = -1;
constexpr int kQueueLen = 128;  // input_queue.rs:6
constexpr int kMaxSteps = 64;   // AdvanceFrames per tick program (max_prediction <= 64)

struct Panic : std::runtime_error {
  using std::runtime_error::runtime_error;
};
#define RB_CHECK(c)                                                                              \
  do {                                                                                           \
    if (!(c)) throw ::rb::Panic(std::string("assertion failed: " #c " (") + __FILE__ + ":" +  \
                                std::to_string(__LINE__) + ")");                                \
  } while (0)

enum ReqKind : int32_t { REQ_SAVE = 0, REQ_LOAD = 1, REQ_ADVANCE = 2 };
struct Req {
  int32_t kind, frame;
};

// input_queue.rs InputQueue, frame bookkeeping only.  Slot of frame f is
// f % 128 (head advances in lock step with last_added_frame).
struct QueueFrames {
  int head = 0, tail = 0, length = 0;
  bool first_frame = true;
  int32_t last_added = kNullFrame, first_incorrect = kNullFrame, last_requested = kNullFrame;
  int32_t prediction_frame = kNullFrame;
  int delay = 0;
  int32_t frames[kQueueLen];

  QueueFrames() {
    for (auto& f : frames) f = kNullFrame;
  }
  int prev_pos() const { return head == 0 ? kQueueLen - 1 : head - 1; }

  void reset_prediction() {  // :63-67
    prediction_frame = kNullFrame;
    first_incorrect = kNullFrame;
    last_requested = kNullFrame;
  }
  void discard_confirmed_frames(int32_t frame) {  // :83-101
    if (last_requested != kNullFrame) frame = frame < last_requested ? frame : last_requested;
    if (frame >= last_added) {
      tail = head;
      length = 1;
    } else if (frame <= frames[tail]) {
    } else {
      int offset = frame - frames[tail];
      tail = (tail + offset) % kQueueLen;
      length -= offset;
    }
  }
  // :104-146.  Returns the ring slot holding `requested`; the engine never
  // predicts (SyncTest inputs are always present), so a prediction is a panic.
  int input(int32_t requested) {
    RB_CHECK(first_incorrect == kNullFrame);
    last_requested = requested;
    RB_CHECK(requested >= frames[tail]);
    RB_CHECK(prediction_frame < 0);
    int offset = requested - frames[tail];
    if (offset < length) {
      offset = (offset + tail) % kQueueLen;
      RB_CHECK(frames[offset] == requested);
      return offset;
    }
    throw Panic("input prediction requested in a SyncTest batch (no confirmed input for frame " +
                std::to_string(requested) + ")");
  }
  void add_by_frame(int32_t frame_number) {  // :167-204 (prediction branch unreachable: asserted)
    RB_CHECK(last_added == kNullFrame || frame_number == last_added + 1);
    RB_CHECK(frame_number == 0 || frames[prev_pos()] == frame_number - 1);
    RB_CHECK(prediction_frame == kNullFrame);
    frames[head] = frame_number;
    head = (head + 1) % kQueueLen;
    length += 1;
    RB_CHECK(length <= kQueueLen);
    first_frame = false;
    last_added = frame_number;
  }
  // :149-163 + :207-239.  Appends the device writes the add implies:
  // replicated slots (dst <- src) and the slot that receives the user input.
  int32_t add_input(int32_t in_frame, std::vector<int32_t>* repl_dst, int32_t* repl_src, int32_t* user_slot) {
    RB_CHECK(last_added == kNullFrame || in_frame + delay == last_added + 1);
    const int prev = prev_pos();
    int32_t expected = first_frame ? 0 : frames[prev] + 1;
    int32_t input_frame = in_frame + delay;
    if (expected > input_frame) {
      *user_slot = -1;
      return kNullFrame;
    }
    while (expected < input_frame) {  // replicate inputs[prev] (blank at start)
      repl_dst->push_back(head);
      *repl_src = prev;
      add_by_frame(expected);
      expected += 1;
    }
    RB_CHECK(input_frame == 0 || input_frame == frames[prev_pos()] + 1);
    *user_slot = head;
    add_by_frame(input_frame);
    return input_frame;
  }
};

// One tick, lowered: [LOAD load_frame | live] then n_steps consecutive steps,
// step k = [SAVE frame f0+k with save_mode[k]] + ADVANCE from f0+k.
struct TickProgram {
  bool load = false;
  int32_t load_frame = kNullFrame;
  int32_t f0 = 0, n_steps = 0;
  uint8_t save_mode[kMaxSteps] = {};
  bool live_out = false;
  // input ingestion for this tick
  int32_t user_slot = -1;           // ring slot that receives the new inputs
  std::vector<int32_t> repl_dst;    // ring slots replicated from repl_src
  int32_t repl_src = -1;
};

class SyncTestPlan {
 public:
  int P, W, cd;
  int32_t current = 0, last_confirmed = kNullFrame, last_saved = kNullFrame;
  std::vector<int32_t> cell_frame;  // GameStateCell::frame of each ring slot (frame % W)
  std::vector<QueueFrames> queues;
  std::vector<bool> have_input;     // keys of local_inputs
  std::vector<Req> trace;           // the Vec<GGRSRequest> of the last advance

  SyncTestPlan(int num_players, int max_prediction, int check_distance, int input_delay)
      : P(num_players), W(max_prediction), cd(check_distance), cell_frame(max_prediction, kNullFrame),
        queues(num_players), have_input(num_players, false) {
    for (auto& q : queues) q.delay = input_delay;  // sync_test_session.rs:36-39
  }

  // sync_test_session.rs:61-74
  bool add_local_input(int handle) {
    if (handle < 0 || handle >= P) return false;
    have_input[handle] = true;
    return true;
  }

  // sync_test_session.rs:85-146.  Returns 0 (Ok), 1 (PredictionThreshold) or
  // 2 (InvalidRequest); fills `prog` and `trace`.  State is committed exactly
  // as the reference commits it (including on the error paths).
  int advance(TickProgram& prog, std::string& info) {
    prog = TickProgram{};
    prog.f0 = current;
    trace.clear();
    pending_tags.clear();
    if (cd > 0 && current > cd) {
      // checksums_consistent(current - i), i = 0..=cd: per-session values,
      // evaluated on the device (a session whose resimulation mismatched in
      // the previous tick is frozen there and reports the frame).
      adjust(current - cd, prog);
    }
    int n = 0;
    for (bool h : have_input) n += h;
    if (n != P) {
      info = "Missing local input while calling advance_frame().";
      trace.clear();
      return 2;
    }
    for (int h = 0; h < P; ++h) {  // sync_layer.rs:159-174
      int32_t frames_ahead = current - last_confirmed;
      if (current >= W && frames_ahead >= W) {
        trace.clear();
        return 1;
      }
      std::vector<int32_t> dst;
      int32_t src = -1, slot = -1;
      queues[h].add_input(current, &dst, &src, &slot);
      if (h == 0) {  // every queue sees the same frames (same delay)
        prog.repl_dst = dst;
        prog.repl_src = src;
        prog.user_slot = slot;
      }
    }
    for (int h = 0; h < P; ++h) have_input[h] = false;
    if (cd > 0) save_current_state(prog, SAVE_RECORD_);
    for (auto& q : queues) q.input(current);  // synchronized_inputs: all Confirmed
    push_advance(prog);
    // set_last_confirmed_frame(current - cd, false) (sync_layer.rs:220-244)
    int32_t safe = current - cd;
    last_confirmed = safe;
    if (last_confirmed > 0)
      for (auto& q : queues) q.discard_confirmed_frames(safe - 1);
    // The requests are executed by the device handler: the saved cells now
    // carry these frames (GameStateCell::save, sync_layer.rs:19-25).
    for (int32_t f : pending_tags) cell_frame[f % W] = f;
    // The next tick starts with a LoadGameState unless cd == 0 or it is still
    // inside the first cd frames; then it continues from the live state.
    prog.live_out = !(cd > 0 && current > cd);
    return 0;
  }

  static constexpr uint8_t SAVE_RECORD_ = 1, SAVE_COMPARE_ = 2;

 private:
  std::vector<int32_t> pending_tags;

  void save_current_state(TickProgram& prog, uint8_t mode) {  // sync_layer.rs:118-125
    last_saved = current;
    trace.push_back({REQ_SAVE, current});
    const int k = current - prog.f0;
    RB_CHECK(k >= 0 && k < kMaxSteps);
    prog.save_mode[k] = mode;
    pending_tags.push_back(current);
  }
  void push_advance(TickProgram& prog) {
    RB_CHECK(current == prog.f0 + prog.n_steps);
    RB_CHECK(prog.n_steps < kMaxSteps);
    trace.push_back({REQ_ADVANCE, current});
    prog.n_steps += 1;
    current += 1;
  }
  void adjust(int32_t frame_to, TickProgram& prog) {  // sync_test_session.rs:178-203
    const int32_t start = current;
    const int32_t count = start - frame_to;
    // load_frame (sync_layer.rs:139-155)
    RB_CHECK(frame_to != kNullFrame && frame_to < current && frame_to >= current - W);
    RB_CHECK(cell_frame[frame_to % W] == frame_to);
    current = frame_to;
    trace.push_back({REQ_LOAD, frame_to});
    prog.load = true;
    prog.load_frame = frame_to;
    prog.f0 = frame_to;
    for (auto& q : queues) q.reset_prediction();
    for (int32_t i = 0; i < count; ++i) {
      for (auto& q : queues) q.input(current);
      if (i > 0) save_current_state(prog, SAVE_COMPARE_);
      push_advance(prog);
    }
    RB_CHECK(current == start);
  }
};

}  // namespace rb
