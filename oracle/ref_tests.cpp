// ============================================================================
// oracle/ref_tests.cpp — TEST INFRASTRUCTURE ONLY.
//
// Pins the CPU restatement (ggrs_oracle.hpp) against every known-answer test
// the reference holds for this path, restated one for one:
//   src/frame_info.rs:83-102            (3 tests)
//   src/input_queue.rs:269-326          (5 tests)
//   src/sync_layer.rs:301-343           (2 tests)
//   tests/test_synctest_session.rs      (5 tests)
//   tests/test_synctest_session_enum.rs (1 test)
//   src/network/compression.rs:81-90    (1 test)
// plus the published vectors for the third-party arithmetic on the path
// (fletcher16, SipHash).  Run by tests/test_oracle.py; exits non-zero on any
// failure and prints one line per test.
// ============================================================================
#include <cstdio>
#include <functional>

#include "ggrs_oracle.hpp"

using namespace orc;

static int g_fail = 0, g_pass = 0;

static void run(const char* name, const std::function<void()>& fn, bool should_panic = false) {
  bool panicked = false;
  std::string what;
  try {
    fn();
  } catch (const Panic& p) {
    panicked = true;
    what = p.what();
  } catch (const std::exception& e) {
    panicked = true;
    what = e.what();
  }
  bool ok = should_panic ? panicked : !panicked;
  std::printf("%s %s%s%s\n", ok ? "PASS" : "FAIL", name, panicked ? " :: " : "", what.c_str());
  (ok ? g_pass : g_fail)++;
}
#define CHECK(c) ORC_ASSERT(c)
#define UNWRAP(e) do { Error _e = (e); if (_e.is_err()) throw Panic("unwrap on Err kind=" + std::to_string(int(_e.kind)) + " frame=" + std::to_string(_e.frame)); } while (0)

struct TestInput { uint8_t inp; };  // input_queue.rs:255-259, sync_layer.rs:287-291

int main() {
  // ---- network/compression.rs:81-90 -------------------------------------------
  run("compression::test_encode_decode", [] {
    std::vector<uint8_t> ref{0, 0, 0, 1};
    std::vector<std::vector<uint8_t>> pend{{0, 0, 1, 0}, {0, 0, 1, 1}, {0, 1, 0, 0}, {0, 1, 0, 1}, {0, 1, 1, 0}};
    auto enc = wire::encode(ref, pend);
    std::vector<std::vector<uint8_t>> dec;
    CHECK(wire::decode(ref, enc.data(), enc.size(), dec));
    CHECK(dec == pend);
  });
  // ---- frame_info.rs:83-102 ------------------------------------------------
  run("frame_info::test_input_equality", [] {
    PlayerInput<TestInput> a(0, {5}), b(0, {5});
    CHECK(a.equal(b, false));
  });
  run("frame_info::test_input_equality_input_only", [] {
    PlayerInput<TestInput> a(0, {5}), b(5, {5});
    CHECK(a.equal(b, true));
  });
  run("frame_info::test_input_equality_fail", [] {
    PlayerInput<TestInput> a(0, {5}), b(0, {7});
    CHECK(!a.equal(b, false));
  });

  // ---- input_queue.rs:269-326 -----------------------------------------------
  run("input_queue::test_add_input_wrong_frame", [] {
    InputQueue<TestInput> q;
    q.add_input(PlayerInput<TestInput>(0, {0}));
    q.add_input(PlayerInput<TestInput>(3, {0}));
  }, /*should_panic=*/true);
  run("input_queue::test_add_input_twice", [] {
    InputQueue<TestInput> q;
    PlayerInput<TestInput> in(0, {0});
    q.add_input(in);
    q.add_input(in);
  }, true);
  run("input_queue::test_add_input_sequentially", [] {
    InputQueue<TestInput> q;
    for (int i = 0; i < 10; ++i) {
      q.add_input(PlayerInput<TestInput>(i, {0}));
      CHECK(q.last_added_frame == i);
      CHECK(q.length == static_cast<size_t>(i + 1));
    }
  });
  run("input_queue::test_input_sequentially", [] {
    InputQueue<TestInput> q;
    for (int i = 0; i < 10; ++i) {
      q.add_input(PlayerInput<TestInput>(i, {static_cast<uint8_t>(i)}));
      CHECK(q.last_added_frame == i);
      CHECK(q.length == static_cast<size_t>(i + 1));
      CHECK(q.input(i).first.inp == i);
    }
  });
  run("input_queue::test_delayed_inputs", [] {
    InputQueue<TestInput> q;
    const int delay = 2;
    q.set_frame_delay(delay);
    for (int i = 0; i < 10; ++i) {
      q.add_input(PlayerInput<TestInput>(i, {static_cast<uint8_t>(i)}));
      CHECK(q.last_added_frame == i + delay);
      CHECK(q.length == static_cast<size_t>(i + delay + 1));
      CHECK(q.input(i).first.inp == std::max(0, i - delay));
    }
  });

  // ---- sync_layer.rs:301-343 ------------------------------------------------
  struct TestConfig { using Input = TestInput; using State = uint8_t; };
  run("sync_layer::test_reach_prediction_threshold", [] {
    SyncLayer<TestConfig> sl(2, 8);
    for (int i = 0; i < 20; ++i) {
      UNWRAP(sl.add_local_input(0, PlayerInput<TestInput>(i, {static_cast<uint8_t>(i)}), nullptr));
      sl.advance_frame();
    }
  }, true);
  run("sync_layer::test_different_delays", [] {
    SyncLayer<TestConfig> sl(2, 8);
    const int p1_delay = 2, p2_delay = 0;
    sl.set_frame_delay(0, p1_delay);
    sl.set_frame_delay(1, p2_delay);
    std::vector<ConnectionStatus> st(2);
    for (int i = 0; i < 20; ++i) {
      PlayerInput<TestInput> in(i, {static_cast<uint8_t>(i)});
      sl.add_remote_input(0, in);
      sl.add_remote_input(1, in);
      st[0].last_frame = i;
      st[1].last_frame = i;
      if (i >= 3) {
        auto si = sl.synchronized_inputs(st);
        CHECK(si[0].first.inp == i - p1_delay);
        CHECK(si[1].first.inp == i - p2_delay);
      }
      sl.advance_frame();
    }
  });

  // ---- tests/test_synctest_session.rs ----------------------------------------
  run("test_synctest_session::test_create_session", [] {
    std::unique_ptr<SyncTestSession<stub::Config>> s;
    CHECK(!SessionBuilder().start_synctest_session<stub::Config>(&s).is_err());
  });
  run("test_synctest_session::test_advance_frame_no_rollbacks", [] {
    stub::GameStub game;
    std::unique_ptr<SyncTestSession<stub::Config>> s;
    UNWRAP(SessionBuilder().with_check_distance(0).start_synctest_session<stub::Config>(&s));
    std::vector<Request<stub::Config>> reqs;
    for (uint32_t i = 0; i < 200; ++i) {
      UNWRAP(s->add_local_input(0, {i}));
      UNWRAP(s->add_local_input(1, {i}));
      UNWRAP(s->advance_frame(reqs));
      CHECK(reqs.size() == 1);
      game.handle_requests(reqs);
      CHECK(game.gs.frame == static_cast<int32_t>(i) + 1);
    }
  });
  run("test_synctest_session::test_advance_frame_with_rollbacks", [] {
    const uint32_t cd = 2;
    stub::GameStub game;
    std::unique_ptr<SyncTestSession<stub::Config>> s;
    UNWRAP(SessionBuilder().with_check_distance(cd).start_synctest_session<stub::Config>(&s));
    std::vector<Request<stub::Config>> reqs;
    for (uint32_t i = 0; i < 200; ++i) {
      UNWRAP(s->add_local_input(0, {i}));
      UNWRAP(s->add_local_input(1, {i}));
      UNWRAP(s->advance_frame(reqs));
      if (i <= cd) {
        CHECK(reqs.size() == 2);
        CHECK(reqs[0].kind == RequestKind::Save);
        CHECK(reqs[1].kind == RequestKind::Advance);
      } else {
        CHECK(reqs.size() == 6);
        CHECK(reqs[0].kind == RequestKind::Load);
        CHECK(reqs[1].kind == RequestKind::Advance);
        CHECK(reqs[2].kind == RequestKind::Save);
        CHECK(reqs[3].kind == RequestKind::Advance);
        CHECK(reqs[4].kind == RequestKind::Save);
        CHECK(reqs[5].kind == RequestKind::Advance);
      }
      game.handle_requests(reqs);
      CHECK(game.gs.frame == static_cast<int32_t>(i) + 1);
    }
  });
  run("test_synctest_session::test_advance_frames_with_delayed_input", [] {
    stub::GameStub game;
    std::unique_ptr<SyncTestSession<stub::Config>> s;
    UNWRAP(SessionBuilder().with_check_distance(7).with_input_delay(2).start_synctest_session<stub::Config>(&s));
    std::vector<Request<stub::Config>> reqs;
    for (uint32_t i = 0; i < 200; ++i) {
      UNWRAP(s->add_local_input(0, {i}));
      UNWRAP(s->add_local_input(1, {i}));
      UNWRAP(s->advance_frame(reqs));
      game.handle_requests(reqs);
      CHECK(game.gs.frame == static_cast<int32_t>(i) + 1);
    }
  });
  run("test_synctest_session::test_advance_frames_with_random_checksums", [] {
    stub::RandomChecksumGameStub game(0x67677273);
    std::unique_ptr<SyncTestSession<stub::Config>> s;
    UNWRAP(SessionBuilder().with_input_delay(2).start_synctest_session<stub::Config>(&s));
    std::vector<Request<stub::Config>> reqs;
    for (uint32_t i = 0; i < 200; ++i) {
      UNWRAP(s->add_local_input(0, {i}));
      UNWRAP(s->add_local_input(1, {i}));
      UNWRAP(s->advance_frame(reqs));  // MismatchedChecksum -> panic
      game.handle_requests(reqs);
      CHECK(game.gs.frame == static_cast<int32_t>(i) + 1);
    }
  }, true);
  // ---- tests/test_synctest_session_enum.rs ------------------------------------
  run("test_synctest_session_enum::test_enum_advance_frames_with_delayed_input", [] {
    stub::GameStubEnum game;
    std::unique_ptr<SyncTestSession<stub::EnumConfig>> s;
    UNWRAP(SessionBuilder().with_check_distance(7).with_input_delay(2).start_synctest_session<stub::EnumConfig>(&s));
    const stub::EnumInput ins[2] = {stub::EnumInput::Val1, stub::EnumInput::Val2};
    std::vector<Request<stub::EnumConfig>> reqs;
    for (size_t i = 0; i < 200; ++i) {
      UNWRAP(s->add_local_input(0, ins[i % 2]));
      UNWRAP(s->add_local_input(1, ins[i % 2]));
      UNWRAP(s->advance_frame(reqs));
      game.handle_requests(reqs);
      CHECK(game.gs.frame == static_cast<int32_t>(i) + 1);
    }
  });
  // builder.rs:342-347 and :136-141 validation
  run("builder::check_distance_too_big", [] {
    std::unique_ptr<SyncTestSession<stub::Config>> s;
    Error e = SessionBuilder().with_check_distance(8).start_synctest_session<stub::Config>(&s);
    CHECK(e.kind == ErrorKind::InvalidRequest && e.info == "Check distance too big.");
  });
  run("builder::zero_prediction_window", [] {
    SessionBuilder b;
    CHECK(b.with_max_prediction_window(0).kind == ErrorKind::InvalidRequest);
  });

  // ---- third-party arithmetic: published vectors ---------------------------
  run("fletcher16::wikipedia_vectors", [] {
    auto f = [](const char* s) { return fletcher16(reinterpret_cast<const uint8_t*>(s), std::strlen(s)); };
    CHECK(f("abcde") == 0xC8F0);
    CHECK(f("abcdef") == 0x2057);
    CHECK(f("abcdefgh") == 0x0627);
  });
  run("siphash24::paper_vector", [] {
    uint8_t key[16], msg[15];
    for (int i = 0; i < 16; ++i) key[i] = static_cast<uint8_t>(i);
    for (int i = 0; i < 15; ++i) msg[i] = static_cast<uint8_t>(i);
    uint64_t k0, k1;
    std::memcpy(&k0, key, 8);
    std::memcpy(&k1, key + 8, 8);
    CHECK(siphash(2, 4, k0, k1, msg, 15) == 0xa129ca6149be45e5ULL);
    CHECK(siphash(2, 4, k0, k1, msg, 0) == 0x726fdb47dd0e0e31ULL);
  });

  std::printf("SUMMARY pass=%d fail=%d\n", g_pass, g_fail);
  return g_fail == 0 ? 0 : 1;
}
