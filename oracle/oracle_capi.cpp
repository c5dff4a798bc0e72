// ============================================================================
// oracle/oracle_capi.cpp — TEST INFRASTRUCTURE ONLY.
//
// extern "C" surface of the CPU restatement (oracle/ggrs_oracle.hpp) so that
// the Python tests (tests/) and bench.py's cpu_baseline leg can drive it via
// ctypes.  A "batch" here is S fully independent reference sessions, each a
// SyncTestSession + its game, driven exactly like ex_game_synctest.rs:59-72:
// add_local_input for every handle, advance_frame, handle_requests.
// Nothing in the product links this library.
// ============================================================================
#include <atomic>
#include <chrono>
#include <thread>

#include "ggrs_oracle.hpp"
#ifdef RB_PLUGIN_GAME  // oracle/Makefile `plugin`: the user's game header is -included
#include "plugin_game.hpp"
using PluginU = RB_PLUGIN_GAME;
#endif

using namespace orc;

namespace {

enum GameId : int32_t { EX_GAME = 1, STUB = 2, STUB_ENUM = 3, STUB_RANDOM_CS = 4, BRAWLER = 5, PLUGIN = 100 };
constexpr int32_t KIND_PANIC = 99;

struct BatchBase {
  virtual ~BatchBase() = default;
  virtual int32_t add_local_input(int32_t handle, const uint8_t* inputs) = 0;
  virtual int32_t advance(int32_t* kinds, int32_t* frames) = 0;
  virtual int32_t trace(int32_t session, int32_t* kinds, int32_t* frames, int32_t cap) = 0;
  virtual int32_t read_cells(int32_t* cell_frames, uint8_t* images, uint8_t* cs_valid, uint64_t* cs) = 0;
  virtual int32_t read_live(uint8_t* images, uint64_t* last_cs, int32_t* last_cs_frame) = 0;
  virtual int32_t current_frame() = 0;
  virtual int32_t corrupt_cell(int32_t session, int32_t frame, int32_t word, uint32_t xor_mask) = 0;
  std::string last_panic;
};

// Canonical state images: bincode image for ex_game, le32(frame)||le32(state) for stubs.
inline std::vector<uint8_t> image_of(const exgame::State& s) { return exgame::bincode_serialize(s); }
inline std::vector<uint8_t> image_of(const stub::StateStub& s) {
  std::vector<uint8_t> v(8);
  std::memcpy(v.data(), &s.frame, 4);
  std::memcpy(v.data() + 4, &s.state, 4);
  return v;
}
inline std::vector<uint8_t> image_of(const stub::StateStubEnum& s) {
  std::vector<uint8_t> v(8);
  std::memcpy(v.data(), &s.frame, 4);
  std::memcpy(v.data() + 4, &s.state, 4);
  return v;
}
inline std::vector<uint8_t> image_of(const brawler::State& s) { return brawler::image(s); }
#ifdef RB_PLUGIN_GAME
inline std::vector<uint8_t> image_of(const plugin::State<PluginU>& s) { return plugin::image(s); }
inline void corrupt_state(plugin::State<PluginU>& st, int32_t k, uint32_t m) { st.w.at(static_cast<size_t>(k)) ^= m; }
#endif
inline uint64_t display_checksum(const exgame::Game& g, int32_t* f) { *f = g.last_checksum.first; return g.last_checksum.second; }
template <class G>
inline uint64_t display_checksum(const G&, int32_t* f) { *f = NULL_FRAME; return 0; }
inline const exgame::State& live_of(const exgame::Game& g) { return g.game_state; }
// Word k of the engine's state layout (positions, velocities, rotations /
// stub state) flipped in place: fault injection for the desync tests.
inline void corrupt_state(exgame::State& st, int32_t k, uint32_t m) {
  const int32_t P = static_cast<int32_t>(st.num_players);
  float* f;
  if (k < 2 * P) f = (k % 2) ? &st.positions[k / 2].second : &st.positions[k / 2].first;
  else if (k < 4 * P) f = ((k - 2 * P) % 2) ? &st.velocities[(k - 2 * P) / 2].second : &st.velocities[(k - 2 * P) / 2].first;
  else f = &st.rotations[k - 4 * P];
  uint32_t u;
  std::memcpy(&u, f, 4);
  u ^= m;
  std::memcpy(f, &u, 4);
}
inline void corrupt_state(brawler::State& st, int32_t k, uint32_t m) {
  st.ent.at(static_cast<size_t>(k)) ^= static_cast<int32_t>(m);  // canonical word k = entity * 8 + field
}
inline void corrupt_state(stub::StateStub& st, int32_t, uint32_t m) { st.state ^= static_cast<int32_t>(m); }
inline void corrupt_state(stub::StateStubEnum& st, int32_t, uint32_t m) { st.state ^= static_cast<int32_t>(m); }
template <class G>
inline const auto& live_of(const G& g) { return g.gs; }
inline exgame::State& mutable_live(exgame::Game& g) { return g.game_state; }
template <class G>
inline auto& mutable_live(G& g) { return g.gs; }

template <class C, class G>
struct Batch : BatchBase {
  using I = typename C::Input;
  std::vector<std::unique_ptr<SyncTestSession<C>>> sess;
  std::vector<G> games;
  std::vector<std::vector<Request<C>>> last_reqs;
  size_t max_pred;

  template <class MakeGame>
  Batch(const SessionBuilder& b, int32_t S, MakeGame mk) : max_pred(b.max_prediction) {
    for (int32_t s = 0; s < S; ++s) {
      std::unique_ptr<SyncTestSession<C>> p;
      Error e = b.start_synctest_session<C>(&p);
      if (e.is_err()) throw std::runtime_error(e.info);
      sess.push_back(std::move(p));
      games.push_back(mk(s));
    }
    last_reqs.resize(S);
  }

  int32_t add_local_input(int32_t handle, const uint8_t* in) override {
    int32_t first = 0;
    for (size_t s = 0; s < sess.size(); ++s) {
      I v{};
      std::memcpy(&v, in + s * sizeof(I), sizeof(I));
      Error e = sess[s]->add_local_input(static_cast<PlayerHandle>(handle < 0 ? SIZE_MAX : handle), v);
      if (e.is_err() && first == 0) first = static_cast<int32_t>(e.kind);
    }
    return first;
  }

  int32_t advance(int32_t* kinds, int32_t* frames) override {
    int32_t nerr = 0;
    for (size_t s = 0; s < sess.size(); ++s) {
      int32_t k = 0;
      Frame f = NULL_FRAME;
      try {
        Error e = sess[s]->advance_frame(last_reqs[s]);
        if (e.is_err()) {
          k = static_cast<int32_t>(e.kind);
          f = e.frame;
          last_reqs[s].clear();
        } else {
          games[s].handle_requests(last_reqs[s]);
        }
      } catch (const Panic& p) {
        k = KIND_PANIC;
        last_panic = p.what();
      }
      if (k) ++nerr;
      if (kinds) kinds[s] = k;
      if (frames) frames[s] = f;
    }
    return nerr;
  }

  int32_t trace(int32_t session, int32_t* kinds, int32_t* frames, int32_t cap) override {
    auto& r = last_reqs.at(session);
    int32_t n = static_cast<int32_t>(r.size());
    for (int32_t i = 0; i < n && i < cap; ++i) {
      kinds[i] = static_cast<int32_t>(r[i].kind);
      frames[i] = r[i].frame;
    }
    return n;
  }

  int32_t read_cells(int32_t* cell_frames, uint8_t* images, uint8_t* cs_valid, uint64_t* cs) override {
    const size_t S = sess.size();
    size_t img = 0;
    for (size_t w = 0; w < max_pred; ++w) {
      for (size_t s = 0; s < S; ++s) {
        const auto& cell = sess[s]->sync_layer.saved_states.states[w];
        if (s == 0 && cell_frames) cell_frames[w] = cell.frame();
        auto d = cell.load();
        if (d) {
          auto v = image_of(*d);
          img = v.size();
          if (images) std::memcpy(images + (w * S + s) * img, v.data(), img);
        }
        auto c = cell.checksum();
        if (cs_valid) cs_valid[w * S + s] = c.has_value();
        if (cs) {
          u128 x = c.value_or(0);
          cs[(w * S + s) * 2 + 0] = static_cast<uint64_t>(x);
          cs[(w * S + s) * 2 + 1] = static_cast<uint64_t>(x >> 64);
        }
      }
    }
    return static_cast<int32_t>(img);
  }

  int32_t read_live(uint8_t* images, uint64_t* last_cs, int32_t* last_cs_frame) override {
    size_t img = 0;
    for (size_t s = 0; s < sess.size(); ++s) {
      auto v = image_of(live_of(games[s]));
      img = v.size();
      if (images) std::memcpy(images + s * img, v.data(), img);
      int32_t f;
      uint64_t c = display_checksum(games[s], &f);
      if (last_cs) last_cs[s] = c;
      if (last_cs_frame) last_cs_frame[s] = f;
    }
    return static_cast<int32_t>(img);
  }

  int32_t current_frame() override { return sess.empty() ? 0 : sess[0]->current_frame(); }

  int32_t corrupt_cell(int32_t session, int32_t frame, int32_t word, uint32_t m) override {
    auto cell = sess.at(session)->sync_layer.saved_state_by_frame(frame);
    if (!cell) return -1;
    auto d = cell->load();
    if (!d) return -1;
    corrupt_state(*d, word, m);
    cell->save(frame, *d, cell->checksum());
    return 0;
  }
};

// S independent network-free P2PSessions (ggrs_oracle.hpp P2PSession) + their
// games, driven like ex_game_p2p.rs:105-125: deliver the remote inputs that
// "arrived" (poll_remote_clients), add_local_input for every local handle,
// advance_frame, handle_requests.
struct P2PBatchBase {
  virtual ~P2PBatchBase() = default;
  virtual int32_t deliver(int32_t handle, const int32_t* upto, const uint8_t* by_frame, int32_t n_frames) = 0;
  virtual int32_t add_local_input(int32_t handle, const uint8_t* inputs) = 0;
  virtual int32_t disconnect(int32_t handle, const uint8_t* mask) = 0;
  virtual int32_t advance(int32_t* status, int32_t* load_frame, int32_t* n_adv, int32_t* n_save) = 0;
  virtual int32_t trace(int32_t session, int32_t* kinds, int32_t* frames, int32_t cap) = 0;
  virtual int32_t read_cells(int32_t* cell_frames, uint8_t* images, uint64_t* cs) = 0;
  virtual int32_t read_live(uint8_t* images, int32_t* frames) = 0;
  virtual int32_t frames(int32_t* current, int32_t* confirmed) = 0;
  virtual int32_t queues(int32_t* out) = 0;  // [S][P][8], rb_p2p_read_queues's layout
  // desync detection (p2p_session.rs:873-928)
  virtual void set_desync(uint32_t interval) = 0;
  virtual int32_t take_reports(int32_t* frames, uint64_t* cs, int32_t K) = 0;
  virtual int32_t receive_reports(int32_t handle, const int32_t* frames, const uint64_t* cs, int32_t K) = 0;
  virtual int32_t events(uint32_t* counts, int32_t* frames, int32_t* handles, uint64_t* local, uint64_t* remote,
                         int32_t E) = 0;
  virtual int32_t corrupt(int32_t session, int32_t word, uint32_t mask) = 0;
  virtual int32_t receive_peer_status(int32_t endpoint, const int32_t* last_frames, const uint8_t* disconnected) = 0;
  std::string last_panic;
};

template <class C, class G>
struct P2PBatch : P2PBatchBase {
  using I = typename C::Input;
  std::vector<std::unique_ptr<P2PSession<C>>> sess;
  std::vector<G> games;
  std::vector<std::vector<Request<C>>> last_reqs;
  int32_t remote_first;  // frame of a remote's first input (the remote's input delay)
  size_t max_pred;

  template <class MakeGame>
  P2PBatch(int32_t P, int32_t W, int32_t delay, uint32_t local_mask, bool sparse, int32_t remote_delay, int32_t S,
           MakeGame mk)
      : remote_first(remote_delay), max_pred(static_cast<size_t>(W)) {
    std::vector<bool> local(static_cast<size_t>(P));
    for (int32_t h = 0; h < P; ++h) local[h] = (local_mask >> h) & 1u;
    for (int32_t s = 0; s < S; ++s) {
      sess.push_back(std::make_unique<P2PSession<C>>(P, W, sparse, delay, local));
      games.push_back(mk(s));
    }
    last_reqs.resize(S);
    panicked.assign(S, false);
  }
  // A reference panic aborts the process; a batch freezes the session that hit
  // it and keeps reporting the panic (the device does the same).
  std::vector<bool> panicked;

  int32_t deliver(int32_t handle, const int32_t* upto, const uint8_t* by_frame, int32_t n_frames) override {
    const size_t S = sess.size();
    int32_t rc = 0;
    for (size_t s = 0; s < S; ++s) {
      if (panicked[s]) continue;
      auto& ss = *sess[s];
      try {  // poll_remote_clients: a reference assert here panics this session only
        Frame last = ss.local_connect_status.at(handle).last_frame;
        Frame f0 = last == NULL_FRAME ? remote_first : last + 1;
        for (Frame f = f0; f <= upto[s]; ++f) {
          if (f >= n_frames) throw Panic("deliver: frame beyond the provided inputs");
          I v{};
          std::memcpy(&v, by_frame + (static_cast<size_t>(f) * S + s) * sizeof(I), sizeof(I));
          ss.deliver_remote_input(static_cast<PlayerHandle>(handle), PlayerInput<I>(f, v));
        }
      } catch (const Panic& p) {
        last_panic = p.what();
        panicked[s] = true;
        last_reqs[s].clear();
        rc = KIND_PANIC;
      }
    }
    return rc;
  }

  int32_t add_local_input(int32_t handle, const uint8_t* in) override {
    int32_t first = 0;
    for (size_t s = 0; s < sess.size(); ++s) {
      if (panicked[s]) continue;
      I v{};
      std::memcpy(&v, in + s * sizeof(I), sizeof(I));
      Error e = sess[s]->add_local_input(static_cast<PlayerHandle>(handle), v);
      if (e.is_err() && first == 0) first = static_cast<int32_t>(e.kind);
    }
    return first;
  }

  // disconnect_player(handle) in every session whose mask byte is set (NULL: all);
  // returns the first error kind (0 = ok)
  int32_t disconnect(int32_t handle, const uint8_t* mask) override {
    int32_t first = 0;
    for (size_t s = 0; s < sess.size(); ++s) {
      if ((mask && !mask[s]) || panicked[s]) continue;
      Error e = sess[s]->disconnect_player(static_cast<PlayerHandle>(handle));
      if (e.is_err() && first == 0) first = static_cast<int32_t>(e.kind);
    }
    return first;
  }

  int32_t advance(int32_t* status, int32_t* load_frame, int32_t* n_adv, int32_t* n_save) override {
    int32_t nerr = 0;
    for (size_t s = 0; s < sess.size(); ++s) {
      int32_t k = 0;
      if (panicked[s]) {
        k = KIND_PANIC;
      } else try {
        Error e = sess[s]->advance_frame(last_reqs[s]);
        if (e.is_err()) k = static_cast<int32_t>(e.kind);
        // on Err the requests built before the failure stay in the Vec the
        // reference drops; the game never sees them, but the session's
        // bookkeeping (rollback, saves) has happened (p2p_session.rs:253-337)
        if (!e.is_err()) games[s].handle_requests(last_reqs[s]);
        else last_reqs[s].clear();
      } catch (const Panic& p) {
        k = KIND_PANIC;
        last_panic = p.what();
        panicked[s] = true;
      }
      Frame lf = NULL_FRAME;
      int32_t na = 0, ns = 0;
      for (auto& r : last_reqs[s]) {
        if (r.kind == RequestKind::Load) lf = r.frame;
        na += r.kind == RequestKind::Advance;
        ns += r.kind == RequestKind::Save;
      }
      if (k) ++nerr;
      if (status) status[s] = k;
      if (load_frame) load_frame[s] = lf;
      if (n_adv) n_adv[s] = na;
      if (n_save) n_save[s] = ns;
    }
    return nerr;
  }

  int32_t trace(int32_t session, int32_t* kinds, int32_t* frames, int32_t cap) override {
    auto& r = last_reqs.at(session);
    int32_t n = static_cast<int32_t>(r.size());
    for (int32_t i = 0; i < n && i < cap; ++i) {
      kinds[i] = static_cast<int32_t>(r[i].kind);
      frames[i] = r[i].frame;
    }
    return n;
  }

  // cells [W][S]: per-session frame tag, image, checksum (lo, hi)
  int32_t read_cells(int32_t* cell_frames, uint8_t* images, uint64_t* cs) override {
    const size_t S = sess.size();
    size_t img = 0;
    for (size_t w = 0; w < max_pred; ++w)
      for (size_t s = 0; s < S; ++s) {
        const auto& cell = sess[s]->sync_layer.saved_states.states[w];
        if (cell_frames) cell_frames[w * S + s] = cell.frame();
        auto d = cell.load();
        if (d) {
          auto v = image_of(*d);
          img = v.size();
          if (images) std::memcpy(images + (w * S + s) * img, v.data(), img);
        }
        u128 x = cell.checksum().value_or(0);
        if (cs) {
          cs[(w * S + s) * 2 + 0] = static_cast<uint64_t>(x);
          cs[(w * S + s) * 2 + 1] = static_cast<uint64_t>(x >> 64);
        }
      }
    return static_cast<int32_t>(img);
  }

  int32_t read_live(uint8_t* images, int32_t* frames_out) override {
    size_t img = 0;
    for (size_t s = 0; s < sess.size(); ++s) {
      auto v = image_of(live_of(games[s]));
      img = v.size();
      if (images) std::memcpy(images + s * img, v.data(), img);
      if (frames_out) frames_out[s] = sess[s]->current_frame();
    }
    return static_cast<int32_t>(img);
  }

  int32_t frames(int32_t* current, int32_t* confirmed) override {
    for (size_t s = 0; s < sess.size(); ++s) {
      if (current) current[s] = sess[s]->current_frame();
      if (confirmed) confirmed[s] = sess[s]->sync_layer.last_confirmed_frame;
    }
    return 0;
  }

  int32_t queues(int32_t* out) override {
    for (size_t s = 0; s < sess.size(); ++s) {
      const auto& sl = sess[s]->sync_layer;
      for (size_t h = 0; h < sl.input_queues.size(); ++h) {
        const auto& q = sl.input_queues[h];
        const auto& cs = sess[s]->local_connect_status[h];
        int32_t* o = out + (s * sl.input_queues.size() + h) * 8;
        o[0] = q.last_added_frame;
        o[1] = q.inputs[q.tail].frame;
        o[2] = static_cast<int32_t>(q.length);
        o[3] = q.last_requested_frame;
        o[4] = q.prediction.frame;
        o[5] = q.first_incorrect_frame();
        o[6] = cs.last_frame;
        o[7] = cs.disconnected ? 1 : 0;
      }
    }
    return 0;
  }

  void set_desync(uint32_t interval) override {
    for (auto& ss : sess) ss->desync_interval = interval;
  }
  // The ChecksumReports each session sent since the last take, oldest first:
  // frames [K][S] (NULL_FRAME = none), checksums [K][S][2] (u128 lo, hi).  When
  // more than K were sent only the newest K are kept (a lost datagram).
  int32_t take_reports(int32_t* frames, uint64_t* cs, int32_t K) override {
    const size_t S = sess.size();
    for (size_t s = 0; s < S; ++s) {
      auto& r = sess[s]->sent_reports;
      const size_t n = r.size(), first = n > static_cast<size_t>(K) ? n - K : 0;
      for (int32_t k = 0; k < K; ++k) {
        const size_t i = first + static_cast<size_t>(k);
        const bool has = i < n;
        frames[k * S + s] = has ? r[i].first : NULL_FRAME;
        cs[(k * S + s) * 2 + 0] = has ? static_cast<uint64_t>(r[i].second) : 0;
        cs[(k * S + s) * 2 + 1] = has ? static_cast<uint64_t>(r[i].second >> 64) : 0;
      }
      r.clear();
    }
    return 0;
  }
  // The peer's reports for remote handle `handle`, in the same layout, applied
  // in order by UdpProtocol::on_checksum_report.
  int32_t receive_reports(int32_t handle, const int32_t* frames, const uint64_t* cs, int32_t K) override {
    const size_t S = sess.size();
    try {
      for (size_t s = 0; s < S; ++s) {
        if (panicked[s]) continue;
        for (int32_t k = 0; k < K; ++k) {
          const Frame f = frames[k * S + s];
          if (f == NULL_FRAME) continue;
          const u128 c = (static_cast<u128>(cs[(k * S + s) * 2 + 1]) << 64) | cs[(k * S + s) * 2 + 0];
          sess[s]->on_checksum_report(static_cast<PlayerHandle>(handle), f, c);
        }
      }
    } catch (const Panic& p) {
      last_panic = p.what();
      return KIND_PANIC;
    }
    return 0;
  }
  // DesyncDetected events: total per session, and the newest E in order
  // (frames [S][E] NULL_FRAME-padded, remote handle, local/remote checksum low words).
  int32_t events(uint32_t* counts, int32_t* frames, int32_t* handles, uint64_t* local, uint64_t* remote,
                 int32_t E) override {
    for (size_t s = 0; s < sess.size(); ++s) {
      auto& ev = sess[s]->events;
      const size_t n = ev.size(), first = n > static_cast<size_t>(E) ? n - E : 0;
      if (counts) counts[s] = static_cast<uint32_t>(n);
      for (int32_t e = 0; e < E; ++e) {
        const size_t i = first + static_cast<size_t>(e);
        const bool has = i < n;
        const size_t o = s * E + e;
        if (frames) frames[o] = has ? ev[i].frame : NULL_FRAME;
        if (handles) handles[o] = has ? static_cast<int32_t>(ev[i].handle) : -1;
        if (local) local[o] = has ? static_cast<uint64_t>(ev[i].local_checksum) : 0;
        if (remote) remote[o] = has ? static_cast<uint64_t>(ev[i].remote_checksum) : 0;
      }
    }
    return 0;
  }
  // The peer behind remote handle `endpoint` reported every player's connection
  // status: last_frames [P][S], disconnected [P][S] (UdpProtocol::on_input merge).
  int32_t receive_peer_status(int32_t endpoint, const int32_t* last_frames, const uint8_t* disconnected) override {
    const size_t S = sess.size();
    for (size_t s = 0; s < S; ++s) {
      if (panicked[s]) continue;
      for (size_t i = 0; i < sess[s]->num_players; ++i)
        sess[s]->receive_peer_connect_status(static_cast<PlayerHandle>(endpoint), i, disconnected[i * S + s] != 0,
                                             last_frames[i * S + s]);
    }
    return 0;
  }
  // Fault injection (ex_game.rs:211-215 trigger_desync, generalised): flip
  // word `word` of the session's live game state and of every saved cell's
  // state (cell checksums unchanged), so no rollback can undo it.
  int32_t corrupt(int32_t session, int32_t word, uint32_t mask) override {
    auto& ss = *sess.at(static_cast<size_t>(session));
    corrupt_state(mutable_live(games[static_cast<size_t>(session)]), word, mask);
    for (auto& cell : ss.sync_layer.saved_states.states) {
      auto d = cell.load();
      if (!d || cell.frame() == NULL_FRAME) continue;
      corrupt_state(*d, word, mask);
      cell.save(cell.frame(), *d, cell.checksum());
    }
    return 0;
  }
};

thread_local std::string g_err;

}  // namespace

extern "C" {

int32_t orc_image_bytes(int32_t game, int32_t num_players) {
#ifdef RB_PLUGIN_GAME
  if (game == PLUGIN) return 4 + 4 * PluginU::kStateWords;
#endif
  if (game == BRAWLER) return 4 + brawler::N * 32;
  return game == EX_GAME ? 36 + 20 * num_players : 8;
}
int32_t orc_input_bytes(int32_t game) {
#ifdef RB_PLUGIN_GAME
  if (game == PLUGIN) return PluginU::kInputBytes;
#endif
  return (game == STUB || game == STUB_RANDOM_CS) ? 4 : 1;
}

// Returns NULL on a builder error (message via orc_last_error).
void* orc_batch_create(int32_t game, int32_t num_players, int32_t max_prediction, int32_t check_distance,
                       int32_t input_delay, int32_t num_sessions, uint64_t seed) {
  try {
    SessionBuilder b;
    b.with_num_players(num_players).with_check_distance(check_distance).with_input_delay(input_delay);
    Error e = b.with_max_prediction_window(static_cast<size_t>(max_prediction));
    if (e.is_err()) { g_err = e.info; return nullptr; }
    switch (game) {
      case EX_GAME:
        return new Batch<exgame::Config, exgame::Game>(b, num_sessions, [&](int32_t) { return exgame::Game(num_players); });
      case STUB:
        return new Batch<stub::Config, stub::GameStub>(b, num_sessions, [&](int32_t) { return stub::GameStub{}; });
      case STUB_ENUM:
        return new Batch<stub::EnumConfig, stub::GameStubEnum>(b, num_sessions, [&](int32_t) { return stub::GameStubEnum{}; });
      case BRAWLER:
        return new Batch<brawler::Config, brawler::Game>(b, num_sessions, [&](int32_t) { return brawler::Game(num_players); });
      case STUB_RANDOM_CS:
        return new Batch<stub::Config, stub::RandomChecksumGameStub>(
            b, num_sessions, [&](int32_t s) { return stub::RandomChecksumGameStub(seed ^ (uint64_t(s) * 0x9e37ULL)); });
#ifdef RB_PLUGIN_GAME
      case PLUGIN:
        if (num_players != PluginU::kPlayers) { g_err = "num_players differs from the plugin game's"; return nullptr; }
        return new Batch<plugin::Config<PluginU>, plugin::Game<PluginU>>(b, num_sessions,
                                                                       [&](int32_t) { return plugin::Game<PluginU>(); });
#endif
      default: g_err = "unknown game"; return nullptr;
    }
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return nullptr;
  }
}
const char* orc_last_error() { return g_err.c_str(); }
const char* orc_last_panic(void* b) { return static_cast<BatchBase*>(b)->last_panic.c_str(); }
void orc_batch_destroy(void* b) { delete static_cast<BatchBase*>(b); }
int32_t orc_batch_add_local_input(void* b, int32_t handle, const uint8_t* inputs) {
  return static_cast<BatchBase*>(b)->add_local_input(handle, inputs);
}
int32_t orc_batch_advance(void* b, int32_t* kinds, int32_t* frames) {
  return static_cast<BatchBase*>(b)->advance(kinds, frames);
}
int32_t orc_batch_trace(void* b, int32_t session, int32_t* kinds, int32_t* frames, int32_t cap) {
  return static_cast<BatchBase*>(b)->trace(session, kinds, frames, cap);
}
int32_t orc_batch_read_cells(void* b, int32_t* cell_frames, uint8_t* images, uint8_t* cs_valid, uint64_t* cs) {
  return static_cast<BatchBase*>(b)->read_cells(cell_frames, images, cs_valid, cs);
}
int32_t orc_batch_read_live(void* b, uint8_t* images, uint64_t* last_cs, int32_t* last_cs_frame) {
  return static_cast<BatchBase*>(b)->read_live(images, last_cs, last_cs_frame);
}
int32_t orc_batch_current_frame(void* b) { return static_cast<BatchBase*>(b)->current_frame(); }

// Network-free P2P batches (P2PBatch above).  local_mask: bit h set = handle h
// is local; remote_delay: frame of every remote's first input.
void* orc_p2p_create(int32_t game, int32_t num_players, int32_t max_prediction, int32_t input_delay,
                     uint32_t local_mask, int32_t sparse, int32_t remote_delay, int32_t num_sessions) {
  try {
    if (max_prediction <= 0) { g_err = "Currently, only prediction windows above 0 are supported"; return nullptr; }
    const bool sp = sparse != 0;
    switch (game) {
      case EX_GAME:
        return new P2PBatch<exgame::Config, exgame::Game>(num_players, max_prediction, input_delay, local_mask, sp,
                                                           remote_delay, num_sessions,
                                                           [&](int32_t) { return exgame::Game(num_players); });
      case STUB:
        return new P2PBatch<stub::Config, stub::GameStub>(num_players, max_prediction, input_delay, local_mask, sp,
                                                          remote_delay, num_sessions, [&](int32_t) { return stub::GameStub{}; });
      case STUB_ENUM:
        return new P2PBatch<stub::EnumConfig, stub::GameStubEnum>(num_players, max_prediction, input_delay, local_mask,
                                                                  sp, remote_delay, num_sessions,
                                                                  [&](int32_t) { return stub::GameStubEnum{}; });
#ifdef RB_PLUGIN_GAME
      case PLUGIN:
        if (num_players != PluginU::kPlayers) { g_err = "num_players differs from the plugin game's"; return nullptr; }
        return new P2PBatch<plugin::Config<PluginU>, plugin::Game<PluginU>>(
            num_players, max_prediction, input_delay, local_mask, sp, remote_delay, num_sessions,
            [&](int32_t) { return plugin::Game<PluginU>(); });
#endif
      case BRAWLER:
        return new P2PBatch<brawler::Config, brawler::Game>(num_players, max_prediction, input_delay, local_mask, sp,
                                                            remote_delay, num_sessions,
                                                            [&](int32_t) { return brawler::Game(num_players); });
      default: g_err = "unknown game for p2p"; return nullptr;
    }
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return nullptr;
  }
}
void orc_p2p_destroy(void* b) { delete static_cast<P2PBatchBase*>(b); }
const char* orc_p2p_last_panic(void* b) { return static_cast<P2PBatchBase*>(b)->last_panic.c_str(); }
int32_t orc_p2p_deliver(void* b, int32_t handle, const int32_t* upto, const uint8_t* by_frame, int32_t n_frames) {
  return static_cast<P2PBatchBase*>(b)->deliver(handle, upto, by_frame, n_frames);
}
int32_t orc_p2p_add_local_input(void* b, int32_t handle, const uint8_t* inputs) {
  return static_cast<P2PBatchBase*>(b)->add_local_input(handle, inputs);
}
int32_t orc_p2p_disconnect(void* b, int32_t handle, const uint8_t* mask) {
  return static_cast<P2PBatchBase*>(b)->disconnect(handle, mask);
}
int32_t orc_p2p_advance(void* b, int32_t* status, int32_t* load_frame, int32_t* n_adv, int32_t* n_save) {
  return static_cast<P2PBatchBase*>(b)->advance(status, load_frame, n_adv, n_save);
}
int32_t orc_p2p_trace(void* b, int32_t session, int32_t* kinds, int32_t* frames, int32_t cap) {
  return static_cast<P2PBatchBase*>(b)->trace(session, kinds, frames, cap);
}
int32_t orc_p2p_read_cells(void* b, int32_t* cell_frames, uint8_t* images, uint64_t* cs) {
  return static_cast<P2PBatchBase*>(b)->read_cells(cell_frames, images, cs);
}
int32_t orc_p2p_read_live(void* b, uint8_t* images, int32_t* frames) {
  return static_cast<P2PBatchBase*>(b)->read_live(images, frames);
}
int32_t orc_p2p_frames(void* b, int32_t* current, int32_t* confirmed) {
  return static_cast<P2PBatchBase*>(b)->frames(current, confirmed);
}
int32_t orc_p2p_queues(void* b, int32_t* out) { return static_cast<P2PBatchBase*>(b)->queues(out); }
void orc_p2p_set_desync(void* b, uint32_t interval) { static_cast<P2PBatchBase*>(b)->set_desync(interval); }
int32_t orc_p2p_take_reports(void* b, int32_t* frames, uint64_t* cs, int32_t K) {
  return static_cast<P2PBatchBase*>(b)->take_reports(frames, cs, K);
}
int32_t orc_p2p_receive_reports(void* b, int32_t handle, const int32_t* frames, const uint64_t* cs, int32_t K) {
  return static_cast<P2PBatchBase*>(b)->receive_reports(handle, frames, cs, K);
}
int32_t orc_p2p_events(void* b, uint32_t* counts, int32_t* frames, int32_t* handles, uint64_t* local, uint64_t* remote,
                       int32_t E) {
  return static_cast<P2PBatchBase*>(b)->events(counts, frames, handles, local, remote, E);
}
int32_t orc_p2p_corrupt(void* b, int32_t session, int32_t word, uint32_t mask) {
  return static_cast<P2PBatchBase*>(b)->corrupt(session, word, mask);
}
int32_t orc_p2p_receive_peer_status(void* b, int32_t endpoint, const int32_t* last_frames, const uint8_t* disc) {
  return static_cast<P2PBatchBase*>(b)->receive_peer_status(endpoint, last_frames, disc);
}

// network/compression.rs wire format (ggrs_oracle.hpp namespace wire).
// encode: n inputs of ref_len bytes against ref; returns the encoded length or
// -1 if cap is too small.  decode: returns the number of inputs, -1 malformed,
// -2 if cap is too small.
int32_t orc_wire_encode(const uint8_t* ref, int32_t ref_len, const uint8_t* inputs, int32_t n, uint8_t* out,
                        int32_t cap) {
  std::vector<uint8_t> r(ref, ref + ref_len);
  std::vector<std::vector<uint8_t>> pend;
  for (int32_t k = 0; k < n; ++k) pend.emplace_back(inputs + k * ref_len, inputs + (k + 1) * ref_len);
  auto e = wire::encode(r, pend);
  if (static_cast<int32_t>(e.size()) > cap) return -1;
  std::memcpy(out, e.data(), e.size());
  return static_cast<int32_t>(e.size());
}
int32_t orc_wire_decode(const uint8_t* ref, int32_t ref_len, const uint8_t* data, int32_t len, uint8_t* out,
                        int32_t cap_inputs) {
  std::vector<uint8_t> r(ref, ref + ref_len);
  std::vector<std::vector<uint8_t>> dec;
  try {
    if (!wire::decode(r, data, static_cast<size_t>(len), dec)) return -1;
  } catch (const Panic&) {
    return -1;
  }
  if (static_cast<int32_t>(dec.size()) > cap_inputs) return -2;
  for (size_t k = 0; k < dec.size(); ++k) std::memcpy(out + k * ref_len, dec[k].data(), ref_len);
  return static_cast<int32_t>(dec.size());
}

// Third-party arithmetic, exposed for the known-answer tests.
uint16_t orc_fletcher16(const uint8_t* d, uint64_t n) { return fletcher16(d, n); }
uint64_t orc_siphash(int32_t c, int32_t d, uint64_t k0, uint64_t k1, const uint8_t* m, uint64_t n) {
  return siphash(c, d, k0, k1, m, n);
}
float orc_cosf(float x) { return std::cos(x); }
float orc_sinf(float x) { return std::sin(x); }
void orc_sincosf_array(const float* in, float* s, float* c, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    s[i] = std::sin(in[i]);
    c[i] = std::cos(in[i]);
  }
}
// Checker of the device's in-range ex_game arithmetic (rb_debug_exgame_inrange; tests/test_gpu_parity.py):
// for the floats with bits first .. first + n - 1, the device's sin and cos (glibc sinf / cosf,
// ex_game.rs:282-283) and the rotation steps rem_euclid(x + ROTATION_SPEED, 2 pi), rem_euclid(x -
// ROTATION_SPEED, 2 pi) (ex_game.rs:291-296) as the steady kernel (rem_euclid_near) and the fan-out
// (rem_euclid) compute them, in `dev` [6][n], against this host's glibc, bit for bit.  Returns the
// mismatch count; *first_bad = the bits of the first mismatching float (0xFFFFFFFF: none).
int64_t orc_check_exgame_inrange(uint32_t first, int64_t n, const float* dev, int32_t threads, uint32_t* first_bad) {
  if (threads < 1) threads = 1;
  std::vector<int64_t> bad(static_cast<size_t>(threads), 0);
  std::vector<uint32_t> fb(static_cast<size_t>(threads), 0xFFFFFFFFu);
  auto bits = [](float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
  };
  auto work = [&](int t) {
    const int64_t lo = n * t / threads, hi = n * (t + 1) / threads;
    for (int64_t i = lo; i < hi; ++i) {
      const uint32_t xb = first + static_cast<uint32_t>(i);
      float x;
      std::memcpy(&x, &xb, 4);
      const float want[6] = {std::sin(x),
                             std::cos(x),
                             exgame::rem_euclid(x + exgame::ROTATION_SPEED, 2.0f * exgame::PI),
                             exgame::rem_euclid(x - exgame::ROTATION_SPEED, 2.0f * exgame::PI),
                             exgame::rem_euclid(x + exgame::ROTATION_SPEED, 2.0f * exgame::PI),
                             exgame::rem_euclid(x - exgame::ROTATION_SPEED, 2.0f * exgame::PI)};
      bool ok = true;
      for (int k = 0; k < 6; ++k) ok &= bits(dev[static_cast<int64_t>(k) * n + i]) == bits(want[k]);
      if (!ok) {
        if (bad[static_cast<size_t>(t)]++ == 0) fb[static_cast<size_t>(t)] = xb;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  int64_t total = 0;
  *first_bad = 0xFFFFFFFFu;
  for (int t = 0; t < threads; ++t) {
    total += bad[static_cast<size_t>(t)];
    if (*first_bad == 0xFFFFFFFFu) *first_bad = fb[static_cast<size_t>(t)];
  }
  return total;
}
int32_t orc_batch_corrupt_cell(void* b, int32_t session, int32_t frame, int32_t word, uint32_t m) {
  return static_cast<BatchBase*>(b)->corrupt_cell(session, frame, word, m);
}
// Synthetic inputs [T][P][S] (u8 or u32 per input_bytes), see ggrs_oracle.hpp SynthInput.
void orc_synth_inputs(uint64_t seed, uint32_t mask, int32_t S, int32_t P, int32_t T, int32_t f0, int32_t input_bytes,
                      void* out) {
  SynthInput g{seed, mask};
  std::vector<uint32_t> prev(static_cast<size_t>(S) * P, 0);
  // replay the hold model from frame 0 up to f0 first
  for (int32_t f = 0; f < f0 + T; ++f)
    for (int32_t p = 0; p < P; ++p)
      for (int32_t s = 0; s < S; ++s) {
        uint32_t& v = prev[static_cast<size_t>(p) * S + s];
        v = g.next(v, s, p, f);
        if (f >= f0) {
          size_t idx = (static_cast<size_t>(f - f0) * P + p) * S + s;
          if (input_bytes == 1) static_cast<uint8_t*>(out)[idx] = static_cast<uint8_t>(v);
          else static_cast<uint32_t*>(out)[idx] = v;
        }
      }
}

// CPU baseline ("port"): S independent SyncTest sessions of a u8-input game
// driven exactly like ex_game_synctest.rs:59-72 on `threads` host threads.
// Inputs are generated before the timed region (as on the GPU side).  Returns
// the wall seconds of the `ticks` timed ticks (after `warmup` untimed ones);
// writes the number of sessions that reported an error to *n_err.
}  // extern "C"

template <class Cfg, class Game>
double bench_game(int32_t num_players, int32_t check_distance, int32_t input_delay, int32_t max_prediction, int32_t S,
                  int32_t warmup, int32_t ticks, int32_t threads, uint64_t seed, uint32_t mask, int32_t* n_err) {
  SessionBuilder b;
  b.with_num_players(num_players).with_check_distance(check_distance).with_input_delay(input_delay);
  if (b.with_max_prediction_window(max_prediction).is_err()) return -1.0;
  const int32_t P = num_players, T = warmup + ticks;
  std::vector<uint8_t> in(static_cast<size_t>(T) * P * S);
  orc_synth_inputs(seed, mask, S, P, T, 0, 1, in.data());
  if (threads < 1) threads = 1;
  struct Worker {
    std::vector<std::unique_ptr<SyncTestSession<Cfg>>> sess;
    std::vector<Game> games;
    int32_t s0 = 0, s1 = 0, errs = 0;
  };
  std::vector<Worker> ws(threads);
  for (int32_t t = 0; t < threads; ++t) {
    ws[t].s0 = static_cast<int32_t>(static_cast<int64_t>(S) * t / threads);
    ws[t].s1 = static_cast<int32_t>(static_cast<int64_t>(S) * (t + 1) / threads);
  }
  auto run = [&](Worker& w, int32_t f0, int32_t f1) {
    std::vector<Request<Cfg>> reqs;
    for (int32_t f = f0; f < f1; ++f)
      for (int32_t s = w.s0; s < w.s1; ++s) {
        auto& sess = *w.sess[s - w.s0];
        for (int32_t p = 0; p < P; ++p)
          sess.add_local_input(p, typename Cfg::Input{in[(static_cast<size_t>(f) * P + p) * S + s]});
        Error e = sess.advance_frame(reqs);
        if (e.is_err()) { ++w.errs; continue; }
        w.games[s - w.s0].handle_requests(reqs);
      }
  };
  auto parallel = [&](auto fn) {
    std::vector<std::thread> th;
    for (int32_t t = 0; t < threads; ++t) th.emplace_back([&, t] { fn(ws[t]); });
    for (auto& x : th) x.join();
  };
  parallel([&](Worker& w) {
    for (int32_t s = w.s0; s < w.s1; ++s) {
      std::unique_ptr<SyncTestSession<Cfg>> p;
      b.start_synctest_session<Cfg>(&p);
      w.sess.push_back(std::move(p));
      w.games.emplace_back(num_players);
    }
    run(w, 0, warmup);
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel([&](Worker& w) { run(w, warmup, T); });
  auto t1 = std::chrono::steady_clock::now();
  int32_t e = 0;
  for (auto& w : ws) e += w.errs;
  if (n_err) *n_err = e;
  return std::chrono::duration<double>(t1 - t0).count();
}

extern "C" {

double orc_bench_exgame(int32_t num_players, int32_t check_distance, int32_t input_delay, int32_t max_prediction,
                        int32_t S, int32_t warmup, int32_t ticks, int32_t threads, uint64_t seed, int32_t* n_err) {
  return bench_game<exgame::Config, exgame::Game>(num_players, check_distance, input_delay, max_prediction, S, warmup,
                                                  ticks, threads, seed, 0x0F, n_err);
}

double orc_bench_brawler(int32_t num_players, int32_t check_distance, int32_t input_delay, int32_t max_prediction,
                         int32_t S, int32_t warmup, int32_t ticks, int32_t threads, uint64_t seed, int32_t* n_err) {
  return bench_game<brawler::Config, brawler::Game>(num_players, check_distance, input_delay, max_prediction, S,
                                                    warmup, ticks, threads, seed, 0xFF, n_err);
}

}  // extern "C"

// CPU baseline for the P2P rollback batches: S network-free reference
// P2PSessions + games (ex_game), driven like ex_game_p2p.rs:105-125 with the
// delivery schedule bench.py generates (same arrays as the GPU run), split
// over `threads` host threads.  Returns the wall seconds of ticks
// [warmup, T); *adv = AdvanceFrames the games executed in that region.
template <class Cfg, class Game>
double bench_p2p_game(int32_t P, int32_t W, int32_t delay, uint32_t local_mask, int32_t remote_delay, int32_t S,
                      int32_t T, int32_t warmup, int32_t threads, const uint8_t* inputs /*[T][P][S]*/,
                      const int32_t* upto /*[T][P][S]*/, const uint8_t* remote_in /*[F][P][S]*/, int32_t F,
                      int64_t* adv, int32_t* n_err) {
  if (threads < 1) threads = 1;
  std::vector<bool> local(static_cast<size_t>(P));
  for (int32_t h = 0; h < P; ++h) local[h] = (local_mask >> h) & 1u;
  struct Worker {
    std::vector<std::unique_ptr<P2PSession<Cfg>>> sess;
    std::vector<Game> games;
    int32_t s0 = 0, s1 = 0, errs = 0;
    int64_t adv = 0;
  };
  std::vector<Worker> ws(threads);
  for (int32_t t = 0; t < threads; ++t) {
    ws[t].s0 = static_cast<int32_t>(static_cast<int64_t>(S) * t / threads);
    ws[t].s1 = static_cast<int32_t>(static_cast<int64_t>(S) * (t + 1) / threads);
  }
  auto idx = [&](int32_t f, int32_t h, int32_t s) { return (static_cast<size_t>(f) * P + h) * S + s; };
  auto run = [&](Worker& w, int32_t t0, int32_t t1, bool count) {
    std::vector<Request<Cfg>> reqs;
    for (int32_t t = t0; t < t1; ++t)
      for (int32_t s = w.s0; s < w.s1; ++s) {
        auto& ss = *w.sess[s - w.s0];
        for (int32_t h = 0; h < P; ++h) {
          if (local[h]) continue;
          Frame last = ss.local_connect_status[h].last_frame;
          for (Frame f = last == NULL_FRAME ? remote_delay : last + 1; f <= upto[idx(t, h, s)] && f < F; ++f)
            ss.deliver_remote_input(h, PlayerInput<typename Cfg::Input>(f, typename Cfg::Input{remote_in[idx(f, h, s)]}));
        }
        for (int32_t h = 0; h < P; ++h)
          if (local[h]) ss.add_local_input(h, typename Cfg::Input{inputs[idx(t, h, s)]});
        Error e = ss.advance_frame(reqs);
        if (e.is_err()) {
          ++w.errs;
          continue;
        }
        if (count)
          for (auto& r : reqs) w.adv += r.kind == RequestKind::Advance;
        w.games[s - w.s0].handle_requests(reqs);
      }
  };
  auto parallel = [&](auto fn) {
    std::vector<std::thread> th;
    for (int32_t t = 0; t < threads; ++t) th.emplace_back([&, t] { fn(ws[t]); });
    for (auto& x : th) x.join();
  };
  parallel([&](Worker& w) {
    for (int32_t s = w.s0; s < w.s1; ++s) {
      w.sess.push_back(std::make_unique<P2PSession<Cfg>>(P, W, false, delay, local));
      w.games.emplace_back(P);
    }
    run(w, 0, warmup, false);
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel([&](Worker& w) { run(w, warmup, T, true); });
  auto t1 = std::chrono::steady_clock::now();
  int64_t a = 0;
  int32_t e = 0;
  for (auto& w : ws) {
    a += w.adv;
    e += w.errs;
  }
  if (adv) *adv = a;
  if (n_err) *n_err = e;
  return std::chrono::duration<double>(t1 - t0).count();
}

extern "C" {
double orc_bench_p2p_exgame(int32_t P, int32_t W, int32_t delay, uint32_t local_mask, int32_t remote_delay, int32_t S,
                            int32_t T, int32_t warmup, int32_t threads, const uint8_t* inputs, const int32_t* upto,
                            const uint8_t* remote_in, int32_t F, int64_t* adv, int32_t* n_err) {
  return bench_p2p_game<exgame::Config, exgame::Game>(P, W, delay, local_mask, remote_delay, S, T, warmup, threads,
                                                      inputs, upto, remote_in, F, adv, n_err);
}
double orc_bench_p2p_brawler(int32_t P, int32_t W, int32_t delay, uint32_t local_mask, int32_t remote_delay, int32_t S,
                             int32_t T, int32_t warmup, int32_t threads, const uint8_t* inputs, const int32_t* upto,
                             const uint8_t* remote_in, int32_t F, int64_t* adv, int32_t* n_err) {
  return bench_p2p_game<brawler::Config, brawler::Game>(P, W, delay, local_mask, remote_delay, S, T, warmup, threads,
                                                        inputs, upto, remote_in, F, adv, n_err);
}
}  // extern "C"

