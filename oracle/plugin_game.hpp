// ============================================================================
// oracle/plugin_game.hpp — TEST INFRASTRUCTURE ONLY.
//
// A user's game written to include/ggrs_amd_game.hpp, wrapped as a reference
// `Config` (lib.rs:240-262: Input: Pod, State: Clone) plus a handle_requests
// handler in the shape of ex_game.rs:76-112, so the oracle's restatements of
// SyncTestSession and P2PSession (ggrs_oracle.hpp) drive the very same game
// code the plugin library runs on the GPU.  Compiled only into
// oracle/build/liboracle_<name>.so (oracle/Makefile `plugin`).
// ============================================================================
#pragma once
#include <array>
#include <cstring>

#include "ggrs_oracle.hpp"

namespace orc {
namespace plugin {

template <class U>
struct Input {  // a Pod of kInputBytes bytes; zeroed = blank (frame_info.rs:56-61)
  uint8_t b[U::kInputBytes];
};

template <class U>
struct State {
  Frame frame = 0;
  std::array<uint32_t, U::kStateWords> w{};
};

template <class U>
struct Config {
  using Input = plugin::Input<U>;
  using State = plugin::State<U>;
};

template <class U>
struct Game {
  State<U> gs;
  Game() { U::init(gs.w.data()); }
  void handle_requests(std::vector<Request<Config<U>>>& reqs) {
    for (auto& r : reqs) {
      switch (r.kind) {
        case RequestKind::Load: {  // load_game_state
          auto d = r.cell.load();
          if (!d) throw Panic("No data found.");
          gs = *d;
          break;
        }
        case RequestKind::Save:  // save_game_state: assert frame, checksum, cell.save
          ORC_ASSERT(gs.frame == r.frame);
          r.cell.save(r.frame, gs, static_cast<u128>(U::checksum(gs.w.data(), gs.frame)));
          break;
        case RequestKind::Advance: {  // advance_frame(inputs)
          uint32_t in[U::kPlayers];
          uint8_t st[U::kPlayers];
          for (int p = 0; p < U::kPlayers; ++p) {
            in[p] = 0;
            std::memcpy(&in[p], r.inputs.at(static_cast<size_t>(p)).first.b, U::kInputBytes);
            st[p] = static_cast<uint8_t>(r.inputs[static_cast<size_t>(p)].second);
          }
          U::advance(gs.w.data(), in, st);
          gs.frame += 1;
          break;
        }
      }
    }
  }
};

// canonical image: le32 frame || le32 words (the engine's PluginGame::image)
template <class U>
inline std::vector<uint8_t> image(const State<U>& s) {
  std::vector<uint8_t> v(4 + 4 * U::kStateWords);
  std::memcpy(v.data(), &s.frame, 4);
  std::memcpy(v.data() + 4, s.w.data(), 4 * U::kStateWords);
  return v;
}

}  // namespace plugin
}  // namespace orc
