// ggrs_amd/csrc/ops_exgame.hip — device code of examples/ex_game (kernels.hpp
// instantiated for ExGame<P, lane-per-player | lane-per-session>).
#include "kernels.hpp"

namespace rb {
template <bool kSplit>
static std::unique_ptr<GameOps> make_ex_game(int players) {
  switch (players) {
    case 1: return std::make_unique<GameOpsT<ExGame<1, kSplit>>>();
    case 2: return std::make_unique<GameOpsT<ExGame<2, kSplit>>>();
    case 3: return std::make_unique<GameOpsT<ExGame<3, kSplit>>>();
    case 4: return std::make_unique<GameOpsT<ExGame<4, kSplit>>>();
    default: return nullptr;
  }
}
std::unique_ptr<GameOps> make_exgame_ops(int players, bool lane_per_session) {
#if RB_EXGAME_P2_ONLY  // kernel-experiment builds (tools/): the bench configuration only
  if (players == 2 && !lane_per_session) return std::make_unique<GameOpsT<ExGame<2, true>>>();
  return nullptr;
#else
  return lane_per_session ? make_ex_game<false>(players) : make_ex_game<true>(players);
#endif
}
}  // namespace rb
