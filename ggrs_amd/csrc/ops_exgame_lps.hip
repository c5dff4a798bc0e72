// ggrs_amd/csrc/ops_exgame_lps.hip — examples/ex_game with one lane per
// session (ExGame<P, false>: every player's state in one lane), the layout
// RB_FLAG_LANE_PER_SESSION selects.
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_exgame_lps_ops(int players) {
#if RB_EXGAME_P2_ONLY
  (void)players;
  return nullptr;
#else
  switch (players) {
    case 1: return std::make_unique<GameOpsT<ExGame<1, false>>>();
    case 2: return std::make_unique<GameOpsT<ExGame<2, false>>>();
    case 3: return std::make_unique<GameOpsT<ExGame<3, false>>>();
    case 4: return std::make_unique<GameOpsT<ExGame<4, false>>>();
    default: return nullptr;
  }
#endif
}
}  // namespace rb
