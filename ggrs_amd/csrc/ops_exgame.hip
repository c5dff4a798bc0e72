// ggrs_amd/csrc/ops_exgame.hip — device code of examples/ex_game (kernels.hpp
// instantiated for ExGame<P, lane-per-player>; the lane-per-session layout
// builds in ops_exgame_lps.hip, a translation unit of its own so the two
// compile in parallel).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_exgame_lps_ops(int players);  // ops_exgame_lps.hip
std::unique_ptr<GameOps> make_exgame_ops(int players, bool lane_per_session) {
#if RB_EXGAME_P2_ONLY  // kernel-experiment builds (tools/): the bench configuration only
  if (players == 2 && !lane_per_session) return std::make_unique<GameOpsT<ExGame<2, true>>>();
  return nullptr;
#else
  if (lane_per_session) return make_exgame_lps_ops(players);
  switch (players) {
    case 1: return std::make_unique<GameOpsT<ExGame<1, true>>>();
    case 2: return std::make_unique<GameOpsT<ExGame<2, true>>>();
    case 3: return std::make_unique<GameOpsT<ExGame<3, true>>>();
    case 4: return std::make_unique<GameOpsT<ExGame<4, true>>>();
    default: return nullptr;
  }
#endif
}
}  // namespace rb
