// ggrs_amd/csrc/ops_exgame.hip — device code of examples/ex_game: the factory.
// Each player count instantiates kernels.hpp for ExGame<P, lane-per-player> in a
// translation unit of its own (ops_exgame_p<P>.hip), so they compile in
// parallel; the lane-per-session layout (ops_exgame_lps.hip) is an A/B build only.
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_exgame_lps_ops(int players);  // ops_exgame_lps.hip (RB_EXPERIMENTS)
std::unique_ptr<GameOps> make_exgame_p1_ops();
std::unique_ptr<GameOps> make_exgame_p2_ops();
std::unique_ptr<GameOps> make_exgame_p3_ops();
std::unique_ptr<GameOps> make_exgame_p4_ops();
std::unique_ptr<GameOps> make_exgame_ops(int players, bool lane_per_session) {
  // the lane-per-session layout (measured slower: 5.35 vs 4.4 us per tick) is built into A/B
  // builds only (RB_EXPERIMENTS=1); the product library refuses RB_FLAG_LANE_PER_SESSION
#if RB_EXPERIMENTS
  if (lane_per_session) return make_exgame_lps_ops(players);
#else
  if (lane_per_session) return nullptr;
#endif
#if RB_EXGAME_P2_ONLY  // kernel-experiment builds (tools/): the bench configuration only
  return players == 2 ? make_exgame_p2_ops() : nullptr;
#else
  switch (players) {
    case 1: return make_exgame_p1_ops();
    case 2: return make_exgame_p2_ops();
    case 3: return make_exgame_p3_ops();
    case 4: return make_exgame_p4_ops();
    default: return nullptr;
  }
#endif
}
}  // namespace rb
