// ggrs_amd/csrc/ops_exgame_p4.hip — kernels.hpp instantiated for examples/ex_game
// with 4 players, one lane per player (ExGame<4, true>).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_exgame_p4_ops() {
#if RB_EXGAME_P2_ONLY  // kernel-experiment builds (tools/): the bench configuration only
  return nullptr;
#else
  return std::make_unique<GameOpsT<ExGame<4, true>>>();
#endif
}
}  // namespace rb
