// ggrs_amd/csrc/ops_exgame_p2.hip — kernels.hpp instantiated for examples/ex_game
// with 2 players, one lane per player (ExGame<2, true>).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_exgame_p2_ops() {
  return std::make_unique<GameOpsT<ExGame<2, true>>>();
}
}  // namespace rb
