// ggrs_amd/csrc/ops_stub.hip — device code of the integer stub games of
// tests/stubs.rs and tests/stubs_enum.rs (kernels.hpp instantiated per stub).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_stub_ops(int game, int players) {
  if (players != 2) return nullptr;  // the stubs sum exactly two inputs (stubs.rs:114-118)
  switch (game) {
    case RB_GAME_STUB: return std::make_unique<GameOpsT<StubGame>>();
    case RB_GAME_STUB_ENUM: return std::make_unique<GameOpsT<StubEnumGame>>();
    case RB_GAME_STUB_RANDOM_CS: return std::make_unique<GameOpsT<StubRandomCsGame>>();
    default: return nullptr;
  }
}
}  // namespace rb
