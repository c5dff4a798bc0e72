// ggrs_amd/csrc/ops_brawler_p2.hip — kernels.hpp instantiated for the brawler with
// 2 players (Brawler<2>, one wave per session).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_brawler_p2_ops() { return std::make_unique<GameOpsT<Brawler<2>>>(); }
}  // namespace rb
