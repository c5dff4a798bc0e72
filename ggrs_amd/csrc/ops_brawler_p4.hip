// ggrs_amd/csrc/ops_brawler_p4.hip — kernels.hpp instantiated for the brawler with
// 4 players (Brawler<4>, one wave per session).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_brawler_p4_ops() { return std::make_unique<GameOpsT<Brawler<4>>>(); }
}  // namespace rb
