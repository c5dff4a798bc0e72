// ggrs_amd/csrc/ops_brawler_p3.hip — kernels.hpp instantiated for the brawler with
// 3 players (Brawler<3>, one wave per session).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_brawler_p3_ops() { return std::make_unique<GameOpsT<Brawler<3>>>(); }
}  // namespace rb
