// ggrs_amd/csrc/ops_brawler_p1.hip — kernels.hpp instantiated for the brawler with
// 1 player (Brawler<1>, one wave per session).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_brawler_p1_ops() { return std::make_unique<GameOpsT<Brawler<1>>>(); }
}  // namespace rb
