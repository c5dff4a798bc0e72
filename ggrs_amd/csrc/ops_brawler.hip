// ggrs_amd/csrc/ops_brawler.hip — device code of the fixed-point 256-entity
// brawler (BASELINE config 3): the factory.  Each player count instantiates
// kernels.hpp for Brawler<P> in a translation unit of its own
// (ops_brawler_p<P>.hip), so they compile in parallel.
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_brawler_p1_ops();
std::unique_ptr<GameOps> make_brawler_p2_ops();
std::unique_ptr<GameOps> make_brawler_p3_ops();
std::unique_ptr<GameOps> make_brawler_p4_ops();
std::unique_ptr<GameOps> make_brawler_ops(int players) {
  switch (players) {
    case 1: return make_brawler_p1_ops();
    case 2: return make_brawler_p2_ops();
    case 3: return make_brawler_p3_ops();
    case 4: return make_brawler_p4_ops();
    default: return nullptr;
  }
}
}  // namespace rb
