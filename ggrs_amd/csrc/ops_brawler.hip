// ggrs_amd/csrc/ops_brawler.hip — device code of the fixed-point 256-entity
// brawler (BASELINE config 3; kernels.hpp instantiated for Brawler<P>).
#include "kernels.hpp"

namespace rb {
std::unique_ptr<GameOps> make_brawler_ops(int players) {
  switch (players) {
    case 1: return std::make_unique<GameOpsT<Brawler<1>>>();
    case 2: return std::make_unique<GameOpsT<Brawler<2>>>();
    case 3: return std::make_unique<GameOpsT<Brawler<3>>>();
    case 4: return std::make_unique<GameOpsT<Brawler<4>>>();
    default: return nullptr;
  }
}
}  // namespace rb
