// Residual-tower engine (BASELINE config 5, mzgo_tower.hpp) for the 5x5 board.
#include "mzgo_tower_dispatch.hpp"

namespace mzgo {
extern const TowerSet tower_n5 = TLaunch<5>::table();
}  // namespace mzgo
