// Residual-tower engine (BASELINE config 5, mzgo_tower.hpp) for the 19x19 board.
#include "mzgo_tower_dispatch.hpp"

namespace mzgo {
extern const TowerSet tower_n19 = TLaunch<19>::table();
}  // namespace mzgo
