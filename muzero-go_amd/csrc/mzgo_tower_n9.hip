// Residual-tower engine (BASELINE config 5, mzgo_tower.hpp) for the 9x9 board.
#include "mzgo_tower_dispatch.hpp"

namespace mzgo {
extern const TowerSet tower_n9 = TLaunch<9>::table();
}  // namespace mzgo
