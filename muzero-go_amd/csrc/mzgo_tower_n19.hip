// Residual-tower engine (BASELINE config 5, mzgo_tower.hpp) for the 19x19 board.
#include "mzgo_tower_dispatch.hpp"

namespace mzgo {
extern const TowerSet tower_n19 = TLaunch<19>::table();
#ifdef MZGO_TCONV_STAMPS
int tower_stamps_n19(unsigned long long* out) {
  // out[wave * 16 + field], summed over blocks
  static unsigned long long h[4096][8][16];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_tstamps), sizeof h) != hipSuccess) return -2;
  for (int k = 0; k < 128; ++k) out[k] = 0;
  for (int i = 0; i < 4096; ++i)
    for (int k = 0; k < 128; ++k) out[k] += h[i][k >> 4][k & 15];
  static unsigned long long z[4096][8][16];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tstamps), z, sizeof z) == hipSuccess ? 0 : -2;
}
#endif
}  // namespace mzgo
