// Kernel instantiations for the 9x9 board (latent_dim 96, the reference's
// self_play.py:21).  One translation unit per board size keeps builds parallel.
#include "mzgo_dispatch.hpp"

namespace mzgo {
extern const KernelSet kernels_n9_c96 = Launch<9, 96>::table();
}  // namespace mzgo
