// Kernel instantiations for the 6x6 board (latent_dim 96, the reference's
// self_play.py:21).  One translation unit per board size keeps builds parallel.
#include "mzgo_dispatch.hpp"

namespace mzgo {
extern const KernelSet kernels_n6_c96 = Launch<6, 96>::table();
}  // namespace mzgo
