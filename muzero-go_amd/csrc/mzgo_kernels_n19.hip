// Kernel instantiations for the 19x19 board (latent_dim 96, the reference's
// self_play.py:21).  One translation unit per board size keeps builds parallel.
#include "mzgo_dispatch.hpp"

namespace mzgo {
extern const KernelSet kernels_n19_c96 = Launch<19, 96>::table();
}  // namespace mzgo
