// Kernel instantiations for main.py's training configuration: 6x6 board,
// latent_dim 128 (main.py:27-30), used by its self-play and arena evaluator
// (search_variant "main").
#include "mzgo_dispatch.hpp"

namespace mzgo {
extern const KernelSet kernels_n6_c128 = Launch<6, 128>::table();
}  // namespace mzgo
