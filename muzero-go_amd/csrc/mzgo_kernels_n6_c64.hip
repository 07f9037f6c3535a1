// Kernel instantiations for play.py's configuration: 6x6 board, latent_dim
// 64 (play.py:16-19), used by the interactive agent (mzgo.play, search
// variant "main" with play.py's constants).
#include "mzgo_dispatch.hpp"

namespace mzgo {
extern const KernelSet kernels_n6_c64 = Launch<6, 64>::table();
}  // namespace mzgo
