#!/bin/bash
# Diagnostic variant of libmzgo.so with per-phase s_memtime stamps
# (-DMZGO_STAMPS).  Load it with MZGO_LIB=muzero-go_amd/mzgo/libmzgo_${VARIANT:-stamps}.so.
set -e
cd "$(dirname "$0")/.."
B=muzero-go_amd/build_${VARIANT:-stamps}
mkdir -p $B
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -DMZGO_STAMPS ${EXTRA:-}"
ls muzero-go_amd/csrc/*.hip | xargs -P 8 -I{} sh -c "/opt/rocm/bin/hipcc $FLAGS -c -o $B/\$(basename {} .hip).o {}"
/opt/rocm/bin/hipcc $FLAGS -shared -o muzero-go_amd/mzgo/libmzgo_${VARIANT:-stamps}.so $B/*.o
