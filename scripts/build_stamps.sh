#!/bin/bash
# Diagnostic variant of libmzgo.so with per-phase s_memtime stamps
# (-DMZGO_STAMPS).  Load it with MZGO_LIB=muzero-go_amd/mzgo/libmzgo_${VARIANT:-stamps}.so.
set -e
cd "$(dirname "$0")/.."
B=muzero-go_amd/build_${VARIANT:-stamps}
mkdir -p $B
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -DMZGO_STAMPS ${EXTRA:-}"
KFLAGS="-mllvm -disable-machine-licm -mllvm -disable-machine-sink"   # the megakernels (see __graft_entry__.py)
ls muzero-go_amd/csrc/*.hip | xargs -P 8 -I{} sh -c "case {} in *mzgo_kernels_n*) K=\"$KFLAGS\";; *) K=;; esac; /opt/rocm/bin/hipcc $FLAGS \$K -c -o $B/\$(basename {} .hip).o {}"
/opt/rocm/bin/hipcc $FLAGS -shared -o muzero-go_amd/mzgo/libmzgo_${VARIANT:-stamps}.so $B/*.o
