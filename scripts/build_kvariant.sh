#!/bin/bash
# Fast experimental build of the 9x9 megakernel knobs: only mzgo_kernels_n9.hip and mzgo_capi.hip (the
# host packing follows MZGO_WINO_XG) get EXTRA defines, the rest reuse muzero-go_amd/build/*.o.
#   VARIANT=pf10 EXTRA="-DMZGO_WINO_PF=10" bash scripts/build_kvariant.sh
set -e
cd "$(dirname "$0")/.."
: "${VARIANT:?set VARIANT}"
B=muzero-go_amd/build_$VARIANT
mkdir -p $B
cp muzero-go_amd/build/*.o $B/
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result ${EXTRA:-}"
KFLAGS="-mllvm -disable-machine-licm -mllvm -disable-machine-sink"
/opt/rocm/bin/hipcc $FLAGS $KFLAGS -c -o $B/mzgo_kernels_n9.o muzero-go_amd/csrc/mzgo_kernels_n9.hip &
/opt/rocm/bin/hipcc $FLAGS -c -o $B/mzgo_capi.o muzero-go_amd/csrc/mzgo_capi.hip &
wait
/opt/rocm/bin/hipcc $FLAGS -shared -o muzero-go_amd/mzgo/libmzgo_$VARIANT.so $B/*.o
