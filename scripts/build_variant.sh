#!/bin/bash
# Non-diagnostic variant of libmzgo.so with extra -D flags:
#   VARIANT=name EXTRA="-DFOO=1" bash scripts/build_variant.sh
# -> muzero-go_amd/mzgo/libmzgo_<name>.so (load with MZGO_LIB=...)
set -e
cd "$(dirname "$0")/.."
B=muzero-go_amd/build_${VARIANT:?}
mkdir -p $B
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result $EXTRA"
for f in muzero-go_amd/csrc/*.hip; do /opt/rocm/bin/hipcc $FLAGS -c -o $B/$(basename ${f%.hip}).o $f & done
wait
/opt/rocm/bin/hipcc $FLAGS -shared -o muzero-go_amd/mzgo/libmzgo_${VARIANT}.so $B/*.o
