#!/bin/bash
# Fast experimental build: only the tower translation units get EXTRA defines,
# the rest reuse muzero-go_amd/build/*.o (run __graft_entry__.build() first).
#   VARIANT=p1 EXTRA="-DMZGO_TCONV_PRIO=1" bash scripts/build_tvariant.sh
set -e
cd "$(dirname "$0")/.."
: "${VARIANT:?set VARIANT}"
B=muzero-go_amd/build_$VARIANT
mkdir -p $B
cp muzero-go_amd/build/*.o $B/
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result ${EXTRA:-}"
ls muzero-go_amd/csrc/mzgo_tower_*.hip | xargs -P 4 -I{} sh -c "/opt/rocm/bin/hipcc $FLAGS -c -o $B/\$(basename {} .hip).o {}"
/opt/rocm/bin/hipcc $FLAGS -shared -o muzero-go_amd/mzgo/libmzgo_$VARIANT.so $B/*.o
