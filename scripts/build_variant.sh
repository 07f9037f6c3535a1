#!/bin/bash
# Diagnostic / A-B build of libmzgo.so with extra defines.  Always compiled
# with -DMZGO_DIAG_BUILD (the wrong-result switches of mzgo_diag.hpp compile
# only there); never the product library.
#   VARIANT=a3 EXTRA="-DMZGO_TCONV_KS_ADIST=3" [SCOPE=all|tower|n9|n19] bash scripts/build_variant.sh
# -> muzero-go_amd/mzgo/libmzgo_a3.so, loaded with MZGO_LIB=... (bench / tests).
# SCOPE=tower / n9 / n19: only the tower units / the 9x9 megakernel + C API /
# the 19x19 megakernel get EXTRA,
# the rest reuse muzero-go_amd/build/*.o (run __graft_entry__.build() first).
set -e
cd "$(dirname "$0")/.."
: "${VARIANT:?set VARIANT}"
B=muzero-go_amd/build_$VARIANT
mkdir -p $B
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -DMZGO_DIAG_BUILD ${EXTRA:-}"
KFLAGS="-mllvm -disable-machine-licm -mllvm -disable-machine-sink"   # the megakernels (see __graft_entry__.py)
case "${SCOPE:-all}" in
  all) SRCS=$(ls muzero-go_amd/csrc/*.hip) ;;
  tower) cp muzero-go_amd/build/*.o $B/; SRCS=$(ls muzero-go_amd/csrc/mzgo_tower_*.hip) ;;
  n9) cp muzero-go_amd/build/*.o $B/; SRCS="muzero-go_amd/csrc/mzgo_kernels_n9.hip muzero-go_amd/csrc/mzgo_capi.hip" ;;
  n19) cp muzero-go_amd/build/*.o $B/; SRCS="muzero-go_amd/csrc/mzgo_kernels_n19.hip" ;;
  *) echo "SCOPE must be all, tower, n9 or n19" >&2; exit 2 ;;
esac
echo $SRCS | tr ' ' '\n' | xargs -P 8 -I{} sh -c "case {} in *mzgo_kernels_n*) K=\"$KFLAGS\";; *) K=;; esac; /opt/rocm/bin/hipcc $FLAGS \$K -c -o $B/\$(basename {} .hip).o {}"
/opt/rocm/bin/hipcc $FLAGS -shared -o muzero-go_amd/mzgo/libmzgo_$VARIANT.so $B/*.o
