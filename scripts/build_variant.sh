#!/bin/bash
# Experimental build of libmzgo.so with extra defines (A/B of kernel knobs):
#   VARIANT=a3 EXTRA="-DMZGO_TCONV_ADIST=3" bash scripts/build_variant.sh
# -> muzero-go_amd/mzgo/libmzgo_a3.so, loaded with MZGO_LIB=... (bench / tests).
set -e
cd "$(dirname "$0")/.."
: "${VARIANT:?set VARIANT}"
B=muzero-go_amd/build_$VARIANT
mkdir -p $B
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result ${EXTRA:-}"
KFLAGS="-mllvm -disable-machine-licm -mllvm -disable-machine-sink"   # the megakernels (see __graft_entry__.py)
ls muzero-go_amd/csrc/*.hip | xargs -P 8 -I{} sh -c "case {} in *mzgo_kernels_n*) K=\"$KFLAGS\";; *) K=;; esac; /opt/rocm/bin/hipcc $FLAGS \$K -c -o $B/\$(basename {} .hip).o {}"
/opt/rocm/bin/hipcc $FLAGS -shared -o muzero-go_amd/mzgo/libmzgo_$VARIANT.so $B/*.o
