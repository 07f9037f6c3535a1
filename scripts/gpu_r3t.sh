#!/bin/bash
# in-kernel clock of k_tconv vs k_tconv_ks (stamps build with s_memrealtime)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for ks in 0 1 0 1; do
  MZGO_TCONV_KS=$ks MZGO_LIB=muzero-go_amd/mzgo/libmzgo_tss1.so timeout -k 10 300 python scripts/tconv_stamps.py > gpurun_out/ts_k$ks.log 2>&1 || { tail -5 gpurun_out/ts_k$ks.log; exit 1; }
  echo "== ks=$ks"; cat gpurun_out/ts_k$ks.log
done
