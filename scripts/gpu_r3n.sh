#!/bin/bash
# k_tconv vs k_tconv_ks phase stamps (diagnostic build libmzgo_ts.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for ks in 0 1; do
  echo "== ks=$ks"
  MZGO_TCONV_KS=$ks MZGO_LIB=muzero-go_amd/mzgo/libmzgo_ts.so timeout -k 10 300 python scripts/tconv_stamps.py > gpurun_out/ts_ks$ks.log 2>&1 || { tail -5 gpurun_out/ts_ks$ks.log; exit 1; }
  cat gpurun_out/ts_ks$ks.log
done
