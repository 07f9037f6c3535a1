#!/bin/bash
# rocprofv3 trace + PMC passes of config 5 with k_tconv_ks (default), then in-kernel clocks (stamps build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_tower.sh c5r3m || exit 1
for ks in 1 0; do
  MZGO_TCONV_KS=$ks MZGO_LIB=muzero-go_amd/mzgo/libmzgo_ts.so timeout -k 10 300 python scripts/tconv_stamps.py > gpurun_out/ts_k$ks.log 2>&1 || { tail -5 gpurun_out/ts_k$ks.log; exit 1; }
  echo "== ks=$ks"; grep -v amdgpu.ids gpurun_out/ts_k$ks.log | head -3
done
