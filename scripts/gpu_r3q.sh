#!/bin/bash
# k_tconv_ks: DMA spread over the MFMA groups (s1/s2/s3), stamps with and without DMA
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MZGO_TCONV_KS=1
for v in "" _s1 _s2 _s3 ""; do
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5v$v.log 2>&1 || { tail -5 gpurun_out/c5v$v.log; exit 1; }
  echo "lib$v $(tail -1 gpurun_out/c5v$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,2), "us/conv", round(r["frac"],3))')"
done
for v in _tsnd; do
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python scripts/tconv_stamps.py > gpurun_out/ts$v.log 2>&1 || { tail -5 gpurun_out/ts$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/ts$v.log
done
