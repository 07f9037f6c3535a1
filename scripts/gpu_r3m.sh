#!/bin/bash
# k_tconv_ks (K split across the two waves of a SIMD): tower parity with it, then config-5 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MZGO_TCONV_KS=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_tower.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tower_ks.log 2>&1 || { tail -30 gpurun_out/t_tower_ks.log; exit 1; }
tail -2 gpurun_out/t_tower_ks.log
for ks in 0 1 0 1; do
  MZGO_TCONV_KS=$ks timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5ks$ks.log 2>&1 || { tail -5 gpurun_out/c5ks$ks.log; exit 1; }
  echo "ks=$ks $(tail -1 gpurun_out/c5ks$ks.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,2), "us/conv", round(r["frac"],3))')"
done
