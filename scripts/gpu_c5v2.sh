#!/bin/bash
# k_tconv2 (two workgroups per CU, MZGO_TCONV_V2=1) vs k_tconv: tower parity with each, then the config-5 bench (256 sims) both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0; do
  MZGO_TCONV_V2=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -q --timeout 300 --timeout-method thread > gpurun_out/t_tower$v.log 2>&1 || { tail -30 gpurun_out/t_tower$v.log; exit 1; }
  echo "v2=$v $(tail -1 gpurun_out/t_tower$v.log)"
done
for v in 1 0; do
  MZGO_TCONV_V2=$v timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5_v$v.log 2>&1 || { tail -5 gpurun_out/c5_v$v.log; exit 1; }
  echo "v2=$v $(tail -1 gpurun_out/c5_v$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,1), "us/conv", round(r["frac"],3))')"
done
