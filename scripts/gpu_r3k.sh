#!/bin/bash
# Round 3: warp-specialized k_tconv_ws (MZGO_TCONV_WS=1) -- tower parity, then timing vs k_tconv.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MZGO_TCONV_WS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ws.log 2>&1 || { tail -40 gpurun_out/t_ws.log; exit 1; }
tail -2 gpurun_out/t_ws.log
for ws in 0 1 0 1; do
  MZGO_TCONV_WS=$ws timeout -k 10 300 python bench.py --config 5 --sims 128 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c5ws$ws.json 2>&1 || { tail -5 gpurun_out/c5ws$ws.json; exit 1; }
  echo "ws=$ws $(tail -1 gpurun_out/c5ws$ws.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,2), "us/conv", round(r["frac"],3))')"
done
MZGO_TCONV_WS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ws_trace -o run -- python3 bench.py --config 5 --sims 128 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ws_trace.log 2>&1 || { tail -5 gpurun_out/ws_trace.log; exit 1; }
grep -h "k_tconv" gpurun_out/ws_trace/run_kernel_stats.csv | cut -c1-200
