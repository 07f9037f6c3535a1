#!/bin/bash
# k_tconv A/B: 8 waves (default) vs 4 waves; parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -q --timeout 300 --timeout-method thread > gpurun_out/t_tower.log 2>&1 || { tail -30 gpurun_out/t_tower.log; exit 1; }
tail -2 gpurun_out/t_tower.log
for nw in 8 4 8; do
  MZGO_TCONV_WAVES=$nw timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5_nw$nw.log 2>&1 || exit $?
  echo "nw=$nw $(tail -1 gpurun_out/c5_nw$nw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,1), "us/conv", round(r["frac"],3))')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5b -o run -- python3 bench.py --config 5 --sims 64 --steps 1 --no-cpu-baseline > gpurun_out/prof_c5b.log 2>&1 || exit $?
head -3 gpurun_out/prof_c5b/run_kernel_stats.csv | cut -c1-150
