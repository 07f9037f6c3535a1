#!/bin/bash
# config 5 with tower timing sampled every 16th simulation: A/B (the old library with the new bench.py
# times every tower), tower tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tower.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_tower.log 2>&1 || { tail -40 gpurun_out/t_tower.log; exit 1; }
tail -2 gpurun_out/t_tower.log
for v in _old "" _old ""; do
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5v.log 2>&1 || { tail -5 gpurun_out/c5v.log; exit 1; }
  echo "lib$v $(tail -1 gpurun_out/c5v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,2), "us/conv", round(r["boards_per_launch"],1), "boards", round(r["frac"],3))')"
done
