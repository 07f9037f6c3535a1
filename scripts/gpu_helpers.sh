#!/bin/bash
# 19x19 helper workgroups: parity (search/self-play/bench-size), then the
# 19x19 / 64 / 800 whole-game bench with 0 and 3 helpers per game.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_bench_parity.py tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_helpers.log 2>&1 || { tail -40 gpurun_out/t_helpers.log; exit 1; }
tail -2 gpurun_out/t_helpers.log
for h in ${HELPERS:-0 3}; do
  MZGO_HELPERS_PER_GAME=$h timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b19_h$h.json 2>&1 || { tail -5 gpurun_out/b19_h$h.json; exit 1; }
  echo "helpers/game=$h $(tail -1 gpurun_out/b19_h$h.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M sims/s", round(d["ms_per_step"]), "ms/epoch")')"
done
