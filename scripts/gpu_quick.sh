#!/bin/bash
# Search/self-play/bench-size parity, then the 9x9 headline and 19x19/64/800 whole-game lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_bench_parity.py tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_quick.log 2>&1 || { tail -40 gpurun_out/t_quick.log; exit 1; }
tail -1 gpurun_out/t_quick.log
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/q9.json 2>&1 || { tail -5 gpurun_out/q9.json; exit 1; }
echo "9x9 $(tail -1 gpurun_out/q9.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M sims/s", round(d["ms_per_step"],1), "ms/epoch")')"
timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/q19.json 2>&1 || { tail -5 gpurun_out/q19.json; exit 1; }
echo "19x19 $(tail -1 gpurun_out/q19.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M sims/s", round(d["ms_per_step"]), "ms/epoch")')"
