#!/bin/bash
# Round 3 final: full GPU suite, default bench line (cpu_baseline included), refill 2, 19x19/64/800, config 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -60 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2>&1 || { tail -5 gpurun_out/b_default.json; exit 1; }
echo "default $(tail -1 gpurun_out/b_default.json | cut -c1-300)"
timeout -k 10 200 python bench.py --steps 12 --refill 2 --no-cpu-baseline > gpurun_out/g9r2.json 2>&1 || { tail -5 gpurun_out/g9r2.json; exit 1; }
echo "refill2 $(tail -1 gpurun_out/g9r2.json | cut -c1-250)"
timeout -k 10 200 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --no-cpu-baseline > gpurun_out/g19.json 2>&1 || { tail -5 gpurun_out/g19.json; exit 1; }
echo "19x19 $(tail -1 gpurun_out/g19.json | cut -c1-250)"
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5.json 2>&1 || { tail -5 gpurun_out/c5.json; exit 1; }
echo "c5 $(tail -1 gpurun_out/c5.json | cut -c1-250)"
