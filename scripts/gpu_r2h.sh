#!/bin/bash
# Round-2 final refresh: the whole GPU suite, the default bench line, the
# 9x9/400 and 19x19/64/800 lines, PMC passes of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 400 python bench.py > gpurun_out/b_r2h.json 2>&1 || { tail -5 gpurun_out/b_r2h.json; exit 1; }
tail -1 gpurun_out/b_r2h.json | cut -c1-300
timeout -k 10 300 python bench.py --sims 400 --steps 3 --no-cpu-baseline > gpurun_out/b_r2h_9_400.json 2>&1 || { tail -5 gpurun_out/b_r2h_9_400.json; exit 1; }
tail -1 gpurun_out/b_r2h_9_400.json | cut -c1-200
timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_r2h_19_64.json 2>&1 || { tail -5 gpurun_out/b_r2h_19_64.json; exit 1; }
tail -1 gpurun_out/b_r2h_19_64.json | cut -c1-200
bash scripts/pmc_selfplay.sh r2h || exit $?
