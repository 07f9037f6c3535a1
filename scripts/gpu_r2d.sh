#!/bin/bash
# Round-2: whole-game launches -- equality test, A/B bench, configs, PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_selfplay.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_sp.log 2>&1 || { tail -30 gpurun_out/t_sp.log; exit 1; }
tail -3 gpurun_out/t_sp.log
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/b_whole.log 2>&1 || exit $?
tail -1 gpurun_out/b_whole.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --moves-per-launch 1 > gpurun_out/b_permove.log 2>&1 || exit $?
tail -1 gpurun_out/b_permove.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --sims 400 --no-cpu-baseline > gpurun_out/b_9_400.log 2>&1 || exit $?
tail -1 gpurun_out/b_9_400.log | cut -c1-300
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --board-size 19 --games 64 --sims 800 --no-cpu-baseline > gpurun_out/b_19_64.log 2>&1 || exit $?
tail -1 gpurun_out/b_19_64.log | cut -c1-300
bash scripts/pmc_selfplay.sh r2d || exit $?
