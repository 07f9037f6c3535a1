#!/bin/bash
# Round-2: default whole-game bench (with cpu_baseline), then the 9x9/400 and
# 19x19/64/800 per-GPU shares as whole games, and a kernel-trace of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/b_default.log 2>&1 || exit $?
tail -1 gpurun_out/b_default.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --sims 400 --no-cpu-baseline > gpurun_out/b_9_400.log 2>&1 || exit $?
tail -1 gpurun_out/b_9_400.log | cut -c1-300
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --board-size 19 --games 64 --sims 800 --no-cpu-baseline > gpurun_out/b_19_64.log 2>&1 || exit $?
tail -1 gpurun_out/b_19_64.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2c -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r2c.log 2>&1 || exit $?
tail -1 gpurun_out/prof_r2c.log | cut -c1-300
