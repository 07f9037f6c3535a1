#!/bin/bash
# BASELINE config 5 (tower engine): short bench, full bench, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config 5 --sims 64 --steps 2 --no-cpu-baseline > gpurun_out/c5_s64.log 2>&1 || { tail -20 gpurun_out/c5_s64.log; exit 1; }
tail -1 gpurun_out/c5_s64.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --sims 64 --steps 1 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5_full.log 2>&1 || { tail -20 gpurun_out/c5_full.log; exit 1; }
tail -1 gpurun_out/c5_full.log | cut -c1-300
