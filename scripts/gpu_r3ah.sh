#!/bin/bash
# 9x9 / 256 / 400 whole games with the current kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --sims 400 --steps 6 --no-cpu-baseline > gpurun_out/g9_400.json 2>&1 || { tail -5 gpurun_out/g9_400.json; exit 1; }
echo "9x9/400 $(tail -1 gpurun_out/g9_400.json | cut -c1-220)"
