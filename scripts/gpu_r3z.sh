#!/bin/bash
# headline PMC passes on the scratch-free k_selfplay_move, then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_selfplay.sh r3n || exit 1
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2>&1 || { tail -5 gpurun_out/b_default.json; exit 1; }
echo "default $(tail -1 gpurun_out/b_default.json | cut -c1-300)"
