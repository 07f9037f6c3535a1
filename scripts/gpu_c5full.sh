#!/bin/bash
# BASELINE config 5 at full size (64 games x 1600 sims, C=256, 20 blocks): bench with
# cpu_baseline, then the k_tconv PMC passes on a short run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config 5 > gpurun_out/c5_full.log 2>&1 || { tail -20 gpurun_out/c5_full.log; exit 1; }
tail -1 gpurun_out/c5_full.log | cut -c1-400
bash scripts/pmc_tower.sh c5r2 || exit $?
