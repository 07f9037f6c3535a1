#!/bin/bash
# Round 3: rocprofv3 kernel trace + PMC passes of the 9x9 headline and of 19x19 / 64 / 800.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_selfplay.sh r3 || exit $?
bash scripts/pmc_selfplay.sh r3_19 --board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline || exit $?
