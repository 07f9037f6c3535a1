#!/bin/bash
# k_tconv change: tower parity on the default library, then config-5 A/B
# against LIBS (e.g. _old) at 256 sims.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tower.log 2>&1 || { tail -30 gpurun_out/t_tower.log; exit 1; }
tail -2 gpurun_out/t_tower.log
NWS="8" LIBS="- ${LIBS:-}" bash scripts/gpu_c5grid.sh
