#!/bin/bash
# Round 3: whole-game vs per-move determinism diagnostics (19x19 helpers), 9x9 game stamps, quick bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_wholegame.py > gpurun_out/diag_wg.json 2> gpurun_out/diag_wg.err || { tail -20 gpurun_out/diag_wg.err; exit 1; }
cat gpurun_out/diag_wg.json
OUT=stamps9_r3 bash scripts/gpu_stamps9.sh || exit 1
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/q9.json 2>&1 || { tail -5 gpurun_out/q9.json; exit 1; }
tail -1 gpurun_out/q9.json | cut -c1-400
