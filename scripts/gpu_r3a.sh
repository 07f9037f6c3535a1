#!/bin/bash
# Round 3, first call: config-5 depth errors, the new config-5 and whole-game-launch tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/c5_depth_errors.py > gpurun_out/c5_depth.jsonl 2> gpurun_out/c5_depth.err || { tail -20 gpurun_out/c5_depth.err; exit 1; }
cat gpurun_out/c5_depth.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_tower.py::test_tower_search_matches_oracle_tree" \
  "tests/test_gpu_tower.py::test_tower_config5_full_move" \
  "tests/test_gpu_bench_parity.py::test_whole_game_launch_equals_per_move_launches" \
  > gpurun_out/t_r3a.log 2>&1 || { tail -60 gpurun_out/t_r3a.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/t_r3a.log
