#!/bin/bash
# Round-2 GPU check: the new parity tests, the whole-game bench, PMC passes of
# k_selfplay_move, then the whole -m gpu suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_search.py::test_sampled_dirichlet_statistics tests/test_gpu_selfplay.py::test_sharded_engines_equal_single_engine -x -v --timeout 600 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?
tail -12 gpurun_out/t_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_epoch.log 2>&1 || exit $?
tail -1 gpurun_out/b_epoch.log | cut -c1-600
bash scripts/pmc_selfplay.sh r2a || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -3 gpurun_out/t_all.log
exit $rc
