#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py -x -v --timeout 600 --timeout-method thread > gpurun_out/t_bp.log 2>&1; rc=$?
tail -6 gpurun_out/t_bp.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_bench_parity.py > gpurun_out/t_all.log 2>&1; rc=$?
tail -4 gpurun_out/t_all.log
exit $rc
