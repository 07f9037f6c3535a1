#!/bin/bash
# Residual-tower engine (config 5): parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -v --timeout 300 --timeout-method thread > gpurun_out/t_tower.log 2>&1; rc=$?
tail -40 gpurun_out/t_tower.log
exit $rc
