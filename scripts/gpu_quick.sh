#!/bin/bash
# Development loop on the GPU box: search/self-play parity tests, the bench in
# both dynamics modes, and the per-phase stamp breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_selfplay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_quick.log 2>&1; rc=$?
tail -5 gpurun_out/t_quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_fact.log 2>&1 || exit $?
tail -1 gpurun_out/b_fact.log | cut -c1-400
STAMPS=1 MZGO_LIB=muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 200 python scripts/microbench.py || exit $?
