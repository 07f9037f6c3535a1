#!/bin/bash
# Round-2 close after the k_tconv epilogue change: GPU suite, default bench,
# config-5 full bench + its rocprofv3 trace / PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 400 python bench.py > gpurun_out/b_${TAG:-r2i}.json 2>&1 || { tail -5 gpurun_out/b_${TAG:-r2i}.json; exit 1; }
tail -1 gpurun_out/b_${TAG:-r2i}.json | cut -c1-200
timeout -k 10 600 python bench.py --config 5 > gpurun_out/c5_${TAG:-r2i}.json 2>&1 || { tail -20 gpurun_out/c5_${TAG:-r2i}.json; exit 1; }
tail -1 gpurun_out/c5_${TAG:-r2i}.json | cut -c1-300
bash scripts/pmc_tower.sh ${TAG:-c5r2i} || exit $?
