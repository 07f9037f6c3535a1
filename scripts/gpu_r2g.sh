#!/bin/bash
# Round-2 refresh: the whole GPU suite, the default bench line, PMC passes of it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 400 python bench.py > gpurun_out/b_r2g.json 2>&1 || { tail -5 gpurun_out/b_r2g.json; exit 1; }
tail -1 gpurun_out/b_r2g.json | cut -c1-400
bash scripts/pmc_selfplay.sh r2g || exit $?
