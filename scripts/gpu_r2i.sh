#!/bin/bash
# Round-2 re-entry check: the whole GPU suite, the default bench line, a short
# config-5 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/b_r2i.json 2>&1 || { tail -5 gpurun_out/b_r2i.json; exit 1; }
tail -1 gpurun_out/b_r2i.json | cut -c1-300
timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5_r2i.json 2>&1 || { tail -5 gpurun_out/c5_r2i.json; exit 1; }
tail -1 gpurun_out/c5_r2i.json | cut -c1-300
