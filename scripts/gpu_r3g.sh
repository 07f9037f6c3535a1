#!/bin/bash
# Round 3: full GPU suite, then 9x9 headline, 19x19/64/800, refill 2 and 3, determinism of the helper path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -60 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
RUNS=3 timeout -k 10 200 python -u scripts/diag_det.py || exit 1
timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/g9.json 2>&1 || { tail -5 gpurun_out/g9.json; exit 1; }
echo "9x9 $(tail -1 gpurun_out/g9.json | cut -c1-250)"
for r in 2 3; do
timeout -k 10 200 python bench.py --steps 12 --refill $r --no-cpu-baseline > gpurun_out/g9r$r.json 2>&1 || { tail -5 gpurun_out/g9r$r.json; exit 1; }
echo "9x9 refill $r $(tail -1 gpurun_out/g9r$r.json | cut -c1-250)"
done
timeout -k 10 200 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --no-cpu-baseline > gpurun_out/g19.json 2>&1 || { tail -5 gpurun_out/g19.json; exit 1; }
echo "19x19 $(tail -1 gpurun_out/g19.json | cut -c1-250)"
