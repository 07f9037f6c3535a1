#!/bin/bash
# Round 3 close: headline PMC passes, default bench line (cpu_baseline included), refill 2, 19x19/64/800,
# config 5, and the stamps-build phases of the current kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_selfplay.sh r3r > gpurun_out/pmc_r3r.log 2>&1 || { tail -20 gpurun_out/pmc_r3r.log; exit 1; }
echo pmc ok
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python scripts/phases.py r3r > gpurun_out/phases_r3r.log 2>&1 || { tail -5 gpurun_out/phases_r3r.log; exit 1; }
echo phases ok
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2>&1 || { tail -5 gpurun_out/b_default.json; exit 1; }
echo "default $(tail -1 gpurun_out/b_default.json | cut -c1-200)"
timeout -k 10 200 python bench.py --steps 12 --refill 2 --no-cpu-baseline > gpurun_out/g9r2.json 2>&1 || { tail -5 gpurun_out/g9r2.json; exit 1; }
echo "refill2 $(tail -1 gpurun_out/g9r2.json | cut -c1-200)"
timeout -k 10 200 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --no-cpu-baseline > gpurun_out/g19.json 2>&1 || { tail -5 gpurun_out/g19.json; exit 1; }
echo "19x19 $(tail -1 gpurun_out/g19.json | cut -c1-200)"
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5.json 2>&1 || { tail -5 gpurun_out/c5.json; exit 1; }
echo "c5 $(tail -1 gpurun_out/c5.json | cut -c1-200)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
