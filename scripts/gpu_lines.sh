#!/bin/bash
# The bench lines quoted in DESIGN.md, each to profiles/<tag>_<line>.json:
#   bench (9x9/256/200, the headline, with cpu_baseline), 9_400, refill2,
#   19_64 (19x19/64/800), c5 (config 5 opening), c5mid (config 5 at move >= 100)
# Usage: TAG=r4a [LINES="bench 9_400 ..."] bash scripts/gpu_lines.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: "${TAG:?set TAG}"
declare -A A=(
  [bench]="--steps 20 --warmup 3 --cpu-budget 8"
  [9_400]="--sims 400 --steps 8 --warmup 1 --no-cpu-baseline"
  [refill2]="--refill 2 --steps 20 --warmup 2 --no-cpu-baseline"
  [19_64]="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline"
  [c5]="--config 5 --cpu-budget 20"
  [c5mid]="--config 5 --start-move 100 --cpu-budget 20"
)
for l in ${LINES:-bench 9_400 refill2 19_64 c5}; do
  timeout -k 10 ${LIMIT:-420} python bench.py ${A[$l]} > gpurun_out/${TAG}_$l.json 2> gpurun_out/${TAG}_$l.err || { tail -5 gpurun_out/${TAG}_$l.err; exit 1; }
  echo "$l $(tail -1 gpurun_out/${TAG}_$l.json | cut -c1-240)"
done
