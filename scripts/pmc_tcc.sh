#!/bin/bash
# L2 / memory-side request counters of a bench.py line's k_selfplay_move,
# split by request size, one pass per counter group (<= 4 TCC per pass,
# MI355X_MICROARCH.md); the program directly after "--".
#   rd  : TCC_EA0_RDREQ (all), _32B, TCC_BUBBLE (128 B), _DRAM
#   wr  : TCC_EA0_WRREQ (all), _64B, _DRAM
#   l2  : TCC_HIT, TCC_MISS, TCC_READ, TCC_WRITE
# Usage: bash scripts/pmc_tcc.sh <tag> [bench args...]; then python scripts/summarize_tcc.py <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/tcc_$TAG
mkdir -p "$OUT"
ARGS=${*:-"--steps 1 --warmup 1 --no-cpu-baseline"}
pass() {
  local name=$1; shift
  timeout -s KILL 240 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 1 "$OUT/$name.log"
  return $rc
}
pass trace rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS || exit 1
pass rd rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d "$OUT/rd" -o run -- python3 bench.py $ARGS || exit 1
pass wr rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d "$OUT/wr" -o run -- python3 bench.py $ARGS || exit 1
pass l2 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_WRITE_sum --output-format csv -d "$OUT/l2" -o run -- python3 bench.py $ARGS || exit 1
