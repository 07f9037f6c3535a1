#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (k_selfplay_move):
#   1) --kernel-trace --stats          -> per-kernel durations
#   2) --pmc FETCH_SIZE  (own pass)    -> HBM read bytes
#   3) --pmc WRITE_SIZE  (own pass)    -> HBM write bytes
# Usage: bash scripts/profile.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r1}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=${*:-"--steps 6 --warmup 1 --no-cpu-baseline"}
step() {
  local name=$1; shift
  timeout -k 10 500 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log"
  return $rc
}
step trace rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS || exit $?
step fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS || exit $?
step write rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS || exit $?
find "$OUT" -name "*.csv" | head -20
