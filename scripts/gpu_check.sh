#!/bin/bash
# GPU-box check used during development: GPU parity tests, smoke, a short bench.
# Every GPU step has its own time limit; after a fault/abort/timeout nothing
# else touches the GPU (test failures, rc=1, do not stop the chain).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n 3 "gpurun_out/$name.log"
  return $rc
}
run pytest_gpu 1100 python -m pytest tests -m gpu -q -rf --durations=15
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 400 python bench.py --steps 10 --warmup 2 --cpu-budget 8 || exit $?
cat gpurun_out/bench.log
