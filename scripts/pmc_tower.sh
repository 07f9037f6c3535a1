#!/bin/bash
# rocprofv3 evidence for config 5's dominant kernel (k_tconv): kernel trace,
# then one counter group per pass (<= 8 SQ, <= 4 TCC, <= 2 GRBM), the
# program directly after "--".
# Usage: bash scripts/pmc_tower.sh <tag> [bench args...]
# then:  python scripts/summarize_pmc.py <tag> 19x19/C256/B20/G64 tower k_tconv 0 latest_tower_pmc.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-t}; shift || true
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
ARGS=${*:-"--config 5 --sims 64 --steps 1 --warmup 1 --no-cpu-baseline"}
pass() {
  local name=$1; shift
  timeout -s KILL 240 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-200
  return $rc
}
pass trace rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS || exit 1
pass p1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o run -- python3 bench.py $ARGS || exit 1
pass p2 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 bench.py $ARGS || exit 1
pass fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS || exit 1
pass write rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS || exit 1
