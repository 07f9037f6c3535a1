#!/bin/bash
# rocprofv3 evidence for a bench.py line's dominant kernel (k_selfplay_move;
# k_tconv_ks with --config 5), one counter group per pass (MI355X_MICROARCH.md: <= 8 SQ, <= 4 TCC, <= 2 GRBM),
# the program directly after "--":
#   trace : --kernel-trace --stats  (per-kernel durations)
#   p1    : VALU / MFMA / LDS instruction counts and busy cycles
#   p2    : LDS bank conflicts, wait states
#   fetch : FETCH_SIZE (own pass), write : WRITE_SIZE (own pass)
# Usage: bash scripts/pmc.sh <tag> [bench args...]
# then:  python scripts/summarize_pmc.py <tag> [workload] [dynamics] [kernel] [moves/launch] [latest file]
#   (config 5: ... <tag> 19x19/C256/B20/G64 tower k_tconv_ks 0 latest_tower_pmc.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2}; shift || true
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
ARGS=${*:-"--steps 1 --warmup 1 --no-cpu-baseline"}
pass() {
  local name=$1; shift
  timeout -s KILL 240 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log"
  return $rc
}
pass trace rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS || exit 1
pass p1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o run -- python3 bench.py $ARGS || exit 1
pass p2 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 bench.py $ARGS || exit 1
pass fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS || exit 1
pass write rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS || exit 1
find "$OUT" -name "*.csv" | sort
