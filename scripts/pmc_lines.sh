#!/bin/bash
# Counter evidence (scripts/pmc.sh passes) for every bench line DESIGN.md
# quotes, each summarised into profiles/<TAG>_<line>_pmc.json and the
# profiles/latest_pmc*.json file bench.py attaches to that line:
#   head (9x9/256/200), 9_400, refill2, 19_64 (19x19/64/800), c5 (config 5)
# (the move-parallel lines' dominant kernel is k_search_queue; refill2 runs k_selfplay_move)
# Usage: TAG=r4b [LINES="head 19_64"] bash scripts/pmc_lines.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
: "${TAG:?set TAG}"
W9="9x9 Go self-play, 256 parallel games/GPU"
for l in ${LINES:-head 9_400 refill2 19_64 c5}; do
  case $l in
    head)    A="--steps 1 --warmup 1 --no-cpu-baseline"; WL="$W9, 200 sims/move"; K=k_search_queue; F=latest_pmc.json ;;
    9_400)   A="--sims 400 --steps 1 --warmup 1 --no-cpu-baseline"; WL="$W9, 400 sims/move"; K=k_search_queue; F=latest_pmc_9x9_g256_s400.json ;;
    refill2) A="--refill 2 --steps 2 --warmup 2 --no-cpu-baseline"; WL="$W9, 200 sims/move, refill 2"; K=k_selfplay_move; F=latest_pmc_9x9_g256_s200_refill2.json ;;
    19_64)   A="--board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline"; WL="19x19 Go self-play, 64 parallel games/GPU, 800 sims/move"; K=k_search_queue; F=latest_pmc_19x19_g64_s800.json ;;
    c5)      A="--config 5 --sims 64 --steps 1 --warmup 1 --no-cpu-baseline"; WL="19x19/C256/B20/G64"; K=k_tconv_chain; F=latest_tower_pmc.json ;;
    *) echo "unknown line $l" >&2; exit 2 ;;
  esac
  bash scripts/pmc.sh ${TAG}_$l $A > gpurun_out/pmc_${TAG}_$l.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}_$l.log; exit 1; }
  DYN=factored; [ $l = c5 ] && DYN=tower
  python3 scripts/summarize_pmc.py ${TAG}_$l "$WL" $DYN $K 0 $F > gpurun_out/pmc_${TAG}_$l.json || exit 1
  echo "$l: $(python3 -c "import json; d=json.load(open('profiles/${TAG}_${l}_pmc.json')); print(round(d['avg_duration_ms'],3), 'ms', round(d.get('hbm_bytes_per_launch',0)/1e9,3), 'GB', {k: round(v,4) for k, v in d.get('derived', {}).items() if isinstance(v, float)})")"
done
