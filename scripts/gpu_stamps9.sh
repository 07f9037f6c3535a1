#!/bin/bash
# 9x9 / 256 games / 200 sims whole-game phase stamps (libmzgo_stamps.so) -> gpurun_out/${OUT:-stamps9}.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_${VARIANT:-stamps}.so GAME_STAMPS=1 N=9 G=256 S=${S:-200} \
  timeout -k 10 300 python -u scripts/microbench.py > gpurun_out/${OUT:-stamps9}.json 2> gpurun_out/${OUT:-stamps9}.err || { tail -20 gpurun_out/${OUT:-stamps9}.err; exit 1; }
tail -c 3000 gpurun_out/${OUT:-stamps9}.json
