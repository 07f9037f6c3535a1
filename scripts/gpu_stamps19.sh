#!/bin/bash
# 19x19 / 64 games / 800 sims whole-game phase stamps (libmzgo_stamps.so,
# scripts/build_stamps.sh) -> gpurun_out/${OUT:-stamps19}.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_${VARIANT:-stamps}.so GAME_STAMPS=1 N=19 G=64 S=800 \
  timeout -k 10 400 python -u scripts/microbench.py > gpurun_out/${OUT:-stamps19}.json 2> gpurun_out/${OUT:-stamps19}.err || { tail -20 gpurun_out/${OUT:-stamps19}.err; exit 1; }
tail -c 3000 gpurun_out/${OUT:-stamps19}.json
