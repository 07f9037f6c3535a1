#!/bin/bash
# Search/self-play parity (GPU tests), then whole-game stamps at 19x19/64/800 and 9x9/256/200.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_selfplay.py tests/test_gpu_bench_parity.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_verify.log 2>&1 || { tail -40 gpurun_out/t_verify.log; exit 1; }
tail -2 gpurun_out/t_verify.log
if [ "${STAMPS:-1}" = 1 ]; then
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo_stamps.so N=19 G=64 S=800 GAME_STAMPS=1 timeout -k 10 400 python scripts/microbench.py > gpurun_out/game19.json || exit $?
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo_stamps.so N=9 G=256 S=200 GAME_STAMPS=1 timeout -k 10 200 python scripts/microbench.py > gpurun_out/game9.json || exit $?
  tail -1 gpurun_out/game19.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("19x19 game_ms", round(d["game_ms"]), "seq replay sims", d["seq_replay_sims_per_game"], "depth", round(d["mean_leaf_depth"],2))'
  tail -1 gpurun_out/game9.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("9x9 game_ms", round(d["game_ms"],1), "seq replay sims", d["seq_replay_sims_per_game"])'
fi
