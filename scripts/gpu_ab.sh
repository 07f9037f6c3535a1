#!/bin/bash
# A/B of library builds on one bench command, in one GPU call (boxes differ by
# +-1.5 %, so only same-call pairs are compared), REPS rounds alternating:
#   LIBS="'' _v1" REPS=2 ARGS="--steps 20 --no-cpu-baseline" bash scripts/gpu_ab.sh
# '' = muzero-go_amd/mzgo/libmzgo.so, _x = libmzgo_x.so (scripts/build_variant.sh);
# ENVS="A=1 B=2" optional per-variant environment, paired with LIBS by position.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
eval "LIBA=(${LIBS:-''})"
eval "ENVA=(${ENVS:-})"
for rep in $(seq 1 ${REPS:-2}); do
  for i in "${!LIBA[@]}"; do
    v=${LIBA[$i]}; e=${ENVA[$i]:-}
    env $e MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 ${LIMIT:-300} python bench.py ${ARGS:---steps 20 --no-cpu-baseline} > gpurun_out/ab$v.json 2> gpurun_out/ab$v.err || { tail -5 gpurun_out/ab$v.err; exit 1; }
    echo "rep $rep lib$v $e $(tail -1 gpurun_out/ab$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e6,3), "M sims/s", round(d["ms_per_step"],2), "ms/step", r["kernel"], round(r["avg_launch_ms"],4), "ms/launch")')"
  done
done
