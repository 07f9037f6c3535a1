#!/bin/bash
# 9x9 bench (config 2, whole games) over library variants and moves per launch:
# LIBS="- _one" MPL="0 1" (suffixes of muzero-go_amd/mzgo/libmzgo*.so; "-" = default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${LIBS:--}; do
  [ "$v" = "-" ] && v=""
  for mpl in ${MPL:-0}; do
    MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python bench.py --steps ${STEPS:-3} --moves-per-launch $mpl --no-cpu-baseline ${EXTRA_ARGS:-} > gpurun_out/c2_lib${v}_m$mpl.log 2>&1 || exit $?
    echo "lib$v mpl=$mpl $(tail -1 gpurun_out/c2_lib${v}_m$mpl.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M sims/s", round(d["ms_per_step"],1), "ms/epoch")')"
  done
done
