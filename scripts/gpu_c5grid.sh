#!/bin/bash
# k_tconv grid: library variants (LIBS suffixes) x waves per workgroup (NWS),
# config-5 bench at 256 sims; no parity (timing A/B only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${LIBS:-"-"}; do
  [ "$v" = "-" ] && v=""
  for nw in ${NWS:-8 4}; do
    MZGO_TCONV_WAVES=$nw MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5g${v}_$nw.log 2>&1 || { tail -5 gpurun_out/c5g${v}_$nw.log; exit 1; }
    echo "lib$v nw=$nw $(tail -1 gpurun_out/c5g${v}_$nw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,2), "us/conv", round(r["frac"],3))')"
  done
done
