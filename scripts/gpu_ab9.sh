#!/bin/bash
# A/B of library variants on the 9x9 headline (and 19x19): VARIANTS="base pa" (base = libmzgo.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then L=$PWD/muzero-go_amd/mzgo/libmzgo.so; else L=$PWD/muzero-go_amd/mzgo/libmzgo_$v.so; fi
  MZGO_LIB=$L timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/ab9_$v.json 2>&1 || { tail -5 gpurun_out/ab9_$v.json; exit 1; }
  echo "$v 9x9 $(tail -1 gpurun_out/ab9_$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2))')"
  if [ -n "${B19:-}" ]; then
  MZGO_LIB=$L timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ab19_$v.json 2>&1 || { tail -5 gpurun_out/ab19_$v.json; exit 1; }
  echo "$v 19x19 $(tail -1 gpurun_out/ab19_$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2))')"
  fi
done
done
