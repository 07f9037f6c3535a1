#!/bin/bash
# 9x9: small batches replayed one select at a time (MZGO_VERIFY_MIN_B sweep, timing only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in "" _sk14 _sk18 _sk20; do
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b9$v.json 2>&1 || { tail -5 gpurun_out/b9$v.json; exit 1; }
  echo "9x9 lib$v $(tail -1 gpurun_out/b9$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M sims/s", round(d["ms_per_step"],2), "ms/epoch")')"
done
done
