#!/bin/bash
# replay rule (B-1)(depth+1) < 16 by default: GPU suite, A/B against min B 2,
# and the (B - 1)(depth + 1) < K rule variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -60 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
for v in _old "" _old ""; do
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b9$v.json 2>&1 || { tail -5 gpurun_out/b9$v.json; exit 1; }
  echo "9x9 lib$v $(tail -1 gpurun_out/b9$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M sims/s", round(d["ms_per_step"],2), "ms/epoch")')"
done
