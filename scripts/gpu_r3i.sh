#!/bin/bash
# Round 3: parity of the LDS parent read; Winograd wave-priority variants (9x9 epoch A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_selfplay.py tests/test_gpu_bench_parity.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_i.log 2>&1 || { tail -60 gpurun_out/t_i.log; exit 1; }
tail -2 gpurun_out/t_i.log
for rep in 1 2; do
for v in "" _p2 _p3 _s1 _s2; do
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/i9$v.json 2>&1 || { tail -5 gpurun_out/i9$v.json; exit 1; }
  echo "lib$v $(tail -1 gpurun_out/i9$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M", round(d["ms_per_step"],2), "ms")')"
done
done
