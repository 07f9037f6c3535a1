#!/bin/bash
# Round 3: LDS Y copy from the conv epilogue -- parity (search / self-play / bench-size), bench, phases with slots.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_selfplay.py tests/test_gpu_bench_parity.py tests/test_gpu_net.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_h.log 2>&1 || { tail -60 gpurun_out/t_h.log; exit 1; }
tail -2 gpurun_out/t_h.log
timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/h9.json 2>&1 || { tail -5 gpurun_out/h9.json; exit 1; }
echo "9x9 $(tail -1 gpurun_out/h9.json | cut -c1-220)"
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python -u scripts/phases.py r3h > gpurun_out/phases_h.log 2>&1 || { tail -20 gpurun_out/phases_h.log; exit 1; }
tail -c 600 gpurun_out/phases_h.log
