#!/bin/bash
# full GPU suite (k_tconv_ks default), then socket power / sclk samples during config 5 and the 9x9 headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -60 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
rocm-smi -M --json > gpurun_out/pw_max.json 2>&1 || true
sample() {   # $1 = output file; samples until killed
  while true; do echo "$(date +%s.%N) $(rocm-smi -P -c --json 2>/dev/null | tr -d '\n')"; sleep 0.2; done > "$1"
}
sample gpurun_out/pw_c5.txt & PW=$!
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5.json 2>&1; rc=$?
kill $PW; wait $PW 2>/dev/null
[ $rc -eq 0 ] || { tail -5 gpurun_out/c5.json; exit 1; }
echo "c5 $(tail -1 gpurun_out/c5.json | cut -c1-300)"
sample gpurun_out/pw_9.txt & PW=$!
timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline > gpurun_out/b9.json 2>&1; rc=$?
kill $PW; wait $PW 2>/dev/null
[ $rc -eq 0 ] || { tail -5 gpurun_out/b9.json; exit 1; }
echo "9x9 $(tail -1 gpurun_out/b9.json | cut -c1-300)"
