#!/bin/bash
# default k_tconv_ks (register epilogue, DMA spread, dead tile skipped): tower parity, A/B vs k_tconv, clocks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_tower.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tower.log 2>&1 || { tail -30 gpurun_out/t_tower.log; exit 1; }
tail -2 gpurun_out/t_tower.log
for ks in 0 1 0 1; do
  MZGO_TCONV_KS=$ks timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5v.log 2>&1 || { tail -5 gpurun_out/c5v.log; exit 1; }
  echo "ks=$ks $(tail -1 gpurun_out/c5v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,2), "us/conv", round(r["frac"],3))')"
done
for ks in 0 1; do
  MZGO_TCONV_KS=$ks MZGO_LIB=muzero-go_amd/mzgo/libmzgo_ts.so timeout -k 10 300 python scripts/tconv_stamps.py > gpurun_out/ts_k$ks.log 2>&1 || { tail -5 gpurun_out/ts_k$ks.log; exit 1; }
  echo "== ks=$ks"; grep -v amdgpu.ids gpurun_out/ts_k$ks.log
done
