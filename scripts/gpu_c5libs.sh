#!/bin/bash
# Config-5 bench (256 sims) over library variants: LIBS="'' _a1 _a3" (suffixes of
# muzero-go_amd/mzgo/libmzgo*.so); tower parity on the default library first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -q --timeout 300 --timeout-method thread > gpurun_out/t_tower.log 2>&1 || { tail -30 gpurun_out/t_tower.log; exit 1; }
tail -1 gpurun_out/t_tower.log
for v in ${LIBS:-""} ; do
  [ "$v" = "-" ] && v=""
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 300 python bench.py --config 5 --sims 256 --steps 2 --no-cpu-baseline > gpurun_out/c5_lib$v.log 2>&1 || exit $?
  echo "lib$v $(tail -1 gpurun_out/c5_lib$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), "sims/s", round(r["avg_launch_ms"]*1e3,1), "us/conv", round(r["frac"],3))')"
done
if [ -f muzero-go_amd/mzgo/libmzgo_ts.so ] && [ "${STAMPS:-1}" = 1 ]; then
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo_ts.so timeout -k 10 200 python scripts/tconv_stamps.py || exit $?
fi
