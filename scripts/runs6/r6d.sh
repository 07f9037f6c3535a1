# round 6, call d: rank-based speculative tower batches -- tower suite, config-5 lines per speculation cap
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_tower.py > gpurun_out/r6d_t.log 2>&1; rc=$?; tail -12 gpurun_out/r6d_t.log; [ $rc -eq 0 ] || exit $rc
for sp in 16 32 64; do
  MZGO_TOWER_SPEC=$sp timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/r6d_c5_spec$sp.json 2> gpurun_out/r6d_c5_spec$sp.err || { tail -5 gpurun_out/r6d_c5_spec$sp.err; exit 1; }
  echo "spec $sp $(tail -1 gpurun_out/r6d_c5_spec$sp.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],1), round(r["frac"],3), round(r["us_per_64_board_conv"],2), round(r["towers_per_simulation"],3), round(r["share_of_step"],3))')"
done
