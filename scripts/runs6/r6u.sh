# round 6: lazy policy rows in the 19x19 queue's batches (sp.lazy_rows) -- the 19x19 tests, then an A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6u}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_selfplay.py tests/test_gpu_search.py -x -v --timeout 600 --timeout-method thread \
  -k "19" > gpurun_out/${TAG}_t.log 2>&1; rc=$?; grep -c PASSED gpurun_out/${TAG}_t.log; tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
for lz in 1 0 1; do
  MZGO_LAZY_ROWS=$lz timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_lz$lz.json 2> gpurun_out/${TAG}_lz$lz.err || { tail -5 gpurun_out/${TAG}_lz$lz.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print('19x19 lazy',sys.argv[2],round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms',round(r['avg_launch_ms'],2),'rows/move',round(r['prior_rows_per_move'],1))" gpurun_out/${TAG}_lz$lz.json $lz
done
