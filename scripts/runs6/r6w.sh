# round 6: two children per wave in the 9x9 lazy batches (ExpandLds::PAIR) -- the self-play /
# search / parity tests, then a same-box A/B of the headline (MZGO_PAIR_EXPAND)
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6w}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_selfplay.py tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread \
  > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
for pe in 1 0 1 0; do
  MZGO_PAIR_EXPAND=$pe timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_pe$pe.json 2> gpurun_out/${TAG}_pe$pe.err || { tail -5 gpurun_out/${TAG}_pe$pe.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print('9x9 pairs',sys.argv[2],round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms',round(r['avg_launch_ms'],2))" gpurun_out/${TAG}_pe$pe.json $pe
done
