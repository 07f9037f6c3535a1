# round 6: helpers in the 19x19 queue (MZGO_QUEUE_HELPERS) -- exactness, then an A/B at 19x19/64/800
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "move_parallel and 19x19" > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -4 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
for h in 0 1 3 0 1; do
  MZGO_QUEUE_HELPERS=$h timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_h$h.json 2> gpurun_out/${TAG}_h$h.err || { tail -5 gpurun_out/${TAG}_h$h.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print('19x19 qh',sys.argv[2],round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms',round(r['avg_launch_ms'],2))" gpurun_out/${TAG}_h$h.json $h
done
