# round 6: 19x19 pair expansion with Y loads two passes ahead -- the 19x19 tests, then 19x19/64/800 twice
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6y}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_selfplay.py -x -q --timeout 600 --timeout-method thread \
  -k "19" > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_19_$i.json 2> gpurun_out/${TAG}_19_$i.err || { tail -5 gpurun_out/${TAG}_19_$i.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print('19x19',round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms',round(r['avg_launch_ms'],2))" gpurun_out/${TAG}_19_$i.json
done
