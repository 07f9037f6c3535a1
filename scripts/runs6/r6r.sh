# round 6: the boards launch as its own small kernel (k_selfplay_boards) -- exactness tests, then the lines
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6r}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py -x -v --timeout 600 --timeout-method thread \
  -k "move_parallel or whole_game" > gpurun_out/${TAG}_t.log 2>&1; rc=$?; grep -c PASSED gpurun_out/${TAG}_t.log; tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
for l in 9 9 19; do
  if [ $l = 9 ]; then A="--steps 20 --warmup 3"; else A="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1"; fi
  timeout -k 10 300 python bench.py $A --no-cpu-baseline > gpurun_out/${TAG}_$l.json 2> gpurun_out/${TAG}_$l.err || { tail -5 gpurun_out/${TAG}_$l.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms queue',round(r['avg_launch_ms'],2),'boards',round(r['boards_launch_ms'],3))" gpurun_out/${TAG}_$l.json $l
done
