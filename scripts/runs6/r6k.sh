# round 6: the move-parallel epoch (boards launch + k_search_queue) -- its exactness
# tests against the game-per-workgroup launch, then a same-box A/B of the headline
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6k}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py -x -v --timeout 600 --timeout-method thread \
  -k "move_parallel or whole_game or tail_helpers" > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -12 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
for mp in 1 0 1 0; do
  MZGO_MOVE_PARALLEL=$mp timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_mp$mp.json 2> gpurun_out/${TAG}_mp$mp.err || { tail -5 gpurun_out/${TAG}_mp$mp.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms',r['kernel'],round(r['avg_launch_ms'],2),r.get('boards_launch_ms'))" gpurun_out/${TAG}_mp$mp.json $mp
done
for mp in 1 0; do
  MZGO_MOVE_PARALLEL=$mp timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_19mp$mp.json 2> gpurun_out/${TAG}_19mp$mp.err || { tail -5 gpurun_out/${TAG}_19mp$mp.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print('19x19',sys.argv[2],round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms',r['kernel'],round(r['avg_launch_ms'],2),r.get('boards_launch_ms'))" gpurun_out/${TAG}_19mp$mp.json $mp
done
