export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_bench_parity.py -x -v --timeout 150 --timeout-method thread -k "helper or 19 or tail" > gpurun_out/r5v_a.log 2>&1; rc=$?; tail -5 gpurun_out/r5v_a.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _prev" REPS=2 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
