export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_selfplay.py -x -q --timeout 120 --timeout-method thread -k "helper" > gpurun_out/r5s_a.log 2>&1; rc=$?; tail -5 gpurun_out/r5s_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s_t.log 2>&1; rc=$?; tail -15 gpurun_out/r5s_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _prev" REPS=2 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
