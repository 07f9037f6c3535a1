export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ag_t.log 2>&1; rc=$?; tail -4 gpurun_out/r5ag_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _prev" REPS=2 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh && LIBS="'' _prev" REPS=2 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh
