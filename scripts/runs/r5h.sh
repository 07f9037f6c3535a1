set -e
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5h_t.log 2>&1 || { tail -40 gpurun_out/r5h_t.log; exit 1; }
tail -1 gpurun_out/r5h_t.log
LIBS="'' _base" REPS=2 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh
LIBS="'' _base" REPS=1 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
