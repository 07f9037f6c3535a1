export TMPDIR=/tmp
# tail conv units: the first unit's second slab transformed under its GEMM
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5an_t.log 2>&1; rc=$?; tail -3 gpurun_out/r5an_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _prev" REPS=3 ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash scripts/gpu_ab.sh || exit 1
LIBS="'' _prev" REPS=2 ARGS="--sims 400 --steps 8 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
