export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5af_t.log 2>&1; rc=$?; tail -4 gpurun_out/r5af_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _prev" REPS=3 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh
