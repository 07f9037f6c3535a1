export TMPDIR=/tmp
# 9x9 tail: speculative batches as jobs the tail helpers share
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_parity.py -k "tail or whole_game" -x -v --timeout 200 --timeout-method thread > gpurun_out/r5aq_tail.log 2>&1; rc=$?; tail -2 gpurun_out/r5aq_tail.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5aq_t.log 2>&1; rc=$?; tail -2 gpurun_out/r5aq_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _prev" REPS=3 ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash scripts/gpu_ab.sh
