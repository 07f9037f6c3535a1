set -e
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_bench_parity.py -x -q --timeout 400 --timeout-method thread -k "not refill" > gpurun_out/r5m_t.log 2>&1 || { tail -30 gpurun_out/r5m_t.log; exit 1; }
tail -1 gpurun_out/r5m_t.log
LIBS="'' _nopf" REPS=3 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh
