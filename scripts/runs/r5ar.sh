export TMPDIR=/tmp
# 9x9 tail batch jobs: the smallest shared batch (12 / 24 / 48) against HEAD without them
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_b24.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_parity.py -k "tail" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ar_t.log 2>&1; rc=$?; tail -1 gpurun_out/r5ar_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="_prev _b12 _b24 _b48" REPS=2 ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash scripts/gpu_ab.sh
