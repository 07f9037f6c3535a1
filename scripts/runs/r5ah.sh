export TMPDIR=/tmp
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_sb.so timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_selfplay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ah_t.log 2>&1; rc=$?; tail -3 gpurun_out/r5ah_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _sb" REPS=3 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh && LIBS="'' _sb" REPS=1 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
