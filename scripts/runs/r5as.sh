export TMPDIR=/tmp
# job hand-off polling: s_sleep (job_wait 4, helper poll 8) against (1, 2)
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_s12.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_parity.py -k "tail or whole_game" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5as_t.log 2>&1; rc=$?; tail -1 gpurun_out/r5as_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="_s48 _s12" REPS=3 ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash scripts/gpu_ab.sh || exit 1
LIBS="_s48 _s12" REPS=2 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
