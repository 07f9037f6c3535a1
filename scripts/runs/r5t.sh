export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -q --timeout 200 --timeout-method thread -k "chain_wait_expiry" > gpurun_out/r5t_a.log 2>&1; tail -3 gpurun_out/r5t_a.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_trainer.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5t_t.log 2>&1; rc=$?; tail -8 gpurun_out/r5t_t.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LIBS="'' _prev" REPS=2 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
