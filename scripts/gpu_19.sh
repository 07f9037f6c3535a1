set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_selfplay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_19.log 2>&1; rc=$?
tail -5 gpurun_out/t_19.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --board-size 19 --games 64 --sims 800 > gpurun_out/b19.log 2>&1 || exit $?
tail -1 gpurun_out/b19.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b9.log 2>&1 || exit $?
tail -1 gpurun_out/b9.log | cut -c1-300
