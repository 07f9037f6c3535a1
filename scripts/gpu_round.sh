set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -3 gpurun_out/t_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
bash scripts/profile.sh r1 --steps 6 --warmup 1 --no-cpu-baseline || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-budget 8 > gpurun_out/bench_full.log 2>&1 || exit $?
tail -1 gpurun_out/bench_full.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dynamics direct > gpurun_out/bench_direct.log 2>&1 || exit $?
tail -1 gpurun_out/bench_direct.log | cut -c1-300
