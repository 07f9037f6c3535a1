# round 6, call g: full GPU suite + smoke, CPU baseline scaling on the box's host cores, default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6g_t.log 2>&1; rc=$?; tail -3 gpurun_out/r6g_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6g_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r6g_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/cpu_scaling.py --procs 16 32 64 --budget 8 > gpurun_out/r6g_cpu_scaling.json 2> gpurun_out/r6g_cpu_scaling.err; rc=$?; cat gpurun_out/r6g_cpu_scaling.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r6g_bench.json 2> gpurun_out/r6g_bench.err; rc=$?; tail -1 gpurun_out/r6g_bench.json | cut -c1-300; exit $rc
