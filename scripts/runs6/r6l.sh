# round 6, the move-parallel build: GPU suite, smoke(), the bench lines DESIGN quotes
# (headline with cpu_baseline, 9x9/400, refill 2, 19x19/64/800)
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6l}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG LINES="bench 9_400 refill2 19_64" bash scripts/gpu_lines.sh
