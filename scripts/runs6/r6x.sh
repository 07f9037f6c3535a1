# round 6, the move-parallel build with k_selfplay_boards, the 19x19 pair expansion and lazy 19x19 rows: GPU suite,
# smoke(), counter passes of k_search_queue (their summaries land in profiles/ on the box, so the
# bench lines after them carry the counters), memory-side requests, then the lines
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6x}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG LINES="head 19_64" bash scripts/pmc_lines.sh || exit 1
cp profiles/${TAG}_head_pmc.json profiles/${TAG}_19_64_pmc.json profiles/${TAG}_head_kernel_stats.csv profiles/${TAG}_19_64_kernel_stats.csv gpurun_out/
bash scripts/pmc_tcc.sh ${TAG}_head --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_tcc.log 2>&1 || { tail -3 gpurun_out/${TAG}_tcc.log; exit 1; }
TAG=$TAG LINES="bench 9_400 19_64" bash scripts/gpu_lines.sh
