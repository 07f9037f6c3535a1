# round 6, the move-parallel build: counter passes of k_search_queue (headline, 19x19/64/800)
# and the headline's memory-side requests
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6m}
TAG=$TAG LINES="head 19_64" bash scripts/pmc_lines.sh || exit 1
bash scripts/pmc_tcc.sh ${TAG}_head --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_tcc.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_tcc.log; exit $rc
