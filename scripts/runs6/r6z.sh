# round 6, final build: GPU suite, smoke(), every bench line DESIGN quotes (config 5 with its
# cpu_baseline), counter passes of the headline and config-5 kernels, memory-side requests
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG LINES="bench 9_400 refill2 19_64 c5 c5mid" bash scripts/gpu_lines.sh || exit 1
TAG=$TAG LINES="head c5" bash scripts/pmc_lines.sh || exit 1
bash scripts/pmc_tcc.sh ${TAG}_head --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_tcc.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_tcc.log; exit $rc
