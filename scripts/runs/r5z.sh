export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5z_t.log 2>&1; rc=$?; tail -3 gpurun_out/r5z_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5z_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r5z_smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=r5z LINES="bench 19_64 c5 c5mid" bash scripts/gpu_lines.sh || exit 1
bash scripts/pmc.sh r5z --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5z_pmc.log 2>&1; rc=$?; tail -8 gpurun_out/r5z_pmc.log; exit $rc
