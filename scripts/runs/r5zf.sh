export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5zf_t.log 2>&1; rc=$?; tail -3 gpurun_out/r5zf_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5zf_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r5zf_smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=r5zf LINES="bench 9_400 refill2 19_64 c5" bash scripts/gpu_lines.sh || exit 1
bash scripts/pmc.sh r5zf --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5zf_pmc.log 2>&1 || { tail -5 gpurun_out/r5zf_pmc.log; exit 1; }
bash scripts/pmc_tcc.sh r5zf --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5zf_tcc.log 2>&1; rc=$?; tail -3 gpurun_out/r5zf_tcc.log; exit $rc
