export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5ak_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r5ak_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r5ak_default.json 2> gpurun_out/r5ak_default.err; rc=$?; tail -c 400 gpurun_out/r5ak_default.json; exit $rc
