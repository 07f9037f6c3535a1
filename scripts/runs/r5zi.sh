export TMPDIR=/tmp
# the driver's round-end commands on the committed tree: smoke() and the default bench line
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5zi_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r5zi_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r5zi_default_bench.json 2> gpurun_out/r5zi_default_bench.err; rc=$?; tail -c 1500 gpurun_out/r5zi_default_bench.json; exit $rc
