# round 6, call c: batched tower steps -- identity vs one-leaf steps, the tower suite, config-5 lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_tower.py > gpurun_out/r6c_t.log 2>&1; rc=$?; tail -30 gpurun_out/r6c_t.log; [ $rc -eq 0 ] || exit $rc
for sp in 8 32 128; do
  MZGO_TOWER_SPEC=$sp timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/r6c_c5_spec$sp.json 2> gpurun_out/r6c_c5_spec$sp.err || { tail -5 gpurun_out/r6c_c5_spec$sp.err; exit 1; }
  echo "spec $sp $(tail -1 gpurun_out/r6c_c5_spec$sp.json | cut -c1-200)"
done
MZGO_TOWER_BATCH=0 timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/r6c_c5_oneleaf.json 2> gpurun_out/r6c_c5_oneleaf.err || { tail -5 gpurun_out/r6c_c5_oneleaf.err; exit 1; }
echo "oneleaf $(tail -1 gpurun_out/r6c_c5_oneleaf.json | cut -c1-200)"
