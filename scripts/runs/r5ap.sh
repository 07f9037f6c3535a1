export TMPDIR=/tmp
# tail conv job granularity: (units, helpers) = (3, 2) base, (2, 1), (3, 1)
for v in t21 t31; do
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_parity.py -k "tail or whole_game" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ap_$v.log 2>&1; rc=$?; tail -1 gpurun_out/r5ap_$v.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="_t32 _t21 _t31" REPS=3 ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash scripts/gpu_ab.sh
