export TMPDIR=/tmp
# tail conv job granularity: (units, helpers) = (3, 2) base, (6, 5), (6, 3)
for v in t65 t63; do
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_parity.py -k "tail or whole_game" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ao_$v.log 2>&1; rc=$?; tail -1 gpurun_out/r5ao_$v.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="_t32 _t65 _t63" REPS=3 ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash scripts/gpu_ab.sh
