set -e
export TMPDIR=/tmp
REPS=3 timeout -k 10 300 python scripts/rccl_standin.py 8 32 2000 > gpurun_out/r5c_standin_8_32_2000.json 2> gpurun_out/r5c_si.err || { tail -20 gpurun_out/r5c_si.err; exit 1; }
cat gpurun_out/r5c_standin_8_32_2000.json
REPS=3 timeout -k 10 300 python scripts/rccl_standin.py 1 8 500 > gpurun_out/r5c_standin_1_8_500.json 2> gpurun_out/r5c_si.err || { tail -20 gpurun_out/r5c_si.err; exit 1; }
cat gpurun_out/r5c_standin_1_8_500.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c_t.log 2>&1 || { tail -30 gpurun_out/r5c_t.log; exit 1; }
tail -2 gpurun_out/r5c_t.log
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/r5c_bench.json 2> gpurun_out/r5c_bench.err || { tail -5 gpurun_out/r5c_bench.err; exit 1; }
cut -c1-600 gpurun_out/r5c_bench.json
