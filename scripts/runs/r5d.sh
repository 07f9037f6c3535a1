set -e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_tower.py -x -v --timeout 600 --timeout-method thread -k "bench_config_matches_oracle or exact_replay" > gpurun_out/r5d_t.log 2>&1 || { tail -40 gpurun_out/r5d_t.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r5d_t.log | tail -8
REPS=3 timeout -k 10 300 python scripts/rccl_standin.py 8 32 2000 > gpurun_out/r5d_standin_8_32_2000.json 2> gpurun_out/r5d_si.err || { tail -20 gpurun_out/r5d_si.err; exit 1; }
cat gpurun_out/r5d_standin_8_32_2000.json
