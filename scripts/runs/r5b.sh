set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_tower.py -x -q --timeout 300 --timeout-method thread -k "tail_helpers or chain_wait or chain_launch or multi_move" > gpurun_out/r5b_t.log 2>&1 || { tail -30 gpurun_out/r5b_t.log; exit 1; }
tail -3 gpurun_out/r5b_t.log
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python scripts/phases.py r5b > gpurun_out/r5b_ph.log 2>&1 || { tail -20 gpurun_out/r5b_ph.log; exit 1; }
tail -5 gpurun_out/r5b_ph.log
