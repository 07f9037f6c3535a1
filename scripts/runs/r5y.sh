export TMPDIR=/tmp
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_diag.so G=16 S=96 M=3 timeout -k 10 120 python scripts/xcc_diag.py > gpurun_out/r5y_a.log 2>&1; tail -1 gpurun_out/r5y_a.log
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_diag.so G=64 S=800 M=3 timeout -k 10 120 python scripts/xcc_diag.py > gpurun_out/r5y_b.log 2>&1; tail -1 gpurun_out/r5y_b.log
