set -e
export TMPDIR=/tmp
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python scripts/phases.py r5k > gpurun_out/r5k_ph.log 2>&1 || { tail -20 gpurun_out/r5k_ph.log; exit 1; }
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python scripts/phases_split.py > gpurun_out/r5k_split.json 2> gpurun_out/r5k_split.err || { tail -20 gpurun_out/r5k_split.err; exit 1; }
tail -c 3000 gpurun_out/r5k_split.json
