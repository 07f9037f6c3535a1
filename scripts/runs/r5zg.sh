set -e
export TMPDIR=/tmp
# final build's phase stamps (9x9 / 256 / 200 whole epoch): the tail shares bench.py attaches
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python scripts/phases.py r5zg > gpurun_out/r5zg_ph.log 2>&1 || { tail -20 gpurun_out/r5zg_ph.log; exit 1; }
tail -c 600 gpurun_out/r5zg_ph.log
