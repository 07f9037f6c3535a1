# round 6: 19x19 move-parallel phase slots with the two-child expansion (stamps build)
export TMPDIR=/tmp
mkdir -p gpurun_out
export MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so MZGO_MOVE_PARALLEL=1
N=19 G=64 S=800 timeout -k 10 300 python scripts/phases.py r6q_mp19 > gpurun_out/r6q_mp19.log 2>&1 || { tail -5 gpurun_out/r6q_mp19.log; exit 1; }
