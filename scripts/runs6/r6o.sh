# round 6: phase shares of the move-parallel epoch (stamps build), 9x9/256/200 and 19x19/64/800
export TMPDIR=/tmp
mkdir -p gpurun_out
export MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so MZGO_MOVE_PARALLEL=1
timeout -k 10 300 python scripts/phases.py r6o_mp9 > gpurun_out/r6o_mp9.log 2>&1 || { tail -5 gpurun_out/r6o_mp9.log; exit 1; }
N=19 G=64 S=800 timeout -k 10 300 python scripts/phases.py r6o_mp19 > gpurun_out/r6o_mp19.log 2>&1 || { tail -5 gpurun_out/r6o_mp19.log; exit 1; }
python -c "
import json
for t in ('r6o_mp9','r6o_mp19'):
    d=json.load(open('gpurun_out/%s_phases.json'%t)); print(t, round(d['epoch_ms_stamps_build'],1), {k: round(v,3) for k,v in d['shares'].items()})"
