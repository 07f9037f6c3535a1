# round 6: 19x19 queue phases with lazy rows (stamps build)
export TMPDIR=/tmp
mkdir -p gpurun_out
export MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so MZGO_MOVE_PARALLEL=1
N=19 G=64 S=800 timeout -k 10 300 python scripts/phases.py r6v_mp19 > gpurun_out/r6v_mp19.log 2>&1 || { tail -5 gpurun_out/r6v_mp19.log; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/r6v_mp19_phases.json')); print(round(d['epoch_ms_stamps_build'],1), {k: round(v,3) for k,v in d['shares'].items()})"
