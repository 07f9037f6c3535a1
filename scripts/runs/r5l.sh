set -e
export TMPDIR=/tmp
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python scripts/phases.py r5n > gpurun_out/r5n_ph.log 2>&1 || { tail -20 gpurun_out/r5n_ph.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5n_phases.json')); s=d['slots_mean_per_game']
print(d['shares'], d['tail']['idle_cu_share'])
print({k: s.get(k) for k in ['0','22','23','24','25','26','27','32','33','35','36','37','38','39']})
"
