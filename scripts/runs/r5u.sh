set -e
export TMPDIR=/tmp
N=19 G=64 S=800 MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 400 python scripts/phases.py r5u_19 > gpurun_out/r5u_19.log 2>&1 || { tail -20 gpurun_out/r5u_19.log; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5u_19_phases.json"))
print(d["shares"], d["tail"]["idle_cu_share"], d["epoch_ms_stamps_build"])
s = d["slots_mean_per_game"]
print({k: round(v / 1e6, 2) for k, v in sorted(s.items(), key=lambda x: int(x[0]))})
PY
