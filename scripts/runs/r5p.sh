set -e
export TMPDIR=/tmp
for v in stamps stpf; do
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_$v.so timeout -k 10 300 python scripts/phases.py r5p_$v > gpurun_out/r5p_$v.log 2>&1 || { tail -20 gpurun_out/r5p_$v.log; exit 1; }
done
python3 - <<'PY'
import json
for v in ("stamps", "stpf"):
    d = json.load(open(f"gpurun_out/r5p_{v}_phases.json"))
    s = d["slots_mean_per_game"]
    print(v, "mean game", round(d["tail"]["mean_game_cycles"]/1e6, 2), "max", round(d["tail"]["max_game_cycles"]/1e6, 2),
          {k: round(s.get(k, 0)/1e6, 3) for k in ("22", "23", "24", "35", "36", "37", "38", "48", "91")})
PY
