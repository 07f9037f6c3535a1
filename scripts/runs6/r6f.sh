# round 6, call f: config 5 -- batched steps (root batch + speculative cap 1 / 4 / 8, virtual-visit predictor) vs one leaf per step
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/diag/tower_predict.py > gpurun_out/r6f_predict.json 2> gpurun_out/r6f_predict.err || { tail -3 gpurun_out/r6f_predict.err; exit 1; }
cat gpurun_out/r6f_predict.json
for v in "MZGO_TOWER_SPEC=1" "MZGO_TOWER_SPEC=4" "MZGO_TOWER_SPEC=8" "MZGO_TOWER_BATCH=0"; do
  env $v timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/r6f_c5.json 2> gpurun_out/r6f_c5.err || { tail -5 gpurun_out/r6f_c5.err; exit 1; }
  echo "$v $(tail -1 gpurun_out/r6f_c5.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]), round(d["ms_per_step"],1), round(r["frac"],3), round(r["us_per_64_board_conv"],2), round(r["towers_per_simulation"],3), round(r["share_of_step"],3))')"
done
