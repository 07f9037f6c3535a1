set -e
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5e_t.log 2>&1 || { tail -40 gpurun_out/r5e_t.log; exit 1; }
tail -2 gpurun_out/r5e_t.log
for cfg in "8 32 2000" "8 32 20000"; do
  REPS=3 timeout -k 10 300 python scripts/rccl_standin.py $cfg > gpurun_out/r5e_standin_${cfg// /_}.json 2> gpurun_out/r5e_si.err || { tail -20 gpurun_out/r5e_si.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['standin'], {m: round(d[m]['mean_ms'],3) for m in ('none','overlap','ordered','gated')}, {k: {kk: round(vv,3) for kk,vv in v.items()} for k,v in d.items() if k.endswith('delay_ms')})" gpurun_out/r5e_standin_${cfg// /_}.json
done
