# round 6: 19x19/64/800 with one child per wave in the lazy batches (the pair loop's claim of 1), twice
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r6y2_19_$i.json 2> gpurun_out/r6y2_19_$i.err || { tail -5 gpurun_out/r6y2_19_$i.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print('19x19 singles',round(d['value']/1e6,2),'M',round(d['ms_per_step'],2),'ms')" gpurun_out/r6y2_19_$i.json
done
