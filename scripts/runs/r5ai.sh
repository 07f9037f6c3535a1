export TMPDIR=/tmp
mkdir -p gpurun_out/icache
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/icache -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/icache/run.log 2>&1; echo "rc=$?"; tail -3 gpurun_out/icache/run.log
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/icache/**/run_counter_collection.csv", recursive=True)
print(f)
if f:
    s = collections.defaultdict(float)
    for r in csv.DictReader(open(f[0])):
        if "k_selfplay_move" in r["Kernel_Name"]:
            s[r["Counter_Name"]] += float(r["Counter_Value"])
    print(dict(s))
PY
