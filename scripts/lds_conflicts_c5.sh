#!/bin/bash
# LDS bank conflicts of k_tconv_ks (config 5, 64 simulations) for library
# builds, one --pmc pass each (profiles/r4m_c5_lds_conflicts.txt):
#   LIBS="'' _swz" bash scripts/lds_conflicts_c5.sh
# '' = muzero-go_amd/mzgo/libmzgo.so, _x = libmzgo_x.so (scripts/build_variant.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
eval "LIBA=(${LIBS:-''})"
for v in "${LIBA[@]}"; do
  MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/p2_lib$v -o run -- python3 bench.py --config 5 --sims 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/p2_lib$v.log 2>&1 || exit 1
  python3 - "lib$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/p2_{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "k_tconv_ks" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[1], {k: v / max(n[k], 1) for k, v in acc.items()}, "conflict/active", acc["SQ_LDS_BANK_CONFLICT"] / acc["SQ_LDS_IDX_ACTIVE"])
PY
done
