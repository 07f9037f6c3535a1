#!/bin/bash
# Round 3: helper determinism for pairs of job kinds; no-LICM build vs default (bench A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/diag_det2.jsonl
for v in _hs51 _hs58 _hs54 _hs11 _hs14 _hs7; do
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo$v.so RUNS=2 timeout -k 10 200 python -u scripts/diag_det.py >> gpurun_out/diag_det2.jsonl 2> gpurun_out/diag_det$v.err || { tail -5 gpurun_out/diag_det$v.err; exit 1; }
done
cat gpurun_out/diag_det2.jsonl
for v in "" _nolicm "" _nolicm; do
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/ab9$v.json 2>&1 || { tail -5 gpurun_out/ab9$v.json; exit 1; }
  echo "9x9 lib$v $(tail -1 gpurun_out/ab9$v.json | cut -c1-200)"
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 200 python bench.py --board-size 19 --games 64 --sims 800 --steps 2 --no-cpu-baseline > gpurun_out/ab19$v.json 2>&1 || { tail -5 gpurun_out/ab19$v.json; exit 1; }
  echo "19x19 lib$v $(tail -1 gpurun_out/ab19$v.json | cut -c1-200)"
done
