#!/bin/bash
# Round 3: helper determinism per job kind, trainer HIP backward tests, 9x9 epoch phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/diag_det.jsonl
for v in "" _hs63 _hs62 _hs59 _hs55; do
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 200 python -u scripts/diag_det.py >> gpurun_out/diag_det.jsonl 2> gpurun_out/diag_det$v.err || { tail -5 gpurun_out/diag_det$v.err; exit 1; }
done
cat gpurun_out/diag_det.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trainer.py > gpurun_out/t_trainer.log 2>&1 || { tail -40 gpurun_out/t_trainer.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_trainer.log | tail -2
MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python -u scripts/phases.py r3e > gpurun_out/phases.log 2>&1 || { tail -20 gpurun_out/phases.log; exit 1; }
tail -c 1500 gpurun_out/phases.log
