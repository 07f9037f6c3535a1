#!/bin/bash
# Helper-path determinism per job kind (libmzgo_hs*.so: helpers skip job kinds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in _hs63 _hs62 _hs59 _hs55; do
  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 200 python -u scripts/diag_det.py >> gpurun_out/diag_det.jsonl 2> gpurun_out/diag_det$v.err || { tail -5 gpurun_out/diag_det$v.err; exit 1; }
done
cat gpurun_out/diag_det.jsonl
