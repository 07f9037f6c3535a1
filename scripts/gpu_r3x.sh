#!/bin/bash
# 9x9 epoch phases per move segment (stamps build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MZGO_LIB=muzero-go_amd/mzgo/libmzgo_stamps.so timeout -k 10 300 python scripts/phases_split.py > gpurun_out/phsplit.json 2>gpurun_out/phsplit.err || { tail -5 gpurun_out/phsplit.err; exit 1; }
cat gpurun_out/phsplit.json
