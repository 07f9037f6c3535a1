#!/bin/bash
# Compare diagnostic build variants (libmzgo_<v>.so, scripts/build_stamps.sh)
# on the 9x9 search: VARIANTS="stamps sync1 ..." bash scripts/gpu_variants.sh
set -e
cd "$(dirname "$0")/.."
for v in ${VARIANTS:-stamps}; do
  echo "== $v"
  STAMPS=1 MZGO_LIB=muzero-go_amd/mzgo/libmzgo_$v.so timeout -k 10 300 python scripts/microbench.py
done
