#!/bin/bash
# Phase stamps of diagnostic library variants (libmzgo_<v>.so), one line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  echo "== $v"
  STAMPS=1 MZGO_LIB=muzero-go_amd/mzgo/libmzgo_$v.so timeout -k 10 120 python scripts/microbench.py || exit $?
done
