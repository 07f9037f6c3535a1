export TMPDIR=/tmp
bash scripts/r5y.sh
bash scripts/r5z2.sh
