export TMPDIR=/tmp
bash scripts/runs/r5y.sh
bash scripts/runs/r5z2.sh
