export TMPDIR=/tmp
LIBS="'' _p1 _p2 _p3" REPS=2 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh
