export TMPDIR=/tmp
LIBS="'' _p3 _p4 _p5 _p6" REPS=2 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh
