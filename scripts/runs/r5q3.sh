export TMPDIR=/tmp
LIBS="'' _lg" REPS=2 LIMIT=120 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
