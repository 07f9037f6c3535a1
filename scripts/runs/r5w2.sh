export TMPDIR=/tmp
LIBS="'' _agent" REPS=2 LIMIT=150 ARGS="--board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --moves-per-launch 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
