export TMPDIR=/tmp
bash scripts/runs/r5ak.sh || exit 1
LIBS="'' _xg5 _xg10" REPS=2 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh && LIBS="'' _xg5 _xg10" REPS=1 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
