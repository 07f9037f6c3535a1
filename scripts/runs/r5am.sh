export TMPDIR=/tmp
LIBS="'' _pn _ph _pf" REPS=2 ARGS="--steps 10 --no-cpu-baseline" bash scripts/gpu_ab.sh && LIBS="'' _pn _ph _pf" REPS=1 LIMIT=200 ARGS="--board-size 19 --games 64 --sims 800 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_ab.sh
