# round 6, call j: config 5 A/B -- '' = rotated cin order + LDS hand-off, _rot = rotated order only, _base = r6z build
LIBS="'' _rot _base" REPS=3 ARGS="--config 5 --no-cpu-baseline" bash scripts/gpu_ab.sh
