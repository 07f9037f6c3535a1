# round 6, call i: the chain's own output chunk handed to the next layer in LDS (+ rotated cin order):
# tower suite, then config 5 A/B against the base build (libmzgo_base.so = the r6z build)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_tower.py > gpurun_out/r6i_t.log 2>&1; rc=$?; tail -3 gpurun_out/r6i_t.log; [ $rc -eq 0 ] || exit $rc
LIBS="'' _base" REPS=2 ARGS="--config 5 --no-cpu-baseline" bash scripts/gpu_ab.sh
