export TMPDIR=/tmp
TAG=r5zz2 LINES="19_64" bash scripts/gpu_lines.sh || exit 1
A="--board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline"
bash scripts/pmc.sh r5zz2_19_64 $A > gpurun_out/r5zz2_pmc.log 2>&1 || { tail -5 gpurun_out/r5zz2_pmc.log; exit 1; }
bash scripts/pmc_tcc.sh r5zz2_19_64 $A > gpurun_out/r5zz2_tcc.log 2>&1; rc=$?; tail -2 gpurun_out/r5zz2_tcc.log; exit $rc
