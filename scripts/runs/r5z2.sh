export TMPDIR=/tmp
bash scripts/pmc_tcc.sh r5z --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5z_tcc.log 2>&1; rc=$?; tail -6 gpurun_out/r5z_tcc.log; exit $rc
