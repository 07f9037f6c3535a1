set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# factored dynamics only: the other bench configurations (1 GPU)
for cfg in "--board-size 9 --games 256 --sims 400" "--board-size 19 --games 64 --sims 800" "--board-size 19 --games 256 --sims 800"; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline $cfg > gpurun_out/b.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/b.log').read().splitlines()[-1]); print('$cfg', round(d['value']/1e6,2), 'M sims/s', round(d['ms_per_step'],2), 'ms/step')"
done
