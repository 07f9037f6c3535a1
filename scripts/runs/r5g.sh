set -e
export TMPDIR=/tmp
timeout -k 10 600 python scripts/trainer_timing.py > gpurun_out/r5g_trainer.json 2> gpurun_out/r5g_trainer.err || { tail -20 gpurun_out/r5g_trainer.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5g_trainer.json')); print({k: d[k] for k in ('hip_ms','torch_miopen_ms','network_fwd_bwd')})"
bash scripts/pmc_tcc.sh r5g_19_64 --board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline
bash scripts/pmc_tcc.sh r5g_head --steps 2 --warmup 1 --no-cpu-baseline
bash scripts/pmc.sh r5g_19_64 --board-size 19 --games 64 --sims 800 --steps 1 --warmup 1 --no-cpu-baseline
bash scripts/pmc.sh r5g_head --steps 2 --warmup 1 --no-cpu-baseline
