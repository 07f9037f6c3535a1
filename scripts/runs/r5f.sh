set -e
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/r5f_avail.txt 2>&1 || true
grep -c . gpurun_out/r5f_avail.txt || true
timeout -k 10 600 python scripts/trainer_timing.py > gpurun_out/r5f_trainer.json 2> gpurun_out/r5f_trainer.err || { tail -20 gpurun_out/r5f_trainer.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5f_trainer.json')); print({k: d[k] for k in ('hip_ms','torch_miopen_ms','speedup_hip_over_torch')})"
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f_t.log 2>&1 || { tail -30 gpurun_out/r5f_t.log; exit 1; }
tail -1 gpurun_out/r5f_t.log
