# round 6, call a: the L1 visibility probe, the chain (config-5 shape) and
# compat "fixed" parity tests, the config-5 and default lines after the
# dma16_l2 sc0 -> sc1 change, and the host's CPU affinity
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import os, json; print(json.dumps({'cpu_count': os.cpu_count(), 'affinity': len(os.sched_getaffinity(0))}))" > gpurun_out/r6a_cpus.json; cat gpurun_out/r6a_cpus.json; nproc
timeout -k 10 60 tools/l1_visibility_probe > gpurun_out/r6a_probe.json 2>&1; rc=$?; cat gpurun_out/r6a_probe.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python -u -m pytest -x -v --timeout 800 --timeout-method thread \
  tests/test_gpu_tower.py::test_tower_chain_equals_per_conv_config5 \
  tests/test_gpu_tower.py::test_tower_chain_launch_equals_per_conv_launches \
  tests/test_gpu_selfplay.py::test_fixed_compat_games_match_oracle > gpurun_out/r6a_t.log 2>&1; rc=$?; tail -8 gpurun_out/r6a_t.log; [ $rc -eq 0 ] || exit $rc
TAG=r6a LINES="c5 bench" bash scripts/gpu_lines.sh
