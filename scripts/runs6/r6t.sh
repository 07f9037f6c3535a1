# round 6: the move-parallel tests (injected-noise case added), then batch sizes of the queue (stamps build)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py -x -v --timeout 600 --timeout-method thread \
  -k "move_parallel" > gpurun_out/r6t_t.log 2>&1; rc=$?; grep -c PASSED gpurun_out/r6t_t.log; tail -2 gpurun_out/r6t_t.log; [ $rc -eq 0 ] || exit $rc
export MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so MZGO_MOVE_PARALLEL=1
timeout -k 10 300 python scripts/phases.py r6t_mp9 > gpurun_out/r6t_mp9.log 2>&1 || { tail -5 gpurun_out/r6t_mp9.log; exit 1; }
N=19 G=64 S=800 timeout -k 10 300 python scripts/phases.py r6t_mp19 > gpurun_out/r6t_mp19.log 2>&1 || { tail -5 gpurun_out/r6t_mp19.log; exit 1; }
python -c "
import json
for t in ('r6t_mp9','r6t_mp19'):
    d=json.load(open('gpurun_out/%s_phases.json'%t)); s=d['slots_sum']
    print(t, 'batches', s.get('48'), 'children', s.get('55'), 'mean B', s.get('55',0)/max(1,s.get('48',1)))"
