set -e
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5j_t.log 2>&1 || { tail -40 gpurun_out/r5j_t.log; exit 1; }
tail -1 gpurun_out/r5j_t.log
timeout -k 10 400 python bench.py --cpu-budget 8 > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err || { tail -5 gpurun_out/r5j_bench.err; exit 1; }
tail -1 gpurun_out/r5j_bench.json | cut -c1-300
timeout -k 10 400 python bench.py --config 5 --cpu-budget 8 > gpurun_out/r5j_c5.json 2> gpurun_out/r5j_c5.err || { tail -5 gpurun_out/r5j_c5.err; exit 1; }
tail -1 gpurun_out/r5j_c5.json | cut -c1-300
timeout -k 10 400 python bench.py --config 5 --moves-per-step 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5j_c5seg.json 2> gpurun_out/r5j_c5seg.err || { tail -5 gpurun_out/r5j_c5seg.err; exit 1; }
tail -1 gpurun_out/r5j_c5seg.json | cut -c1-300
