export TMPDIR=/tmp
for v in _agent ''; do
MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 60 python bench.py --board-size 19 --games 64 --sims 800 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5w$v.json 2> gpurun_out/r5w$v.err; echo "lib$v rc=$?"; tail -c 200 gpurun_out/r5w$v.json; echo
done
