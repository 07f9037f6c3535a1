export TMPDIR=/tmp
for v in _lg _lh; do
MZGO_LIB=muzero-go_amd/mzgo/libmzgo$v.so timeout -k 10 60 python bench.py --board-size 19 --games 64 --sims 800 --steps 1 --warmup 0 --moves-per-launch 1 --no-cpu-baseline > gpurun_out/r5q2$v.json 2> gpurun_out/r5q2$v.err; rc=$?; echo "lib$v rc=$rc $(tail -c 120 gpurun_out/r5q2$v.json)"
[ $rc -eq 124 ] || [ $rc -eq 137 ] && break
done
exit 0
