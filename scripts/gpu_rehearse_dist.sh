#!/bin/bash
# Rehearsal of bench.py's N>1 path on a one-GPU box: 2 ranks under
# torch.distributed.run, both on cuda:0, gloo instead of RCCL
# (MZGO_SHARE_DEVICE / MZGO_DIST_BACKEND; the driver's runs use neither).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp MZGO_SHARE_DEVICE=1 MZGO_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/rehearse2.log 2>&1 || { tail -30 gpurun_out/rehearse2.log; exit 1; }
tail -1 gpurun_out/rehearse2.log | cut -c1-400
# the self-play CLI: 2 ranks x 6 games vs one process x 12 games, same seeds:
# the pickled batches must be byte-identical (games keyed by global id)
export PYTHONPATH=$PWD/muzero-go_amd:${PYTHONPATH:-}
rm -rf gpurun_out/sp1 gpurun_out/sp2
timeout -k 10 300 python -m mzgo.selfplay --random-init 0 --board-size 9 --num_games 12 --simulations 32 --save-interval 4 --output_dir gpurun_out/sp1 > gpurun_out/sp1.log 2>&1 || { tail -20 gpurun_out/sp1.log; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 -m mzgo.selfplay --random-init 0 --board-size 9 --num_games 12 --simulations 32 --save-interval 4 --output_dir gpurun_out/sp2 > gpurun_out/sp2.log 2>&1 || { tail -30 gpurun_out/sp2.log; exit 1; }
ls gpurun_out/sp1 gpurun_out/sp2
diff -r gpurun_out/sp1 gpurun_out/sp2 && echo "sharded self-play == single-process self-play (byte-identical batches)"
