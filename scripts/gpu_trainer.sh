set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_train.log 2>&1; rc=$?
tail -30 gpurun_out/t_train.log
exit $rc
