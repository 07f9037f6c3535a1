"""GPU: the multi-process self-play path end to end ("checked
against the single-GPU record set for the same seeds").

`python -m mzgo.selfplay` run as ONE process and as TWO ranks under
torch.distributed.run (games sharded by global id, weights broadcast from
rank 0, packed records gathered to rank 0) must write byte-identical pickled
batches (self_play.py:554-583's format).  On a one-GPU box both ranks share
cuda:0 and gloo stands in for RCCL (MZGO_SHARE_DEVICE / MZGO_DIST_BACKEND);
the sharding, broadcast, pack / gather and record ordering are the ones the
RCCL runs use.
"""
import filecmp
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, env, timeout=240):
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


def test_sharded_selfplay_cli_equals_single_process(tmp_path):
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "muzero-go_amd") + os.pathsep + os.environ.get("PYTHONPATH", ""),
               MZGO_SHARE_DEVICE="1", MZGO_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    args = ["--random-init", "0", "--board-size", "9", "--num_games", "10", "--simulations", "24",
            "--save-interval", "4"]
    one, two = tmp_path / "one", tmp_path / "two"
    _run([sys.executable, "-m", "mzgo.selfplay", *args, "--output_dir", str(one)], env)
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
          "--master-addr", "127.0.0.1", "--master-port", "29531", "-m", "mzgo.selfplay", *args,
          "--output_dir", str(two)], env)
    names = sorted(os.listdir(one))
    assert names and names == sorted(os.listdir(two))
    match, mismatch, errors = filecmp.cmpfiles(one, two, names, shallow=False)
    assert not mismatch and not errors, (mismatch, errors)
