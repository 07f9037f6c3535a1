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


def test_selfplay_cli_gpus_flag_starts_the_ranks(tmp_path):
    """``python -m mzgo.selfplay --gpus 2`` without a launcher: the CLI starts
    its two rank processes itself; same batches as one process."""
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "muzero-go_amd") + os.pathsep + os.environ.get("PYTHONPATH", ""),
               MZGO_SHARE_DEVICE="1", MZGO_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    args = ["--random-init", "0", "--board-size", "9", "--num_games", "6", "--simulations", "16",
            "--save-interval", "3"]
    one, two = tmp_path / "one", tmp_path / "two"
    _run([sys.executable, "-m", "mzgo.selfplay", *args, "--output_dir", str(one)], env)
    _run([sys.executable, "-m", "mzgo.selfplay", *args, "--gpus", "2", "--output_dir", str(two)], env)
    names = sorted(os.listdir(one))
    assert names and names == sorted(os.listdir(two))
    match, mismatch, errors = filecmp.cmpfiles(one, two, names, shallow=False)
    assert not mismatch and not errors, (mismatch, errors)


def test_bench_gpus_2_starts_two_ranks_and_gathers_every_epoch_once():
    """``bench.py --gpus 2`` as the driver runs it (no launcher): two rank
    processes (here both on cuda:0 with gloo standing in for RCCL), every
    timed epoch's records staged and gathered in one collective at the end
    of the timed loop, n_gpus 2 in the rank-0 line, the CPU
    baseline measured by the launcher before the ranks start, and no
    1-GPU counters or phase shares attached to the 2-GPU line."""
    import json
    env = dict(os.environ, MZGO_SHARE_DEVICE="1", MZGO_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MZGO_CPU_BASELINE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--cpu-budget", "2", "--cpu-procs", "2"], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3
    assert out["config"]["parallelism"] == "game-sharded x2"
    assert out["gather"]["count"] == 1 and out["gather"]["epochs_per_gather"] == 3
    assert out["gather"]["bytes_per_epoch_per_rank"] > 256 * 81 * 82 * 8
    assert out["gather"]["bytes_per_rank"] == 3 * out["gather"]["bytes_per_epoch_per_rank"]
    assert out["value"] > 0
    cb = out["cpu_baseline"]
    assert cb["cores"] == 2 and cb["value"] > 0 and cb["measured_in"].startswith("launcher"), cb
    assert "pmc_source" not in out["roofline"]["units"] and "phases" not in out, out["roofline"]
