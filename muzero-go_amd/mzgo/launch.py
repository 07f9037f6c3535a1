"""One process per GPU without a launcher: ``spawn_ranks(n, argv)`` starts n
fresh child processes with the environment torch.distributed.run would give
them (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), so ``bench.py --gpus N`` and
``python -m mzgo.selfplay --gpus N`` run N ranks by themselves.

Standard library only, and importable by file path (bench.py does that before
anything loads libmzgo.so or touches a GPU): the parent never initialises the
GPU and never execs itself -- every rank is a new process.
"""
import os


def free_port(host="127.0.0.1"):
    import socket
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def rank_envs(n, base_env=None, master_port=None, master_addr="127.0.0.1"):
    """The environment of each of ``n`` ranks on one node, as
    torch.distributed.run sets it: RANK = LOCAL_RANK = r, WORLD_SIZE =
    LOCAL_WORLD_SIZE = n, MASTER_ADDR / MASTER_PORT (127.0.0.1: the container
    hostname may not resolve).  Everything else is inherited from
    ``base_env`` (HSA_ENABLE_IPC_MODE_LEGACY=0 included)."""
    base = dict(os.environ if base_env is None else base_env)
    port = master_port or free_port(master_addr)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR=master_addr, MASTER_PORT=str(port))
        envs.append(e)
    return envs


def spawn_ranks(n, cmd, base_env=None, master_port=None, poll_s=0.2):
    """Run ``cmd`` (argv list) as ``n`` fresh child processes, one per rank /
    GPU (``rank_envs``), and return the exit status: 0 if every rank exited 0,
    else the first failing rank's status -- the others are then terminated
    (their process groups), so a rank stuck in a collective cannot outlive a
    failed peer.  The caller must not have touched the GPU: children are new
    processes (subprocess), never an exec of this one."""
    import signal
    import subprocess
    import time
    procs = [subprocess.Popen(cmd, env=e, start_new_session=True)
             for e in rank_envs(n, base_env, master_port)]
    status = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    for q in live:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
    return status
