"""Multi-process checks of the game-sharded path on the CPU (gloo backend,
world_size 2): sharding by global game id and the trajectory gather to rank 0
(the only collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mzgo import distributed as mdist

N, G, M = 5, 3, 7


def test_shard_covers_every_game_once():
    for games, world in ((512, 8), (2048, 8), (10, 3), (7, 8), (1, 2)):
        seen = []
        for r in range(world):
            base, n = mdist.shard(games, world, r)
            seen.extend(range(base, base + n))
        assert seen == list(range(games))


def synthetic_buffer(rank):
    """A packed buffer as mzgo_records_pack lays it out, game content keyed by
    global game id = rank * G + slot."""
    fields, total = mdist.layout(G, M, N)
    buf = np.zeros(total, np.uint8)
    arr = {name: np.frombuffer(buf, dtype=dt, count=int(np.prod(shape)), offset=off).reshape(shape)
           for name, dt, shape, off in fields}
    for g in range(G):
        gid = rank * G + g
        L = 2 + gid % 5
        arr["meta"][g] = (gid % 2, 0, 0, L)
        arr["status"][g] = 1
        arr["action"][g, :L] = gid
        arr["value"][g, :L] = gid / 10.0
        arr["policy"][g, :L] = 1.0 / (N * N + 1)
        arr["stones"][g, :L, gid % (N * N)] = 1
        arr["final"][g] = 0.0
    return buf


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        parts = mdist.gather_packed(torch.from_numpy(synthetic_buffer(rank)))
        if rank == 0:
            from mzgo.selfplay import history_from_device
            hists = []
            for p in parts:
                a = mdist.unpack(p, G, M, N)
                hists.extend(history_from_device(mdist.slot_records(a, g), N, 0.99) for g in range(G))
            out.put([(h.actions, h.values, len(h)) for h in hists])
        else:
            assert parts is None
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gather_records_to_rank0_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(got) == world * G
    for gid, (actions, values, length) in enumerate(got):
        assert length == 2 + gid % 5
        assert actions == [gid] * length
        assert values == [gid / 10.0] * length


def _bcast_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mzgo
        net = mzgo.MuZeroNet(96, N * N + 1)
        net.load_state_dict(mzgo.deterministic_state_dict(96, N * N + 1, rank))   # ranks differ
        mdist.broadcast_weights(net, src=0)
        want = mzgo.deterministic_state_dict(96, N * N + 1, 0)
        got = net.state_dict()
        out.put((rank, max(float((got[k] - torch.as_tensor(want[k])).abs().max()) for k in want)))
    finally:
        dist.destroy_process_group()


def test_broadcast_weights_gloo():
    """Every rank ends with rank 0's network after one flattened broadcast."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == {0: 0.0, 1: 0.0}


def test_rank_envs_as_torchrun_sets_them():
    """bench.py --gpus N / mzgo.selfplay --gpus N without a launcher: the
    environment each rank process gets (the one torch.distributed.run gives)."""
    from mzgo.launch import rank_envs
    base = {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "PATH": "/usr/bin", "KEEP": "x"}
    envs = rank_envs(8, base, master_port=29999)
    assert len(envs) == 8
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "8", "8")
        assert (e["MASTER_ADDR"], e["MASTER_PORT"]) == ("127.0.0.1", "29999")
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["KEEP"] == "x"
    assert "RANK" not in base                       # the parent's environment is not modified
    ports = {e["MASTER_PORT"] for e in rank_envs(2, base)}
    assert len(ports) == 1 and int(ports.pop()) > 0


def test_spawn_ranks_runs_every_rank(tmp_path):
    import sys
    from mzgo.launch import spawn_ranks
    code = ("import os, pathlib; e = os.environ; "
            "pathlib.Path(r'%s', e['RANK']).write_text(','.join(e[k] for k in "
            "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR')))" % tmp_path)
    assert spawn_ranks(3, [sys.executable, "-c", code]) == 0
    got = sorted(p.read_text() for p in tmp_path.iterdir())
    assert got == [f"{r},{r},3,127.0.0.1" for r in range(3)]


def test_spawn_ranks_stops_the_others_when_a_rank_fails():
    """A failed rank ends the run with its status; a peer stuck (e.g. in a
    collective) is terminated instead of outliving it."""
    import sys
    import time
    from mzgo.launch import spawn_ranks
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(0.5) if r == 1 else time.sleep(600); " \
           "sys.exit(3)"
    t0 = time.time()
    assert spawn_ranks(2, [sys.executable, "-c", code]) == 3
    assert time.time() - t0 < 60


def _per_epoch_worker(rank, world, port, out):
    """Several asynchronous gathers in flight (mzgo.selfplay's per-batch
    gathers), waited on at the end: rank 0 holds each one's buffers from
    every rank, in order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        works = []
        for epoch in range(3):
            buf = torch.full((64,), 10 * epoch + rank, dtype=torch.uint8)
            works.append(mdist.gather_packed(buf, async_op=True))
        for w, _ in works:
            w.wait()
        if rank == 0:
            out.put([[int(p[0]) for p in parts] for _, parts in works])
        else:
            assert all(parts is None for _, parts in works)
    finally:
        dist.destroy_process_group()


def test_gather_every_epoch_async_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_per_epoch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [[0, 1], [10, 11], [20, 21]]


def _staged_worker(rank, world, port, out):
    """bench.py's timed loop: every epoch's packed records into its slice of
    a staging buffer, ONE gather at the end; rank 0 splits each rank's part
    back into epochs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        steps, per = 3, 64
        staged = torch.empty(steps * per, dtype=torch.uint8)
        for epoch in range(steps):
            staged[epoch * per:(epoch + 1) * per] = 10 * epoch + rank
        work, parts = mdist.gather_packed(staged, async_op=True)
        work.wait()
        if rank == 0:
            out.put([[int(p[e * per]) for p in parts] for e in range(steps)])
        else:
            assert parts is None
    finally:
        dist.destroy_process_group()


def test_staged_epochs_one_gather_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_staged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [[0, 1], [10, 11], [20, 21]]
