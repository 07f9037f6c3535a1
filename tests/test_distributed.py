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
