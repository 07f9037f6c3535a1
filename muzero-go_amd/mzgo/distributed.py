"""Multi-GPU self-play: one process per GPU, games sharded by global id, and
finished trajectories gathered to rank 0 over RCCL (torch.distributed
"nccl" on ROCm) -- the only collective on the data path.

The reference has no distribution layer (single process, one game at a time,
self_play.py:554-558); game sharding is sound because games never interact.

Records travel as one packed device buffer per rank (``mzgo_records_pack``,
layout in include/mzgo.h); rank 0 unpacks them into the reference's
GameHistory objects ordered by global game id.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from .launch import free_port, rank_envs, spawn_ranks  # noqa: F401  (re-exported)

FIELDS = ("stones", "invd", "flags", "action", "value", "policy", "reward", "meta", "status", "final")


def shard(num_games, world, rank):
    """Contiguous block of global game ids for ``rank``: (game_base, count)."""
    per = (num_games + world - 1) // world
    base = min(rank * per, num_games)
    return base, max(0, min(per, num_games - base))


def layout(G, M, N):
    """(name, dtype, shape, offset) of each field of the packed buffer, and its size."""
    C, A = N * N, N * N + 1
    spec = [("stones", np.int8, (G, M, C)), ("invd", np.uint8, (G, M, C)), ("flags", np.uint8, (G, M)),
            ("action", np.int32, (G, M)), ("value", np.float64, (G, M)), ("policy", np.float64, (G, M, A)),
            ("reward", np.float64, (G, M)), ("meta", np.int32, (G, 4)), ("status", np.int32, (G,)),
            ("final", np.float64, (G,))]
    out, off = [], 0
    for name, dt, shape in spec:
        nbytes = int(np.prod(shape)) * np.dtype(dt).itemsize
        out.append((name, dt, shape, off))
        off += (nbytes + 15) // 16 * 16
    return out, off


def unpack(buf, G, M, N):
    """Packed bytes (numpy uint8) -> dict of numpy arrays."""
    fields, total = layout(G, M, N)
    assert buf.nbytes >= total
    return {name: np.frombuffer(buf, dtype=dt, count=int(np.prod(shape)), offset=off).reshape(shape)
            for name, dt, shape, off in fields}


def slot_records(arrays, g):
    """Engine-record dict (as Engine.record returns) for slot g of unpacked arrays."""
    L = int(arrays["meta"][g, 3])
    return dict(length=L, status=int(arrays["status"][g]), stones=arrays["stones"][g, :L],
                invd=arrays["invd"][g, :L], flags=arrays["flags"][g, :L], action=arrays["action"][g, :L],
                value=arrays["value"][g, :L], policy=arrays["policy"][g, :L], reward=arrays["reward"][g, :L],
                final_reward=float(arrays["final"][g]))


def pack_engine(engine, out=None):
    """All slots' records of an mzgo Engine as one uint8 CUDA tensor (into
    ``out``, a contiguous uint8 CUDA tensor of exactly the packed size, if
    given: e.g. one epoch's slice of a staging buffer)."""
    from ._lib import check, lib, ptr, stream_of
    need = ctypes.c_int64()
    check(lib.mzgo_records_pack(engine.handle, None, 0, ctypes.byref(need), stream_of(engine.device)))
    if out is None:
        out = torch.empty(need.value, dtype=torch.uint8, device=engine.device)
    assert out.dtype == torch.uint8 and out.is_cuda and out.is_contiguous() and out.numel() == need.value
    check(lib.mzgo_records_pack(engine.handle, ptr(out), need.value, None, stream_of(engine.device)))
    return out


def gather_packed(buf, dst=0, group=None, to_host=True, async_op=False):
    """dist.gather of equal-size packed buffers to ``dst`` (device to device
    over RCCL for CUDA tensors); host numpy arrays there if ``to_host``.

    ``async_op``: return ``(work, parts)`` at once (parts None off ``dst``);
    the gather is ordered after the work already on the current stream (RCCL
    runs it on its own stream), ``work.wait()`` orders later work after it,
    and ``to_host`` is ignored (the device tensors are returned)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if buf.is_cuda and dist.get_backend(group) == "gloo":
        buf = buf.cpu()                       # gloo gathers host tensors (CPU tests, one-GPU rehearsals)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    work = dist.gather(buf, parts, dst=dst, group=group, async_op=async_op)
    if async_op:
        return work, parts
    if rank != dst:
        return None
    return [p.cpu().numpy() for p in parts] if to_host else parts


def broadcast_weights(module, src=0, group=None):
    """Give every rank ``src``'s network: the whole state_dict flattened into
    one f32 buffer and sent with a single broadcast (RCCL for CUDA modules;
    0.75 MB at C=96).  Parameters are updated in place."""
    sd = module.state_dict()
    keys = sorted(sd)
    dev = sd[keys[0]].device
    flat = torch.cat([sd[k].detach().reshape(-1).to(device=dev, dtype=torch.float32) for k in keys])
    dist.broadcast(flat, src=src, group=group)
    off = 0
    with torch.no_grad():
        for k in keys:
            n = sd[k].numel()
            sd[k].copy_(flat[off:off + n].view(sd[k].shape).to(sd[k].dtype))
            off += n
    return module


def gather_histories(engine, board_size, discount=0.99, dst=0, group=None):
    """Gather every rank's game records to ``dst`` as GameHistory objects,
    ordered by (rank, slot) == global game id under ``shard``."""
    from .selfplay import history_from_device
    parts = gather_packed(pack_engine(engine), dst=dst, group=group)
    if parts is None:
        return None
    out = []
    for p in parts:
        arrays = unpack(p, engine.G, engine.M, board_size)
        out.extend(history_from_device(slot_records(arrays, g), board_size, discount) for g in range(engine.G))
    return out
