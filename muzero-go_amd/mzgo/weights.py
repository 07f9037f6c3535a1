"""Deterministic reference-architecture weights for ``--random-init SEED``.

The generator (counter RNG of include/mzgo.h's engine, PyTorch-default
scaling) is defined in oracle/weights.py; this is the product's own copy of
the same definition (tests check the two agree bit-for-bit):

    key = stream_key(seed, 0xFFFFFFFF, param_index)
    u24 = draw(key, 4, element) >> 40
    w   = f32((u24 - 2**23) / 2**23) * f32(bound)
"""
import math
from collections import OrderedDict

import numpy as np

_GOLDEN, _C1, _C2 = 0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB
_M64 = (1 << 64) - 1


def _mix(z):
    z = (z + _GOLDEN) & _M64
    z = ((z ^ (z >> 30)) * _C1) & _M64
    z = ((z ^ (z >> 27)) * _C2) & _M64
    return z ^ (z >> 31)


def _mix_np(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(_GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_C1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_C2)
    return z ^ (z >> np.uint64(31))


def _specs(C, A):
    def b(fan_in):
        return float(np.float32(1.0 / math.sqrt(fan_in)))
    return [
        ("representation.conv1.weight", (64, 6, 3, 3), b(54)), ("representation.conv1.bias", (64,), b(54)),
        ("representation.conv2.weight", (64, 64, 3, 3), b(576)), ("representation.conv2.bias", (64,), b(576)),
        ("representation.conv3.weight", (C, 64, 3, 3), b(576)), ("representation.conv3.bias", (C,), b(576)),
        ("dynamics.action_embedding.weight", (A, C), 1.0),
        ("dynamics.conv.weight", (C, C, 3, 3), b(C * 9)), ("dynamics.conv.bias", (C,), b(C * 9)),
        ("dynamics.reward_conv.weight", (1, C, 1, 1), b(C)), ("dynamics.reward_conv.bias", (1,), b(C)),
        ("dynamics.fc_reward_hidden.weight", (16, 1), b(1)), ("dynamics.fc_reward_hidden.bias", (16,), b(1)),
        ("dynamics.fc_reward_output.weight", (1, 16), b(16)), ("dynamics.fc_reward_output.bias", (1,), b(16)),
        ("prediction.pass_logit", (1,), 0.5),
        ("prediction.value_conv.weight", (1, C, 1, 1), b(C)), ("prediction.value_conv.bias", (1,), b(C)),
        ("prediction.value_fc.weight", (1, 1), b(1)), ("prediction.value_fc.bias", (1,), b(1)),
        ("prediction.policy_conv.weight", (1, C, 1, 1), b(C)), ("prediction.policy_conv.bias", (1,), b(C)),
    ]


def deterministic_state_dict(latent_dim, action_size, seed=0):
    import torch
    out = OrderedDict()
    for p, (key, shape, bound) in enumerate(_specs(latent_dim, action_size)):
        n = int(np.prod(shape))
        k = _mix(_mix(seed & _M64) ^ ((0xFFFFFFFF << 32) | p))
        idx = np.arange(n, dtype=np.uint64) & np.uint64((1 << 56) - 1)
        h = _mix_np(np.uint64(k) ^ np.uint64(4 << 56) ^ idx)
        u24 = (h >> np.uint64(40)).astype(np.int64)
        unit = ((u24 - (1 << 23)).astype(np.float32) / np.float32(1 << 23)).astype(np.float32)
        out[key] = torch.from_numpy((unit * np.float32(bound)).astype(np.float32).reshape(shape))
    return out


def res_specs(latent_dim, action_size, blocks):
    """(key, shape, bound) of ``mzgo.resnet.ResMuZeroNet`` (BASELINE config 5)
    in its state_dict order; bounds as PyTorch's default initialisation."""
    C, A = latent_dim, action_size

    def b(fan_in):
        return float(np.float32(1.0 / math.sqrt(fan_in)))

    def conv(k, co, ci):
        return [(k + ".weight", (co, ci, 3, 3), b(ci * 9)), (k + ".bias", (co,), b(ci * 9))]

    s = conv("representation.conv_in", C, 6)
    for i in range(blocks):
        s += conv(f"representation.blocks.{i}.conv1", C, C) + conv(f"representation.blocks.{i}.conv2", C, C)
    s += [("dynamics.action_embedding.weight", (A, C), 1.0)]
    s += conv("dynamics.conv_in", C, C)
    for i in range(blocks):
        s += conv(f"dynamics.blocks.{i}.conv1", C, C) + conv(f"dynamics.blocks.{i}.conv2", C, C)
    s += [
        ("dynamics.reward_conv.weight", (1, C, 1, 1), b(C)), ("dynamics.reward_conv.bias", (1,), b(C)),
        ("dynamics.fc_reward_hidden.weight", (16, 1), b(1)), ("dynamics.fc_reward_hidden.bias", (16,), b(1)),
        ("dynamics.fc_reward_output.weight", (1, 16), b(16)), ("dynamics.fc_reward_output.bias", (1,), b(16)),
        ("prediction.pass_logit", (1,), 0.5),
        ("prediction.value_conv.weight", (1, C, 1, 1), b(C)), ("prediction.value_conv.bias", (1,), b(C)),
        ("prediction.value_fc.weight", (1, 1), b(1)), ("prediction.value_fc.bias", (1,), b(1)),
        ("prediction.policy_conv.weight", (1, C, 1, 1), b(C)), ("prediction.policy_conv.bias", (1,), b(C)),
    ]
    return s


def deterministic_res_state_dict(latent_dim, action_size, blocks, seed=0):
    """Weights of the residual-tower network from the same counter generator
    (parameter index = position in ``res_specs``)."""
    import torch
    out = OrderedDict()
    for p, (key, shape, bound) in enumerate(res_specs(latent_dim, action_size, blocks)):
        n = int(np.prod(shape))
        k = _mix(_mix(seed & _M64) ^ ((0xFFFFFFFF << 32) | p))
        idx = np.arange(n, dtype=np.uint64) & np.uint64((1 << 56) - 1)
        h = _mix_np(np.uint64(k) ^ np.uint64(4 << 56) ^ idx)
        u24 = (h >> np.uint64(40)).astype(np.int64)
        unit = ((u24 - (1 << 23)).astype(np.float32) / np.float32(1 << 23)).astype(np.float32)
        out[key] = torch.from_numpy((unit * np.float32(bound)).astype(np.float32).reshape(shape))
    return out
