"""Deterministic MuZeroNet weights (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Fixtures and benchmarks need weights of the reference architecture
(self_play.py:63-128) that every side can regenerate without shipping a
checkpoint.  Each tensor of the state_dict (keys and order exactly as the
reference module registers them) is drawn from the counter RNG of
``oracle/rng.py``:

    key  = stream_key(seed, WEIGHT_GAME, param_index)
    u24  = draw(key, TAG_WEIGHT, element) >> 40            (int in [0, 2**24))
    w    = f32((u24 - 2**23) / 2**23) * f32(bound)          (one f32 rounding)

with ``bound = f32(1/sqrt(fan_in))`` as PyTorch's default Conv2d/Linear
initialisation uses (fan_in of the weight for the bias too), 1.0 for the
embedding and 0.5 for ``pass_logit`` (zero-initialised in the reference; a
non-zero value keeps the pass-logit path covered by parity tests).
``mzgo/weights.py`` restates the same generator for the product's
``--random-init``; a CPU test checks the two agree bit-for-bit.
"""
import math
from collections import OrderedDict

import numpy as np

from .rng import TAG_WEIGHT, WEIGHT_GAME, draw_np, stream_key


def param_specs(latent_dim, action_size):
    """(key, shape, bound) in the reference's state_dict order."""
    C, A = latent_dim, action_size

    def b(fan_in):
        return float(np.float32(1.0 / math.sqrt(fan_in)))

    return [
        ("representation.conv1.weight", (64, 6, 3, 3), b(6 * 9)),
        ("representation.conv1.bias", (64,), b(6 * 9)),
        ("representation.conv2.weight", (64, 64, 3, 3), b(64 * 9)),
        ("representation.conv2.bias", (64,), b(64 * 9)),
        ("representation.conv3.weight", (C, 64, 3, 3), b(64 * 9)),
        ("representation.conv3.bias", (C,), b(64 * 9)),
        ("dynamics.action_embedding.weight", (A, C), 1.0),
        ("dynamics.conv.weight", (C, C, 3, 3), b(C * 9)),
        ("dynamics.conv.bias", (C,), b(C * 9)),
        ("dynamics.reward_conv.weight", (1, C, 1, 1), b(C)),
        ("dynamics.reward_conv.bias", (1,), b(C)),
        ("dynamics.fc_reward_hidden.weight", (16, 1), b(1)),
        ("dynamics.fc_reward_hidden.bias", (16,), b(1)),
        ("dynamics.fc_reward_output.weight", (1, 16), b(16)),
        ("dynamics.fc_reward_output.bias", (1,), b(16)),
        ("prediction.pass_logit", (1,), 0.5),
        ("prediction.value_conv.weight", (1, C, 1, 1), b(C)),
        ("prediction.value_conv.bias", (1,), b(C)),
        ("prediction.value_fc.weight", (1, 1), b(1)),
        ("prediction.value_fc.bias", (1,), b(1)),
        ("prediction.policy_conv.weight", (1, C, 1, 1), b(C)),
        ("prediction.policy_conv.bias", (1,), b(C)),
    ]


def deterministic_state_dict(latent_dim, action_size, seed=0):
    """OrderedDict[str, np.ndarray(float32)] loadable into the reference net."""
    out = OrderedDict()
    for p, (key, shape, bound) in enumerate(param_specs(latent_dim, action_size)):
        n = int(np.prod(shape))
        k = stream_key(seed, WEIGHT_GAME, p)
        h = draw_np(k, TAG_WEIGHT, np.arange(n, dtype=np.uint64))
        u24 = (h >> np.uint64(40)).astype(np.int64)
        unit = ((u24 - (1 << 23)).astype(np.float32) / np.float32(1 << 23)).astype(np.float32)
        out[key] = (unit * np.float32(bound)).astype(np.float32).reshape(shape)
    return out
