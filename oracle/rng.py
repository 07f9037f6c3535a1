"""Counter-based RNG streams (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

The reference draws from CPython ``random`` (MT19937: ``random.choice`` at
self_play.py:287 and :388) and numpy's legacy global ``RandomState``
(``np.random.dirichlet`` at :38, ``np.random.choice`` at :400).  Thousands of
concurrent games on the GPU cannot share one sequential stream, so the engine
uses a stateless counter-based generator keyed by (seed, game, move, purpose,
index).  This module restates that generator bit-for-bit; the oracle installs
it as the hook for the reference's draws so that engine and oracle make the
same choices.  The same definition lives in
``muzero-go_amd/csrc/mzgo_rng.hpp`` (device) and ``mzgo/weights.py``.

    mix64(z)            splitmix64 finaliser with the golden-gamma increment
    stream_key(s,g,m) = mix64(mix64(s) ^ (g << 32 | m))
    draw(k, tag, i)   = mix64(k ^ (tag << 56) ^ i)          (i < 2**56)
    u01(h)            = (h >> 11) * 2**-53                   (float64 in [0,1))
    randbelow(h, n)   = ((h >> 32) * n) >> 32                (int in [0,n))
"""
import numpy as np

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
C1 = 0xBF58476D1CE4E5B9
C2 = 0x94D049BB133111EB

TAG_SELECT = 1     # idx = sim                   (unexpanded-child pick, :287;
                   #  select_leaf returns right after it, so one per sim)
TAG_DIRICHLET = 2  # idx = a << 16 | draw number (root noise, :38)
TAG_ACTION = 3     # idx = 0                     (move choice, :388 / :400)
TAG_WEIGHT = 4     # idx = element               (deterministic init)

WEIGHT_GAME = 0xFFFFFFFF  # stream_key(seed, WEIGHT_GAME, param_index)


def mix64(z):
    z = (z + GOLDEN) & M64
    z = ((z ^ (z >> 30)) * C1) & M64
    z = ((z ^ (z >> 27)) * C2) & M64
    return z ^ (z >> 31)


def stream_key(seed, game, move):
    return mix64(mix64(seed & M64) ^ (((game & 0xFFFFFFFF) << 32) | (move & 0xFFFFFFFF)))


def draw(key, tag, idx):
    return mix64(key ^ ((tag & 0xFF) << 56) ^ (idx & ((1 << 56) - 1)))


def u01(h):
    return float(h >> 11) * (2.0 ** -53)


def randbelow(h, n):
    return ((h >> 32) * n) >> 32


# ---- vectorised forms (numpy uint64 arithmetic wraps modulo 2**64) ----

def mix64_np(z):
    z = z.astype(np.uint64)
    with np.errstate(over='ignore'):
        z = z + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(C1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(C2)
    return z ^ (z >> np.uint64(31))


def draw_np(key, tag, idx):
    idx = np.asarray(idx, dtype=np.uint64) & np.uint64((1 << 56) - 1)
    return mix64_np(np.uint64(key) ^ np.uint64((tag & 0xFF) << 56) ^ idx)


class SearchHooks:
    """Deterministic replacements for the reference's RNG draws in one move.

    ``choice_index(n, sim)`` replaces ``random.choice`` in select_leaf
    (self_play.py:287); ``action_uniform()`` the uniform behind
    ``np.random.choice`` / ``random.choice`` in select_action (:388, :400).
    """

    def __init__(self, seed, game, move):
        self.key = stream_key(seed, game, move)

    def choice_index(self, n, sim):
        return randbelow(draw(self.key, TAG_SELECT, sim), n)

    def action_uniform(self):
        return u01(draw(self.key, TAG_ACTION, 0))

    def action_index(self, n):
        return randbelow(draw(self.key, TAG_ACTION, 0), n)


def injected_noise(seed, game, move, n):
    """Deterministic stand-in for ``np.random.dirichlet([alpha]*n)`` used by
    parity fixtures: strictly positive, float64, normalised with numpy's sum."""
    key = stream_key(seed, game, move)
    u = np.array([u01(draw(key, TAG_DIRICHLET, a << 16)) for a in range(n)]) + 2.0 ** -20
    return u / u.sum()
