"""Random legal positions for fixtures and tests (TEST INFRASTRUCTURE ONLY)."""
import numpy as np

from . import gogame


def random_position(size, moves, seed):
    """A legal position reached by uniform random board moves on the oracle board."""
    rng = np.random.default_rng(seed)
    st = gogame.init_state(size)
    for _ in range(moves):
        if gogame.game_ended(st):
            break
        legal = np.flatnonzero(gogame.invalid_moves(st) == 0)
        legal = legal[legal < size * size]
        if len(legal) == 0:
            break
        st = gogame.next_state(st, int(rng.choice(legal)))
    return st
