"""GymGo board rules restated with numpy + scipy.ndimage (TEST INFRASTRUCTURE ONLY).

PARITY UNPINNED: GymGo (``huangeddie/GymGo``, installed by unpinned ``git
clone`` per README.md:7-13) is an empty submodule in the reference snapshot
and is not installed in this image; the reference has no board test or
fixture.  This file restates upstream master's published algorithm
(``gym_go/gogame.py``, ``gym_go/state_utils.py``, ``gym_go/govars.py``) as
summarised in SURVEY.md Appendix B, and is pinned only by the hand-written
known-answer positions in ``tests/test_oracle_gogame.py``.

Reference call sites: self_play.py:14 (govars), :152/:363 (INVD plane),
:479 (env.step -> next_state), :502/:513 (env.winner -> winning -> areas).

State: float64[6, N, N]; planes BLACK, WHITE, TURN (all 0 = black to move),
INVD (1 where the side to move may not play), PASS (previous move was a
pass), DONE.  Action a: a == N*N is pass, else (row, col) = divmod(a, N).
"""
import numpy as np
from scipy import ndimage

BLACK, WHITE, TURN_CHNL, INVD_CHNL, PASS_CHNL, DONE_CHNL = 0, 1, 2, 3, 4, 5
NUM_CHNLS = 6

# 4-neighbourhood without the centre (upstream state_utils.surround_struct)
_SURROUND = np.array([[0, 1, 0], [1, 0, 1], [0, 1, 0]])
_DELTAS = np.array([[-1, 0], [1, 0], [0, -1], [0, 1]])


def init_state(size):
    return np.zeros((NUM_CHNLS, size, size))


def turn(state):
    return int(np.max(state[TURN_CHNL]))


def prev_player_passed(state):
    return np.max(state[PASS_CHNL] == 1) == 1


def game_ended(state):
    return int(np.count_nonzero(state[DONE_CHNL] == 1) > 0)


def action_size(state):
    return state.shape[1] * state.shape[2] + 1


def invalid_moves(state):
    if game_ended(state):
        return np.zeros(action_size(state))
    return np.append(state[INVD_CHNL].flatten(), 0)


def _neighbours(size, rc):
    nb = _DELTAS + np.asarray(rc)
    keep = np.all((nb >= 0) & (nb < size), axis=1)
    return nb[keep]


def _liberty_maps(groups, count, empties, struct):
    """[count, N, N] liberty indicator per labelled group."""
    libs = np.zeros((count,) + empties.shape)
    for g in range(count):
        libs[g] = empties * ndimage.binary_dilation(groups == (g + 1), struct)
    return libs


def compute_invalid_moves(state, player, ko_protect=None):
    """INVD plane for the opponent of ``player`` (upstream state_utils).

    Occupied points are invalid.  An empty point is invalid when it is
    surrounded on all four sides (off-board counts as occupied) and it is a
    liberty of a ``player`` group with >1 liberty or of an opponent group with
    exactly 1 liberty, and not a liberty of a ``player`` group in atari (a
    capture) or of an opponent group with >1 liberty.  The ko point, if any,
    is invalid too.
    """
    occupied = state[BLACK] + state[WHITE]
    empties = 1 - occupied
    own, n_own = ndimage.label(state[player])
    opp, n_opp = ndimage.label(state[1 - player])
    own_libs = _liberty_maps(own, n_own, empties, _SURROUND)
    opp_libs = _liberty_maps(opp, n_opp, empties, _SURROUND)
    own_cnt = own_libs.sum(axis=(1, 2))
    opp_cnt = opp_libs.sum(axis=(1, 2))

    maybe_bad = own_libs[own_cnt > 1].sum(axis=0) + opp_libs[opp_cnt == 1].sum(axis=0)
    surely_ok = own_libs[own_cnt == 1].sum(axis=0) + opp_libs[opp_cnt > 1].sum(axis=0)
    boxed_in = ndimage.convolve(occupied, _SURROUND, mode="constant", cval=1) == 4
    invalid = occupied + maybe_bad * (surely_ok == 0) * boxed_in
    if ko_protect is not None:
        invalid[ko_protect[0], ko_protect[1]] = 1
    return invalid > 0


def _capture(state, adj, player):
    """Remove opponent groups adjacent to the new stone that have no liberty.

    Liberties are measured on the board as it stands after placement and
    before any removal (upstream state_utils.update_pieces).
    """
    opponent = 1 - player
    empties = 1 - (state[BLACK] + state[WHITE])
    labels, _ = ndimage.label(state[opponent])
    killed = []
    touching = np.unique(labels[adj[:, 0], adj[:, 1]])
    for lab in touching[touching != 0]:
        grp = labels == lab
        if np.sum(empties * ndimage.binary_dilation(grp)) <= 0:
            pts = np.argwhere(grp)
            state[opponent, pts[:, 0], pts[:, 1]] = 0
            killed.append(pts)
    return killed


def next_state(state, action1d, canonical=False):
    if canonical:
        raise NotImplementedError("self_play.py uses canonical=False only")
    state = np.copy(state)
    size = state.shape[1]
    player = turn(state)
    ko_protect = None

    if action1d == size * size:                       # pass
        already = prev_player_passed(state)
        state[PASS_CHNL] = 1
        if already:
            state[DONE_CHNL] = 1
    else:
        r, c = action1d // size, action1d % size
        state[PASS_CHNL] = 0
        assert state[INVD_CHNL, r, c] == 0, ("Invalid move", (r, c))
        state[player, r, c] = 1
        adj = _neighbours(size, (r, c))
        boxed = bool((state[1 - player][adj[:, 0], adj[:, 1]] > 0).all())
        killed = _capture(state, adj, player)
        if len(killed) == 1 and boxed and len(killed[0]) == 1:
            ko_protect = killed[0][0]

    state[INVD_CHNL] = compute_invalid_moves(state, player, ko_protect)
    state[TURN_CHNL] = 1 - state[TURN_CHNL]
    return state


def areas(state):
    """Area (Tromp-Taylor) counts: stones + empty regions bordering one colour."""
    empties = 1 - (state[BLACK] + state[WHITE])
    regions, n = ndimage.label(empties)
    black, white = np.sum(state[BLACK]), np.sum(state[WHITE])
    for lab in range(1, n + 1):
        region = regions == lab
        rim = ndimage.binary_dilation(region)
        b = (state[BLACK] * rim > 0).any()
        w = (state[WHITE] * rim > 0).any()
        if b and not w:
            black += np.sum(region)
        elif w and not b:
            white += np.sum(region)
    return black, white


def winning(state, komi=0):
    black, white = areas(state)
    return np.sign(black - white - komi)
