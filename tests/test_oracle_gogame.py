"""Known-answer positions for the GymGo restatement (board parity is unpinned
by the reference: GymGo is absent and untested there -- see oracle/gogame.py).

Boards are written as strings: ``B``/``W`` stones, ``.`` empty, row 0 first.
"""
import numpy as np
import pytest

from oracle import gogame as gg
from oracle.goenv import GoEnv


def board(rows, to_move="B"):
    n = len(rows)
    st = gg.init_state(n)
    for r, row in enumerate(rows):
        for c, ch in enumerate(row.replace(" ", "")):
            if ch == "B":
                st[gg.BLACK, r, c] = 1
            elif ch == "W":
                st[gg.WHITE, r, c] = 1
    mover_before = 1 if to_move == "B" else 0      # INVD is for the side to move
    st[gg.INVD_CHNL] = gg.compute_invalid_moves(st, mover_before)
    st[gg.TURN_CHNL] = 0 if to_move == "B" else 1
    return st


def play(st, r, c=None):
    n = st.shape[1]
    return gg.next_state(st, n * n if r is None else r * n + c)


def stones(st):
    out = []
    for r in range(st.shape[1]):
        out.append("".join("B" if st[0, r, c] else "W" if st[1, r, c] else "."
                           for c in range(st.shape[2])))
    return out


def test_empty_board_all_legal_black_first():
    st = gg.init_state(9)
    assert gg.turn(st) == 0 and not gg.invalid_moves(st).any()


def test_single_capture_centre():
    st = board([".....", "..W..", ".WBW.", ".....", "....."], to_move="W")
    st = play(st, 3, 2)
    assert stones(st) == [".....", "..W..", ".W.W.", "..W..", "....."]
    assert gg.turn(st) == 0
    # the captured point is a one-stone ko for black? the capturing stone at
    # (3,2) has black-free neighbours, so no ko; black may not play at (2,2)
    # only if suicide: it is surrounded by white groups each with >1 liberty
    assert st[gg.INVD_CHNL, 2, 2] == 1


def test_multi_group_capture():
    st = board(["BW.WB", ".B.B.", ".....", ".....", "....."], to_move="B")
    nxt = play(st, 0, 2)                          # kills (0,1) and (0,3): two groups
    assert stones(nxt)[:2] == ["B.B.B", ".B.B."]
    assert nxt[gg.INVD_CHNL, 0, 1] == 1           # suicide for white (boxed in by black)
    # an empty point enclosed by black whose groups have spare liberties is
    # a legal "own eye" for black and suicide for white
    st = board(["B.B..", ".B...", ".....", ".....", "....."], to_move="W")
    assert st[gg.INVD_CHNL, 0, 1] == 1
    st = board(["B.B..", ".B...", ".....", ".....", "....."], to_move="B")
    assert st[gg.INVD_CHNL, 0, 1] == 0


def test_suicide_is_invalid_but_capture_is_valid():
    st = board([".W...", "W....", ".....", ".....", "....."], to_move="B")
    assert st[gg.INVD_CHNL, 0, 0] == 1            # suicide in the corner
    st = board([".WB..", "WB...", "B....", ".....", "....."], to_move="B")
    assert st[gg.INVD_CHNL, 0, 0] == 0            # captures (0,1) and (1,0)
    nxt = play(st, 0, 0)
    assert stones(nxt)[0] == "B.B.." and stones(nxt)[1] == ".B..."
    with pytest.raises(AssertionError):
        play(board([".W...", "W....", ".....", ".....", "....."], to_move="B"), 0, 0)


def test_ko_point_and_recapture_after_one_move():
    st = board([".BW..", "BW.W.", ".BW..", ".....", "....."], to_move="B")
    st = play(st, 1, 2)                           # black captures white (1,1)
    assert stones(st)[1] == "B.BW."
    assert gg.turn(st) == 1
    assert st[gg.INVD_CHNL, 1, 1] == 1            # white may not retake at once
    st = play(st, 4, 4)                           # white plays elsewhere
    st = play(st, 4, 0)                           # black plays elsewhere
    assert st[gg.INVD_CHNL, 1, 1] == 0            # now white may retake
    st = play(st, 1, 1)
    assert stones(st)[1] == "BW.W."


def test_pass_clears_ko_and_double_pass_ends():
    st = board([".BW..", "BW.W.", ".BW..", ".....", "....."], to_move="B")
    st = play(st, 1, 2)
    assert st[gg.INVD_CHNL, 1, 1] == 1
    st = play(st, None)                           # white passes
    assert gg.prev_player_passed(st) and not gg.game_ended(st)
    st = play(st, None)                           # black passes -> done
    assert gg.game_ended(st)
    assert not gg.invalid_moves(st).any()         # invalid_moves() zeroed when done


def test_area_scoring_with_neutral_points():
    st = board(["B.W..", "B.W..", "B.W..", "B.W..", "B.W.."], to_move="B")
    black, white = gg.areas(st)
    assert (black, white) == (5, 15)              # column 1 is neutral (touches both)
    assert gg.winning(st) == -1
    assert gg.winning(st, komi=-11) == 1
    st = board(["B....", ".....", ".....", ".....", "....."])
    assert gg.areas(st) == (25, 0)
    assert gg.winning(gg.init_state(5)) == 0


def test_env_protocol():
    env = GoEnv(5)
    obs = env.reset()
    assert obs.shape == (6, 5, 5) and obs.dtype == np.float64
    obs, reward, done, info = env.step(25)
    assert reward == 0 and not done and info["prev_player_passed"]
    obs, reward, done, info = env.step(25)
    assert done and env.winner() == 0 and reward == 0
    with pytest.raises(AssertionError):
        env.step(0)
