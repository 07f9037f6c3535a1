"""GPU parity: the integer board kernels vs the GymGo restatement, bit-exact.

Board parity is unpinned by the reference (GymGo is absent from it); the
oracle here is oracle/gogame.py, itself checked by known-answer positions.
Random playouts step G boards at once on the device and one oracle state per
board on the host; all six planes must agree exactly after every move.
"""
import numpy as np
import pytest
import torch

from oracle import gogame as gg

pytestmark = pytest.mark.gpu


def _engine(N, G, komi=0.0):
    from mzgo.engine import Engine, EngineConfig
    return Engine(EngineConfig(board_size=N, latent_dim=0, num_games=G, num_simulations=0, komi=komi))


@pytest.mark.parametrize("N,G,steps,pass_p", [(5, 32, 60, 0.08), (9, 24, 110, 0.03),
                                             (19, 8, 160, 0.01), (6, 16, 60, 0.05)])
def test_random_playouts_bit_exact(N, G, steps, pass_p):
    rng = np.random.default_rng(N * 7 + G)
    eng = _engine(N, G)
    eng.board_reset()
    states = [gg.init_state(N) for _ in range(G)]
    for _ in range(steps):
        acts = np.full(G, -1, np.int32)
        for g in range(G):
            if gg.game_ended(states[g]):
                continue
            legal = np.flatnonzero(gg.invalid_moves(states[g]) == 0)
            board = legal[legal < N * N]
            if len(board) == 0 or rng.random() < pass_p:
                acts[g] = N * N
            else:
                acts[g] = rng.choice(board)
        status, winner = eng.board_step(torch.from_numpy(acts))
        planes = eng.board_planes().cpu().numpy()
        for g in range(G):
            if acts[g] < 0:
                continue
            states[g] = gg.next_state(states[g], int(acts[g]))
            assert status[g] == 0
            np.testing.assert_array_equal(planes[g], states[g], err_msg=f"game {g}")
            want = gg.winning(states[g]) if gg.game_ended(states[g]) else 0
            assert winner[g] == want


def test_invalid_move_and_step_after_done_statuses():
    eng = _engine(5, 2)
    eng.board_reset()
    st = gg.init_state(5)
    st[gg.WHITE, 0, 1] = st[gg.WHITE, 1, 0] = 1
    st[gg.INVD_CHNL] = gg.compute_invalid_moves(st, 1)
    eng.board_set(0, st)
    status, _ = eng.board_step(torch.tensor([0, 25], dtype=torch.int32))   # suicide / pass
    assert list(status) == [2, 0]
    status, winner = eng.board_step(torch.tensor([-1, 25], dtype=torch.int32))
    assert status[1] == 0 and winner[1] == 0.0                 # empty board: draw
    status, _ = eng.board_step(torch.tensor([-1, 3], dtype=torch.int32))
    assert status[1] == 1                                      # after the end


def test_goenv_dropin_protocol():
    import mzgo
    env = mzgo.GoEnv(5)
    ref = gg.init_state(5)
    obs = env.reset()
    np.testing.assert_array_equal(obs, ref)
    for a in (12, 7, 13, 17, 25, 11):
        obs, reward, done, info = env.step(a)
        ref = gg.next_state(ref, a)
        np.testing.assert_array_equal(obs, ref)
        assert reward == 0 and not done
    with pytest.raises(AssertionError):
        env.step(12)                                           # occupied
    env.step(25)
    obs, reward, done, info = env.step(25)
    assert done and reward == env.winner() == gg.winning(gg.next_state(gg.next_state(ref, 25), 25))


@pytest.mark.parametrize("komi", [0.0, 2.5])
def test_scoring_kat(komi):
    eng = _engine(5, 1, komi=komi)
    eng.board_reset()
    st = gg.init_state(5)
    for r in range(5):
        st[gg.BLACK, r, 0] = 1
        st[gg.WHITE, r, 2] = 1
    st[gg.PASS_CHNL] = 1                                       # next pass ends the game
    st[gg.INVD_CHNL] = gg.compute_invalid_moves(st, 1)
    eng.board_set(0, st)
    status, winner = eng.board_step(torch.tensor([25], dtype=torch.int32))
    assert status[0] == 0
    assert winner[0] == gg.winning(gg.next_state(st, 25), komi)
