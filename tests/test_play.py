"""Interactive play (mzgo.play; SURVEY.md §8(f) item 4, the reference's play.py).

CPU: coordinates, board text, the network's int(1.5 N^2)-row embedding
(play.py:193) and its state_dict shapes.  GPU: the agent's search is the
oracle's main.py MCTS with play.py's constants (c_puct 10, Dirichlet(0.01)
at 0.02, pass prior 0.01) on the same hooks -- parity pinned through
oracle.mcts_main, itself pinned by the trees recorded from the reference
main.py (play.py's MCTS is the same algorithm) -- its move is the argmax of
the masked visit counts, and a scripted game runs through ``play``.
"""
import numpy as np
import pytest
import torch


def test_coordinates_round_trip():
    from mzgo.play import action_to_coord, coord_to_action
    N = 6
    for a in range(N * N + 1):
        assert coord_to_action(action_to_coord(a, N), N) == a
    assert action_to_coord(N * N, N) == "pass" and coord_to_action("PASS", N) == N * N
    assert coord_to_action(" b3 ", N) == 2 * N + 1 and action_to_coord(2 * N + 1, N) == "B3"
    with pytest.raises(ValueError):
        coord_to_action("Bx", N)


def test_board_text_is_print_board():
    from mzgo.play import board_text
    obs = np.zeros((6, 3, 3))
    obs[0, 0, 1] = 1
    obs[1, 2, 2] = 1
    assert board_text(obs, 3) == "   A B C\n 1 . B .\n 2 . . .\n 3 . . W"


def test_play_network_keeps_the_large_embedding():
    import mzgo
    net = mzgo.MuZeroNet(64, int(6 * 6 * 1.5), board_size=6)
    sd = net.state_dict()
    assert tuple(sd["dynamics.action_embedding.weight"].shape) == (54, 64)
    assert tuple(sd["representation.conv3.weight"].shape) == (64, 64, 3, 3)
    assert net.board_size == 6
    with pytest.raises(ValueError):
        mzgo.MuZeroNet(64, 30, board_size=6)


def _agent(seed_w=7, sims=48):
    from mzgo.play import PlayAgent
    from oracle.weights import deterministic_state_dict
    N, C = 6, 64
    agent = PlayAgent(N, C, N * N + 1, sims, seed=11, game=3)
    sd = deterministic_state_dict(C, 54, seed_w)
    agent.net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return agent, sd


@pytest.mark.gpu
@pytest.mark.parametrize("moves", [0, 7])
def test_play_agent_search_matches_oracle(moves):
    from oracle.mcts import tree_summary
    from oracle.mcts_main import MCTSMain
    from oracle.net import OracleNet
    from oracle.positions import random_position
    from oracle.rng import SearchHooks, injected_noise
    agent, sd = _agent()
    N, A, S = 6, 37, agent.mcts_simulations
    obs = random_position(N, moves, 500 + moves) if moves else np.zeros((6, N, N))
    seed, game, move = agent.seed, agent.game, agent.move
    noise = injected_noise(seed, game, move, A)
    hooks = SearchHooks(seed, game, move)
    ref = MCTSMain(OracleNet(sd), A, S, c_puct=10.0, dirichlet_alpha=0.01, dirichlet_epsilon=0.02,
                   pass_epsilon=0.01, choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
                   noise=lambda p, a, e: (1 - e) * p + e * noise)
    with torch.no_grad():
        r_root = ref.run(obs)
    m = agent.search(obs, noise=torch.from_numpy(noise))
    r_visits = tree_summary(r_root, A)[0]
    np.testing.assert_array_equal(np.asarray(m.root_child_visits), r_visits)
    mask = (np.append(obs[3].flatten() == 0, True))
    want = int(np.argmax(np.where(mask, r_visits, 0)))
    assert agent.select_action(obs, noise=torch.from_numpy(noise)) == want


@pytest.mark.gpu
def test_scripted_game_runs_to_the_end():
    import mzgo
    from mzgo.play import play
    agent, _ = _agent(sims=16)
    env = mzgo.GoEnv(6)
    replies = iter(["bad", "pass"] * 200)
    out = []
    outcome, reward = play(agent, env, human_is_black=True, read=lambda prompt: next(replies),
                           write=out.append)
    assert outcome in ("win", "loss", "draw")
    assert "Invalid move format. Try again." in out
    assert out[-1].startswith("Final outcome: ")
    assert any(line.startswith("Agent move: ") for line in out)
