"""Arena evaluator (main.py:526-611): host scoring on the CPU, the two-network
move kernel on the GPU."""
import numpy as np
import pytest
import torch

from mzgo.arena import SelfPlayEvaluator


def test_win_rate_keeps_reference_double_flip():
    # games 0, 2: current (black) wins / loses; games 1, 3: best starts (black)
    winners = [1, -1, -1, 1]
    # play_game: g0 1, g1 (start 1) white won -> 1, g2 0, g3 0; evaluate flips g1, g3
    assert SelfPlayEvaluator.win_rate(winners) == (1 + 0 + 0 + 1) / 4
    assert SelfPlayEvaluator.win_rate([0, 0]) == (0 + 1) / 2     # truncated games


def _nets(N, C, seeds):
    import mzgo
    out = []
    for s in seeds:
        net = mzgo.MuZeroNet(C, N * N + 1).to("cuda").eval()
        net.load_state_dict(mzgo.deterministic_state_dict(C, N * N + 1, s))
        out.append(net)
    return out


@pytest.mark.gpu
def test_arena_with_equal_networks_is_main_selfplay():
    import mzgo
    N, C, G, S = 6, 128, 6, 16
    a, a2 = _nets(N, C, [3, 3])
    ev = SelfPlayEvaluator(a, a2, num_games=G, num_simulations=S, seed=8)
    winners = ev.play()
    sp = mzgo.SelfPlay(a, G, S, seed=8, search_variant="main", compat="fixed", c_puct=2.0,
                       dirichlet_alpha=0.03, dirichlet_epsilon=0.25, pass_epsilon=0.05,
                       max_moves=int(N * N * 1.5))
    hists = sp.play()
    assert [float(h.final_reward) for h in hists] == list(winners)
    eng = a.engine(G, S, **ev.cfg)
    for g, h in enumerate(hists):
        rec = eng.record(g)
        assert list(rec["action"]) == list(h.actions)


@pytest.mark.gpu
def test_arena_first_mover_alternates_by_game():
    """Game i's first move is searched by the current network iff i is even."""
    import mzgo
    N, C, G, S = 6, 128, 4, 16
    a, b = _nets(N, C, [3, 4])
    ev = SelfPlayEvaluator(a, b, num_games=G, num_simulations=S, seed=8)
    eng = a.engine(G, S, **ev.cfg)
    opp = b.engine(G, S, **ev.cfg)
    eng.selfplay_reset(0)
    eng.arena_move(opp)
    first = [eng.record(g)["policy"][0].copy() for g in range(G)]
    for net, parity in ((a, 0), (b, 1)):
        e1 = net.engine(G, S, **ev.cfg)
        e1.selfplay_reset(0)
        e1.selfplay_move()
        for g in range(G):
            if g % 2 == parity:
                np.testing.assert_array_equal(first[g], e1.record(g)["policy"][0])


@pytest.mark.gpu
def test_arena_matches_reference_evaluator(golden_dir):
    """Games recorded from the reference SelfPlayEvaluator (main.py:526-611,
    tests/golden/arena_5x5_s16.npz; oracle/make_golden.py make_arena) under
    the counter-stream hooks: the device arena plays the same moves in every
    game, reaches the same winners and the same win rate / Elo update."""
    from oracle.rng import injected_noise
    g = np.load(f"{golden_dir}/arena_5x5_s16.npz")
    N, S, G, C, seed = (int(g[k]) for k in ("N", "S", "G", "C", "seed"))
    A = N * N + 1
    cur, best = _nets(N, C, [int(x) for x in g["seeds"]])
    ev = SelfPlayEvaluator(cur, best, num_games=G, num_simulations=S, seed=seed)
    assert ev.max_moves == int(g["max_moves"])
    noise = np.stack([[injected_noise(seed, i, m, A) for m in range(ev.max_moves)] for i in range(G)])
    winners = ev.play(noise=noise)
    torch.cuda.synchronize()
    eng = cur.engine(G, S, **ev.cfg)
    for i in range(G):
        L = int(g["lengths"][i])
        rec = eng.record(i)
        assert rec["length"] == L, (i, rec["length"], L)
        np.testing.assert_array_equal(rec["action"], g["actions"][i, :L], err_msg=f"game {i}")
    np.testing.assert_array_equal(winners, g["winners"])
    wr = SelfPlayEvaluator.win_rate(winners)
    assert wr == float(g["win_rate"])
    expected = 1 / (1 + 10 ** ((ev.best_elo - ev.current_elo) / 400))
    elo = ev.current_elo + (ev.elo_k * (wr - expected) if wr > ev.win_threshold else 0.0)
    assert elo == float(g["elo"])
