"""GPU parity: the device MCTS (mzgo_search) vs trees recorded from the
reference MCTS.run (self_play.py:148-237).

The reference's draws are replaced on both sides by the same counter streams
(random.choice at :287 -> TAG_SELECT draw per simulation; the Dirichlet sample
at :38 -> oracle.rng.injected_noise), so the trees can be compared node for
node.  The only non-exact input is the network (fp32 with a different
summation order than torch, |diff| ~1e-6), so we require: root value within
1e-5, identical root priors to 1e-12 relative (float64 chain on identical
logits up to that noise), and root-child visit counts identical -- SURVEY.md
§4 measured that 1e-7 output perturbations leave the visit counts unchanged
at every size.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = ["5x5_s25_empty", "5x5_s25_mid", "9x9_s200_empty", "9x9_s200_mid", "9x9_s400_mid",
         "19x19_s800_mid"]


def _net(N, C=96):
    import mzgo
    from oracle.weights import deterministic_state_dict
    net = mzgo.MuZeroNet(C, N * N + 1).to("cuda").eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in deterministic_state_dict(C, N * N + 1, 0).items()})
    return net


@pytest.mark.parametrize("dynamics", ["factored", "direct"])
@pytest.mark.parametrize("case", CASES)
def test_search_matches_reference_tree(golden_dir, case, dynamics):
    import mzgo
    from oracle.mcts import tree_summary
    from oracle.rng import injected_noise
    g = np.load(f"{golden_dir}/mcts_{case}.npz")
    N, S = int(g["N"]), int(g["S"])
    seed, game, move = int(g["seed"]), int(g["game"]), int(g["move"])
    A = N * N + 1
    net = _net(N)
    mcts = mzgo.MCTS(net, A, S, seed=seed, game=game, dynamics=dynamics)
    noise = torch.from_numpy(injected_noise(seed, game, move, A))
    root, visit_counts, root_value = mcts.run(g["obs"], move_index=move, noise=noise)
    assert not visit_counts.any()                       # reference bug reproduced (compat)
    assert root.visit_count == S
    np.testing.assert_allclose([root.children[a]["prior"] for a in range(A)], g["root_priors"],
                               rtol=1e-5, atol=1e-9)
    visits, depth = tree_summary(root, A)
    np.testing.assert_array_equal(visits, g["visits"])
    np.testing.assert_array_equal(np.array(depth), g["depth_hist"])
    assert abs(root_value - float(g["root_value"])) < 1e-5
    np.testing.assert_array_equal(mcts.root_child_visits, g["visits"])


def test_batched_search_equals_single_searches():
    """G roots in one launch == G separate single-root searches (no cross-talk)."""
    import mzgo
    from oracle.positions import random_position
    N, S, G = 9, 64, 8
    net = _net(N)
    obs = np.stack([random_position(N, 5 * i, 40 + i) for i in range(G)])
    eng = net.engine(num_games=G, num_simulations=S, seed=5)
    vis_b, val_b = eng.search(torch.from_numpy(obs), move_index=3)
    vis_b, val_b = vis_b.cpu().numpy(), val_b.cpu().numpy()
    for i in range(G):
        e1 = net.engine(num_games=1, num_simulations=S, seed=5, game_base=i)
        v1, val1 = e1.search(torch.from_numpy(obs[i:i + 1]), move_index=3)
        np.testing.assert_array_equal(v1.cpu().numpy()[0], vis_b[i])
        assert val1.item() == val_b[i]


@pytest.mark.parametrize("N,S,moves", [(5, 40, 6), (6, 128, 10), (9, 200, 20), (9, 600, 12), (19, 300, 60)])
def test_factored_expansion_equals_direct_conv(N, S, moves):
    """The factored expansion (conv once per parent, children as relu(Y +
    E[a]); mzgo_expand.hpp) against a dynamics conv per simulation, the
    reference's formulation (self_play.py:85-95), on G mid-game roots: the same
    trees (node for node), child priors and root values up to fp32 rounding.
    9x9 / 600 simulations runs the HBM-tree variants of the batches and their
    replay (600 + 2 nodes exceed the LDS tree)."""
    from oracle.positions import random_position
    G = 8
    net = _net(N)
    obs = torch.from_numpy(np.stack([random_position(N, moves + i, 300 + i) for i in range(G)]))
    out = {}
    for dyn in ("factored", "direct"):
        eng = net.engine(num_games=G, num_simulations=S, seed=11, dynamics=dyn)
        vis, val = eng.search(obs, move_index=moves)
        out[dyn] = (vis.cpu().numpy(), val.cpu().numpy(), [eng.tree(g) for g in range(G)])
    (vf, rf, tf), (vd, rd, td) = out["factored"], out["direct"]
    np.testing.assert_array_equal(vf, vd)
    np.testing.assert_allclose(rf, rd, rtol=0, atol=1e-5)
    for a, b in zip(tf, td):
        np.testing.assert_array_equal(a["child"], b["child"])
        np.testing.assert_array_equal(a["visits"], b["visits"])
        np.testing.assert_allclose(a["prior"][1:], b["prior"][1:], rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(a["value_sum"], b["value_sum"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("N", [5, 9, 19])
def test_sampled_dirichlet_statistics(N):
    """The device Gamma sampler gives Dirichlet(alpha) roots: with epsilon=1
    the root prior IS the masked, renormalised noise; check its moments.  At
    9x9 (A=82) and 19x19 (A=362) the draws are split over waves 1..AP
    (entries a >= 64 come from the other waves), so those entries are
    checked on their own too (non-stale, same distribution)."""
    S, G = 1, 256
    A = N * N + 1
    net = _net(N)
    eng = net.engine(num_games=G, num_simulations=S, seed=9, dirichlet_epsilon=1.0,
                     pass_epsilon=1.0)
    obs = torch.zeros(G, 6, N, N)
    eng.search(obs, move_index=0)
    pri = np.stack([eng.tree(g)["root_prior"] for g in range(G)])
    assert np.allclose(pri.sum(1), 1.0)
    assert np.all(pri > 0)
    alpha = 0.15
    want_var = (1 / A) * (1 - 1 / A) / (A * alpha + 1)
    assert abs(pri.mean() - 1 / A) < 1e-9
    parts = [pri] if A <= 64 else [pri, pri[:, 64:]]
    for part in parts:
        assert 0.7 * want_var < part.var() < 1.3 * want_var, (part.shape, part.var(), want_var)
    if A > 64:
        hi = pri[:, 64:]
        assert abs(hi.mean() - 1 / A) < 0.1 / A
        # no two games share a draw (a stale / unwritten entry would repeat)
        assert len(np.unique(hi)) == hi.size


@pytest.mark.parametrize("N,S,moves", [(6, 64, 0), (6, 64, 9), (9, 100, 14), (9, 100, 30)])
def test_search_matches_oracle_tree(N, S, moves):
    """Sizes / positions without a reference golden (6x6 is self_play.py's
    default board, :20): the device tree vs the oracle's restatement of
    MCTS.run (itself pinned to the reference goldens above), same hooks."""
    import mzgo
    from oracle.mcts import MCTS, tree_summary
    from oracle.net import OracleNet
    from oracle.positions import random_position
    from oracle.rng import SearchHooks, injected_noise
    from oracle.weights import deterministic_state_dict
    C, A, seed, game, move = 96, N * N + 1, 31, 2, moves
    obs = random_position(N, moves, 100 + moves) if moves else np.zeros((6, N, N))
    noise = injected_noise(seed, game, move, A)
    hooks = SearchHooks(seed, game, move)
    onet = OracleNet(deterministic_state_dict(C, A, 0))
    ref = MCTS(onet, A, S, choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
               noise=lambda p, a, e: (1 - e) * p + e * noise)
    with torch.no_grad():
        r_root, _, r_value = ref.run(obs)
    r_visits, r_depth = tree_summary(r_root, A)
    mcts = mzgo.MCTS(_net(N), A, S, seed=seed, game=game)
    root, _, value = mcts.run(obs, move_index=move, noise=torch.from_numpy(noise))
    visits, depth = tree_summary(root, A)
    np.testing.assert_array_equal(visits, r_visits)
    np.testing.assert_array_equal(np.array(depth), np.array(r_depth))
    assert abs(value - r_value) < 1e-5


@pytest.mark.parametrize("case", ["5x5_s25_mid", "9x9_s200_empty", "9x9_s200_mid"])
def test_main_variant_search_matches_reference_tree(golden_dir, case):
    """search_variant="main": main.py's MCTS (main.py:246-368) on the device vs
    trees recorded from the reference main.py under the same hooks."""
    import mzgo
    from oracle.mcts import tree_summary
    from oracle.rng import injected_noise
    g = np.load(f"{golden_dir}/mctsmain_{case}.npz")
    N, S = int(g["N"]), int(g["S"])
    seed, game, move = int(g["seed"]), int(g["game"]), int(g["move"])
    A = N * N + 1
    m = mzgo.MainMCTS(_net(N), A, S, c_puct=float(g["c_puct"]), seed=seed, game=game,
                      dirichlet_epsilon=float(g["dirichlet_epsilon"]), pass_epsilon=float(g["pass_epsilon"]),
                      discount=float(g["discount"]))
    root = m.run(g["obs"], move_index=move, noise=torch.from_numpy(injected_noise(seed, game, move, A)))
    assert root.visit_count == int(g["root_n"])
    np.testing.assert_allclose([root.children[a]["prior"] for a in range(A)], g["root_priors"],
                               rtol=1e-5, atol=1e-9)
    visits, depth = tree_summary(root, A)
    np.testing.assert_array_equal(visits, g["visits"])
    np.testing.assert_array_equal(np.array(depth), g["depth_hist"])
    assert abs(m.root_value - float(g["root_value"])) < 1e-5


@pytest.mark.parametrize("moves", [0, 8])
def test_main_variant_6x6_c128_matches_oracle(moves):
    """main.py's own configuration (6x6, latent_dim 128, main.py:27-53): the
    device main-variant tree vs oracle.mcts_main (pinned by the main.py
    goldens above) on the same hooks."""
    import mzgo
    from oracle.mcts import tree_summary
    from oracle.mcts_main import MCTSMain
    from oracle.net import OracleNet
    from oracle.positions import random_position
    from oracle.rng import SearchHooks, injected_noise
    from oracle.weights import deterministic_state_dict
    N, C, S, seed, game, move = 6, 128, 96, 17, 1, moves
    A = N * N + 1
    obs = random_position(N, moves, 300 + moves) if moves else np.zeros((6, N, N))
    noise = injected_noise(seed, game, move, A)
    hooks = SearchHooks(seed, game, move)
    sd = deterministic_state_dict(C, A, 0)
    ref = MCTSMain(OracleNet(sd), A, S, choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
                   noise=lambda p, a, e: (1 - e) * p + e * noise)
    with torch.no_grad():
        r_root = ref.run(obs)
    net = mzgo.MuZeroNet(C, A).to("cuda").eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = mzgo.MainMCTS(net, A, S, seed=seed, game=game)
    root = m.run(obs, move_index=move, noise=torch.from_numpy(noise))
    np.testing.assert_array_equal(tree_summary(root, A)[0], tree_summary(r_root, A)[0])
    np.testing.assert_array_equal(np.array(tree_summary(root, A)[1]), np.array(tree_summary(r_root, A)[1]))
    assert abs(m.root_value - r_root.value()) < 1e-5
