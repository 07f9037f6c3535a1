"""Pin the CPU oracle against vectors recorded from the reference itself.

The fixtures in tests/golden/ were produced by ``oracle/make_golden.py``,
which imports the reference ``self_play.py`` (in the build container only).
These tests need neither the reference nor a GPU.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import npsum
from oracle.goenv import GoEnv
from oracle.mcts import MCTS, tree_summary
from oracle.net import OracleNet
from oracle.rng import SearchHooks, injected_noise
from oracle.selfplay import Agent, run_self_play_game
from oracle.weights import deterministic_state_dict


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n", [1, 5, 8, 26, 37, 82, 129, 170, 362, 1000])
def test_pairwise_sum_matches_numpy(dtype, n):
    rng = np.random.default_rng(n)
    for _ in range(50):
        a = (rng.random(n) * rng.choice([1e-4, 1.0, 1e4], n)).astype(dtype)
        assert npsum.pairwise_sum(a, dtype) == np.sum(a)


@pytest.mark.parametrize("N", [5, 9, 19])
def test_net_matches_reference(golden_dir, N):
    g = _load(golden_dir, f"net_N{N}.npz")
    C, A = int(g["C"]), N * N + 1
    net = OracleNet(deterministic_state_dict(C, A, int(g["seed"])))
    with torch.no_grad():
        lat, v0, lg0 = net.initial_inference(torch.FloatTensor(g["obs"]))
        nl, r1, v1, lg1 = net.recurrent_inference(lat, torch.from_numpy(g["action"]))
    for got, key in ((lat, "latent"), (v0, "value0"), (lg0, "logits0"), (nl, "next_latent"),
                     (r1, "reward1"), (v1, "value1"), (lg1, "logits1")):
        np.testing.assert_allclose(got.numpy(), g[key], rtol=0, atol=2e-6, err_msg=key)
        # and the fp32 computation stays within fp32 noise of the fp64 truth
        np.testing.assert_allclose(g[key], g[key + "_f64"] if key != "latent" else g["latent_f64"],
                                   rtol=0, atol=5e-5, err_msg=key)


MCTS_CASES = ["5x5_s25_empty", "5x5_s25_mid", "9x9_s200_empty", "9x9_s200_mid",
              "9x9_s400_mid", "19x19_s800_mid"]


def oracle_tree(g, net=None):
    N, S, C = int(g["N"]), int(g["S"]), int(g["C"])
    A = N * N + 1
    net = net or OracleNet(deterministic_state_dict(C, A, 0))
    seed, game, move = int(g["seed"]), int(g["game"]), int(g["move"])
    hooks = SearchHooks(seed, game, move)
    noise_vec = injected_noise(seed, game, move, A)
    mcts = MCTS(net, A, S,
                choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
                noise=lambda p, alpha, eps: (1 - eps) * p + eps * noise_vec)
    with torch.no_grad():
        root, vc, rv = mcts.run(g["obs"])
    return root, vc, rv, A


@pytest.mark.parametrize("case", MCTS_CASES)
def test_mcts_matches_reference_tree(golden_dir, case):
    g = _load(golden_dir, f"mcts_{case}.npz")
    root, vc, rv, A = oracle_tree(g)
    visits, depth = tree_summary(root, A)
    assert root.visit_count == int(g["root_n"])
    np.testing.assert_array_equal(visits, g["visits"])
    np.testing.assert_array_equal(np.array(depth), g["depth_hist"])
    np.testing.assert_array_equal(vc, g["returned_visit_counts"])   # the all-zero bug
    assert not vc.any()
    priors = np.array([root.children[a]["prior"] for a in range(A)], dtype=np.float64)
    np.testing.assert_array_equal(priors, g["root_priors"])
    assert rv == float(g["root_value"])


def _check_record(hist, g, types):
    rec = hist.to_record()
    assert list(rec.keys()) == types["keys"]
    np.testing.assert_array_equal(np.stack(rec["observations"]), g["observations"])
    np.testing.assert_array_equal(np.array(rec["actions"]), g["actions"])
    np.testing.assert_array_equal(np.stack(rec["policies"]), g["policies"])
    np.testing.assert_array_equal(np.array(rec["values"], dtype=np.float64), g["values"])
    np.testing.assert_array_equal(np.array(rec["rewards"], dtype=np.float64), g["rewards"])
    np.testing.assert_array_equal(np.array(rec["returns"], dtype=np.float64), g["returns"])
    assert float(rec["final_reward"]) == float(g["final_reward"])
    assert [type(r).__name__ for r in rec["rewards"]] == types["rewards"]
    assert [type(r).__name__ for r in rec["returns"]] == types["returns"]
    assert [type(v).__name__ for v in rec["values"]] == types["values"]
    assert [type(a).__name__ for a in rec["actions"]] == types["actions"]
    assert type(rec["final_reward"]).__name__ == types["final_reward"]


@pytest.mark.parametrize("mode", ["hooked", "seeded"])
def test_selfplay_game_matches_reference(golden_dir, mode):
    import random
    g = _load(golden_dir, f"game_5x5_s25_{mode}.npz")
    with open(os.path.join(golden_dir, f"game_5x5_s25_{mode}.json")) as f:
        types = json.load(f)
    N, S, C, seed, game = (int(g[k]) for k in ("N", "S", "C", "seed", "game"))
    A = N * N + 1
    net = OracleNet(deterministic_state_dict(C, A, 0))
    if mode == "hooked":
        factory = lambda move: SearchHooks(seed, game, move)  # noqa: E731
        noise = None
        moves = {"m": 0}

        def noise(p, alpha, eps):
            d = injected_noise(seed, game, moves["m"], len(p))
            moves["m"] += 1
            return (1 - eps) * p + eps * d
        agent = Agent(net, N, A, S, noise=noise)
    else:
        factory = None
        random.seed(seed)
        np.random.seed(seed)
        agent = Agent(net, N, A, S)
    hist = run_self_play_game(agent, GoEnv(N), N, hooks_factory=factory)
    _check_record(hist, g, types)


@pytest.mark.parametrize("case", ["5x5_s25_mid", "9x9_s200_empty", "9x9_s200_mid"])
def test_main_variant_mcts_matches_reference_tree(golden_dir, case):
    """oracle.mcts_main (main.py:246-368 restated) vs trees recorded from the
    reference main.py MCTS under the same counter-stream hooks."""
    from oracle.mcts_main import MCTSMain
    g = np.load(os.path.join(golden_dir, f"mctsmain_{case}.npz"))
    N, S, C = int(g["N"]), int(g["S"]), int(g["C"])
    seed, game, move = int(g["seed"]), int(g["game"]), int(g["move"])
    A = N * N + 1
    hooks = SearchHooks(seed, game, move)
    noise = injected_noise(seed, game, move, A)
    m = MCTSMain(OracleNet(deterministic_state_dict(C, A, 0)), A, S, c_puct=float(g["c_puct"]),
                 dirichlet_epsilon=float(g["dirichlet_epsilon"]), pass_epsilon=float(g["pass_epsilon"]),
                 discount=float(g["discount"]),
                 choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
                 noise=lambda p, a, e: (1 - e) * p + e * noise)
    with torch.no_grad():
        root = m.run(g["obs"])
    visits, depth = tree_summary(root, A)
    np.testing.assert_array_equal(visits, g["visits"])
    np.testing.assert_array_equal(np.array(depth), g["depth_hist"])
    np.testing.assert_array_equal([float(root.children[a]["prior"]) for a in range(A)], g["root_priors"])
    assert root.visit_count == int(g["root_n"])
    assert abs(root.value() - float(g["root_value"])) < 1e-12
