"""GPU parity: whole self-play games on the device (mzgo_selfplay_move) vs the
reference game loop (self_play.py:453-526) and its record format.

* A 5x5 / 25-simulation game recorded from the reference itself
  (tests/golden/game_5x5_s25_hooked.npz, counter-stream hooks, injected
  Dirichlet samples) is replayed by the engine: observations, actions, policy
  targets, rewards, returns and final reward must be identical (types too);
  root values within 1e-5 (fp32 network).
* A batch of 9x9 games is checked move by move against the oracle board and
  the reference's compat-mode policy target.
"""
import json

import numpy as np
import pytest
import torch

from oracle import gogame as gg
from oracle.mcts import root_valid_mask
from oracle.rng import injected_noise

pytestmark = pytest.mark.gpu


def _net(N, C=96):
    import mzgo
    from oracle.weights import deterministic_state_dict
    net = mzgo.MuZeroNet(C, N * N + 1).to("cuda").eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in deterministic_state_dict(C, N * N + 1, 0).items()})
    return net


def test_game_matches_reference_record(golden_dir):
    import mzgo
    g = np.load(f"{golden_dir}/game_5x5_s25_hooked.npz")
    with open(f"{golden_dir}/game_5x5_s25_hooked.json") as f:
        types = json.load(f)
    N, S, seed, game = (int(g[k]) for k in ("N", "S", "seed", "game"))
    A = N * N + 1
    sp = mzgo.SelfPlay(_net(N), 1, S, seed=seed, game_base=game)
    noise = np.stack([[injected_noise(seed, game, m, A) for m in range(sp.max_moves)]])
    sp.engine.inject_noise(noise)
    hist = sp.play()[0]
    rec = hist.to_record()
    assert list(rec) == types["keys"]
    np.testing.assert_array_equal(np.stack(rec["observations"]), g["observations"])
    np.testing.assert_array_equal(np.array(rec["actions"]), g["actions"])
    np.testing.assert_array_equal(np.stack(rec["policies"]), g["policies"])
    np.testing.assert_allclose(np.array(rec["values"]), g["values"], rtol=0, atol=1e-5)
    np.testing.assert_array_equal(np.array(rec["rewards"], dtype=np.float64), g["rewards"])
    np.testing.assert_array_equal(np.array(rec["returns"], dtype=np.float64), g["returns"])
    assert float(rec["final_reward"]) == float(g["final_reward"])
    for key in ("rewards", "returns", "values", "actions"):
        assert [type(x).__name__ for x in rec[key]] == types[key], key
    assert type(rec["final_reward"]).__name__ == types["final_reward"]


@pytest.mark.parametrize("compat", ["reference", "fixed"])
def test_batched_games_replay_on_oracle_board(compat):
    import mzgo
    N, G, S = 9, 24, 12
    A = N * N + 1
    sp = mzgo.SelfPlay(_net(N), G, S, seed=77, compat=compat)
    hists = sp.play()
    c = sp.engine.counters()
    assert c["playing"] == 0 and c["games_finished"] == G
    total_moves = sum(len(h) for h in hists)
    assert c["moves"] == total_moves and c["simulations"] == total_moves * S
    for h in hists:
        st = gg.init_state(N)
        for t, (obs, a, pol) in enumerate(zip(h.observations, h.actions, h.policies)):
            np.testing.assert_array_equal(obs, st)
            mask = root_valid_mask(obs)
            assert mask[a] > 0, "illegal action recorded"
            if compat == "reference":
                np.testing.assert_array_equal(pol, mask / mask.sum())
            else:
                assert abs(pol.sum() - 1.0) < 1e-12 and np.all(pol[mask == 0] == 0)
            st = gg.next_state(st, a)
        ended = bool(gg.game_ended(st))
        assert len(h) == N * N or ended
        assert float(h.final_reward) == (float(gg.winning(st)) if ended else 0.0)


FIXED_CASES = [(5, 4, 25, 1.0), (9, 3, 48, 1.0), (9, 2, 32, 0.5)]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("N,G,S,temp", FIXED_CASES, ids=[f"{n}x{n}_g{g}_s{s}_t{t}" for n, g, s, t in FIXED_CASES])
def test_fixed_compat_games_match_oracle(N, G, S, temp):
    """compat "fixed" (select_action with the TRUE child visits,
    self_play.py:376-400 as main.py:666-669 reads them) on whole games, move
    by move against oracle.selfplay.Agent(compat="fixed"): the same counter
    streams (SearchHooks: the select draws, and the uniform behind
    np.random.choice / random.choice) and the Dirichlet sample the device drew
    at each root (test hook Engine.record_noise: exactly the bench's sampled
    path).  Identical actions -- visits**(1/T) (T = 0.5: an exact square of
    integer counts in any pow), numpy's cumulative-sum inverse CDF, and from
    move 15 on the first-max argmax --, identical policy targets (true visits /
    sum), root values within 1e-5 (fp32 network)."""
    import mzgo
    from oracle.net import OracleNet
    from oracle.rng import SearchHooks
    from oracle.selfplay import Agent
    from oracle.weights import deterministic_state_dict
    A = N * N + 1
    seed, C = 4321, 96
    sp = mzgo.SelfPlay(_net(N, C), G, S, seed=seed, compat="fixed", temperature=temp)
    drawn = torch.zeros(G, sp.max_moves, A, dtype=torch.float64, device="cuda")
    sp.engine.record_noise(drawn)
    try:
        hists = sp.play()                     # epoch 0: game ids 0 .. G-1 key the streams
    finally:
        sp.engine.record_noise(None)
    drawn = drawn.cpu().numpy()
    onet = OracleNet(deterministic_state_dict(C, A, 0))
    nt = torch.get_num_threads()
    torch.set_num_threads(1)                  # batch-1 towers: threads only add overhead
    sampled = argmaxed = 0
    try:
        for g, h in enumerate(hists):
            st = gg.init_state(N)
            for mv, (obs, a, pol, v) in enumerate(zip(h.observations, h.actions, h.policies, h.values)):
                np.testing.assert_array_equal(obs, st)
                nz = drawn[g, mv]
                agent = Agent(onet, N, A, S, compat="fixed", noise=lambda p, act, e, nz=nz: (1 - e) * p + e * nz)
                t = temp if mv < 15 else 0
                oa, opol, oval = agent.select_action(obs, t, SearchHooks(seed, g, mv))
                assert a == oa, (g, mv, a, oa)
                assert pol.tobytes() == np.asarray(opol, np.float64).tobytes(), (g, mv)
                assert abs(v - oval) < 1e-5, (g, mv, v, oval)
                sampled += t > 0
                argmaxed += t == 0
                st = gg.next_state(st, a)
            ended = bool(gg.game_ended(st))
            assert len(h) == N * N or ended
            assert float(h.final_reward) == (float(gg.winning(st)) if ended else 0.0)
    finally:
        torch.set_num_threads(nt)
    assert sampled > 0 and argmaxed > 0


def test_records_pickle_roundtrip(tmp_path):
    import pickle

    import mzgo
    sp = mzgo.SelfPlay(_net(5), 3, 4, seed=3)
    hists = sp.play()
    paths = mzgo.save_batches(hists, str(tmp_path), save_interval=2)
    assert [p.split("/")[-1] for p in paths] == ["self_play_batch_2.pkl", "self_play_batch_3.pkl"]
    with open(paths[-1], "rb") as f:
        batch = pickle.load(f)
    assert len(batch) == 2                      # games 2..3 (the reference's slice)
    assert set(batch[0]) == {"observations", "actions", "policies", "values", "rewards", "returns",
                             "final_reward"}


def test_records_pack_matches_export():
    """mzgo_records_pack (what the multi-GPU gather moves) == per-slot export."""
    import mzgo
    from mzgo import distributed as mdist
    sp = mzgo.SelfPlay(_net(5), 4, 6, seed=21)
    sp.reset()
    for _ in range(9):
        sp.move()
    buf = mdist.pack_engine(sp.engine).cpu().numpy()
    arrays = mdist.unpack(buf, sp.engine.G, sp.engine.M, 5)
    for g in range(4):
        want = sp.engine.record(g)
        got = mdist.slot_records(arrays, g)
        assert got["length"] == want["length"] == 9
        for k in ("stones", "invd", "flags", "action", "value", "policy", "reward"):
            np.testing.assert_array_equal(got[k], want[k], err_msg=k)


def test_main_variant_games_follow_main_move_rule():
    """search_variant="main" (main.py:246-368 search + the :660-673 move rule):
    legal moves on the oracle board, policy = child visits / sum over valid
    actions, action = first argmax of those visits."""
    import mzgo
    N, G, S = 9, 16, 24
    sp = mzgo.SelfPlay(_net(N), G, S, seed=5, search_variant="main", c_puct=2.0, dirichlet_alpha=0.03,
                       dirichlet_epsilon=0.25, pass_epsilon=0.05)
    hists = sp.play()
    for h in hists:
        st = gg.init_state(N)
        for obs, a, pol in zip(h.observations, h.actions, h.policies):
            np.testing.assert_array_equal(obs, st)
            mask = root_valid_mask(obs, 0.05)
            assert mask[a] > 0
            assert abs(pol.sum() - 1.0) < 1e-12 and np.all(pol[mask == 0] == 0)
            assert int(np.argmax(pol)) == a
            st = gg.next_state(st, a)


def test_sharded_engines_equal_single_engine():
    """Multi-GPU readiness on one GPU: the games of
    global ids [0, G) played by two engines holding [0, G/2) and [G/2, G)
    (what two ranks hold under mzgo.distributed.shard) produce the same
    records, byte for byte, as one engine holding all G -- the RNG streams
    are keyed by global game id, so the shard boundary cannot show."""
    import mzgo
    from mzgo import distributed as mdist
    N, G, S = 9, 64, 48
    net = _net(N)

    def packed(g0, n):
        sp = mzgo.SelfPlay(net, n, S, seed=1234, game_base=g0)
        sp.play()
        return mdist.unpack(mdist.pack_engine(sp.engine).cpu().numpy(), n, sp.max_moves, N)

    whole = packed(0, G)
    halves = [packed(mdist.shard(G, 2, r)[0], mdist.shard(G, 2, r)[1]) for r in range(2)]
    for g in range(G):
        r, slot = divmod(g, G // 2)
        want = mdist.slot_records(whole, g)
        got = mdist.slot_records(halves[r], slot)
        assert got["length"] == want["length"] and got["status"] == want["status"]
        assert got["final_reward"] == want["final_reward"]
        for k in ("stones", "invd", "flags", "action", "value", "policy", "reward"):
            assert got[k].tobytes() == want[k].tobytes(), (g, k)


@pytest.mark.parametrize("chunks", [[81], [3] * 27, [7, 30, 1, 50]])
def test_multi_move_launches_equal_single_moves(chunks):
    """mzgo_selfplay_moves: k moves of every game in one launch (a game stops
    at its end inside the launch) give the records of k one-move launches,
    byte for byte -- the RNG streams are keyed by (game, move), not launch."""
    import mzgo
    from mzgo import distributed as mdist
    N, G, S = 9, 32, 40
    net = _net(N)

    def packed(steps):
        sp = mzgo.SelfPlay(net, G, S, seed=99)
        sp.reset()
        c0 = sp.engine.counters()                # engines are cached per config: counters accumulate
        for k in steps:
            sp.move(k)
        c = sp.engine.counters()
        assert c["playing"] == 0
        d = {k: c[k] - c0[k] for k in ("moves", "simulations", "games_finished", "dynamics_convs")}
        return d, mdist.unpack(mdist.pack_engine(sp.engine).cpu().numpy(), G, sp.max_moves, N)

    c1, want = packed([1] * 81)
    c2, got = packed(chunks)
    assert c1 == c2
    for g in range(G):
        a, b = mdist.slot_records(got, g), mdist.slot_records(want, g)
        assert a["length"] == b["length"] and a["final_reward"] == b["final_reward"]
        for k in ("stones", "invd", "flags", "action", "value", "policy", "reward"):
            assert a[k].tobytes() == b[k].tobytes(), (g, k)


@pytest.mark.parametrize("helpers", ["1", "3"])
def test_helper_workgroups_do_not_change_records(helpers, monkeypatch):
    """19x19: the helper workgroups that share each game's batch expansions
    and parent convs (batch_expand_shared / conv_shared) leave every record
    byte for byte as the game's workgroup alone produces it."""
    import mzgo
    from mzgo import distributed as mdist
    N, G, S, M = 19, 16, 96, 12
    net = _net(N)

    def packed(h):
        monkeypatch.setenv("MZGO_HELPERS_PER_GAME", h)
        sp = mzgo.SelfPlay(net, G, S, seed=77)
        sp.reset()
        sp.move(M)
        torch.cuda.synchronize()
        return mdist.unpack(mdist.pack_engine(sp.engine).cpu().numpy(), G, sp.max_moves, N)

    want, got = packed("0"), packed(helpers)
    for g in range(G):
        a, b = mdist.slot_records(got, g), mdist.slot_records(want, g)
        assert a["length"] == b["length"]
        for k in ("stones", "invd", "flags", "action", "value", "policy", "reward"):
            assert a[k].tobytes() == b[k].tobytes(), (g, k)
