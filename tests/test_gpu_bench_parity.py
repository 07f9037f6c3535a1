"""GPU parity at the bench's own kernel configurations.

bench.py times ``k_selfplay_move`` on whole games at 9x9 / 256 games / 200
simulations (config 2); DESIGN.md also quotes 9x9 / 400 (config 3's per-GPU
share) and 19x19 / 64 games / 800 (config 4's).  Self-play is the one path
that leaves lazy rows in the tree (child logits / child ids are formed when a
select first reaches a node; ``k_search`` settles them, a self-play move does
not), so its trees are checked here at those sizes, not only through
``mzgo_search``:

* every game of the batch is replayed on the oracle board
  (oracle/gogame.py): observations bit-exact, every action legal, the
  reference's compat-mode policy target (valid mask / sum, self_play.py:378),
  game length and final reward;
* the engine counters agree with the records;
* for a fixed sample of (game, move) roots the device tree left by that move
  is compared with the oracle's MCTS.run restatement (pinned to the
  reference's own trees, tests/test_oracle_golden.py) under the same counter
  streams and injected Dirichlet sample: identical root-child visit counts,
  root visit count S, root value within 1e-5 (fp32 network).

The sampled-noise run (exactly the bench's code path) records the Dirichlet
sample each root drew (test hook ``Engine.record_noise``) and its sampled
roots are re-searched by the oracle with that sample; the injected-noise run
(same kernel, same sizes; only the Dirichlet source differs) gets the same
tree comparison.
"""
import numpy as np
import pytest
import torch

from oracle import gogame as gg
from oracle.mcts import root_valid_mask

pytestmark = pytest.mark.gpu

SEED = 1234          # bench.py's seed


def _net(N, C=96):
    import mzgo
    from oracle.weights import deterministic_state_dict
    net = mzgo.MuZeroNet(C, N * N + 1).to("cuda").eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in deterministic_state_dict(C, N * N + 1, 0).items()})
    return net


def _noise_table(G, M, A):
    """oracle.rng.injected_noise(SEED, g, mv, A) for every (g, mv), vectorised
    over the actions (the same u01 draws; each row normalised by its own
    numpy sum, as injected_noise does)."""
    from oracle.rng import TAG_DIRICHLET, draw_np, injected_noise, stream_key
    idx = np.arange(A, dtype=np.uint64) << np.uint64(16)
    out = np.empty((G, M, A))
    for g in range(G):
        for mv in range(M):
            h = draw_np(stream_key(SEED, g, mv), TAG_DIRICHLET, idx)
            u = (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53) + 2.0 ** -20
            out[g, mv] = u / u.sum()
    np.testing.assert_array_equal(out[G - 1, M - 1], injected_noise(SEED, G - 1, M - 1, A))
    return out


def _play(net, G, S, check, noise=None, record=None):
    """One epoch of G games from the empty board; returns the histories and
    the trees (root-child visits, root visits, node count) left by the moves
    in ``check`` = {move: [games]}.  record: a float64 [G, M, A] GPU buffer
    that receives every root's normalised Dirichlet sample (test hook)."""
    import mzgo
    sp = mzgo.SelfPlay(net, G, S, seed=SEED)
    eng = sp.engine
    if noise is not None:
        eng.inject_noise(noise)
    if record is not None:
        eng.record_noise(record)
    A = eng.A
    c0 = eng.counters()                    # net.engine() may hand back a used engine
    sp.reset(epoch=0)
    trees = {}
    for mv in range(sp.max_moves):
        sp.move()
        for g in check.get(mv, ()):
            rec_len = eng.record(g)["length"]
            if rec_len != mv + 1:          # the game ended before this move
                continue
            t = eng.tree(g)
            rc = t["child"][0]
            vis = np.array([t["visits"][c] if c >= 0 else 0 for c in rc[:A]], np.int64)
            trees[(g, mv)] = dict(visits=vis, root_n=int(t["visits"][0]), n=int(t["n"]),
                                  value=float(t["value_sum"][0] / t["visits"][0]))
    c1 = eng.counters()
    c = {k: c1[k] - c0[k] for k in ("simulations", "moves", "games_finished")}
    c["playing"] = c1["playing"]
    hists = sp.histories()
    if noise is not None:
        eng.inject_noise(None)
    if record is not None:
        eng.record_noise(None)
    return hists, trees, c


def _replay_all(hists, N, S, counters):
    assert counters["playing"] == 0 and counters["games_finished"] == len(hists)
    total = sum(len(h) for h in hists)
    assert counters["moves"] == total and counters["simulations"] == total * S
    for h in hists:
        st = gg.init_state(N)
        for obs, a, pol, v in zip(h.observations, h.actions, h.policies, h.values):
            np.testing.assert_array_equal(obs, st)
            mask = root_valid_mask(obs)
            assert mask[a] > 0, "illegal action recorded"
            np.testing.assert_array_equal(pol, mask / mask.sum())
            assert np.isfinite(v)
            st = gg.next_state(st, a)
        ended = bool(gg.game_ended(st))
        assert len(h) == N * N or ended
        assert float(h.final_reward) == (float(gg.winning(st)) if ended else 0.0)


def _records(eng):
    """Every slot's record, truncated to its length, from one packed copy."""
    from mzgo.distributed import slot_records, unpack
    arrays = unpack(pack_engine_host(eng), eng.G, eng.M, eng.N)
    return [slot_records(arrays, g) for g in range(eng.G)], arrays


def pack_engine_host(eng):
    from mzgo.distributed import pack_engine
    return pack_engine(eng).cpu().numpy()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("N,G,S,epoch", [(9, 256, 200, 3), (19, 64, 800, 1)],
                         ids=["9x9_g256_s200", "19x19_g64_s800"])
def test_whole_game_launch_equals_per_move_launches(N, G, S, epoch):
    """bench.py plays an epoch as ONE k_selfplay_move launch (the move loop
    inside the kernel: the build that spills); the oracle tests
    above drive one launch per move.  Both launch structures must leave
    byte-identical records (observations, actions, values, policies, rewards,
    lengths, status, final reward) and identical counters at the bench's own
    sizes -- 9x9 / 256 / 200 and 19x19 / 64 / 800 with its 3 helper
    workgroups per game -- so the oracle chain covers the bench's launch."""
    net = _net(N)
    sp = __import__("mzgo").SelfPlay(net, G, S, seed=SEED)
    eng = sp.engine
    M = sp.max_moves

    def run(per_move):
        c0 = eng.counters()
        sp.reset(epoch=epoch)
        if per_move:
            for _ in range(M):
                sp.move()
        else:
            sp.move(M)                       # exactly bench.py's one_epoch()
        c1 = eng.counters()
        recs, arrays = _records(eng)
        c = {k: c1[k] - c0[k] for k in ("simulations", "moves", "games_finished", "dynamics_convs")}
        c["playing"] = c1["playing"]
        return recs, arrays, c

    whole, wa, cw = run(False)
    per, pa, cp = run(True)
    assert cw == cp, (cw, cp)
    assert cw["playing"] == 0 and cw["games_finished"] == G
    np.testing.assert_array_equal(wa["meta"], pa["meta"])
    np.testing.assert_array_equal(wa["status"], pa["status"])
    np.testing.assert_array_equal(wa["final"].view(np.uint64), pa["final"].view(np.uint64))
    for g in range(G):
        a, b = whole[g], per[g]
        assert a["length"] == b["length"], g
        for k in ("stones", "invd", "flags", "action"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"game {g} {k}")
        for k in ("value", "policy", "reward"):      # f64: bit patterns
            np.testing.assert_array_equal(a[k].view(np.uint64), b[k].view(np.uint64), err_msg=f"game {g} {k}")


CONFIGS = [
    # N, G, S, {move: games} sampled for the oracle tree comparison
    (9, 256, 200, {0: [0, 131], 7: [5, 200], 20: [17, 255], 41: [3, 64], 66: [99], 80: [128]}),
    (9, 256, 400, {2: [1], 30: [77], 70: [250]}),
    (19, 64, 800, {0: [0], 45: [33], 200: [63]}),
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("N,G,S,check", CONFIGS, ids=["9x9_g256_s200", "9x9_g256_s400", "19x19_g64_s800"])
def test_selfplay_bench_config_matches_oracle(N, G, S, check):
    from oracle.mcts import MCTS
    from oracle.net import OracleNet
    from oracle.rng import SearchHooks
    from oracle.weights import deterministic_state_dict
    A, M = N * N + 1, N * N
    net = _net(N)

    onet = OracleNet(deterministic_state_dict(96, A, 0))

    def against_oracle(hists, trees, noise):
        assert trees, "no sampled root was still playing"
        for (g, mv), t in sorted(trees.items()):
            obs = hists[g].observations[mv]
            hooks = SearchHooks(SEED, g, mv)
            nz = noise[g, mv]
            ref = MCTS(onet, A, S, choice=lambda seq, sim, h=hooks: seq[h.choice_index(len(seq), sim)],
                       noise=lambda p, a, e, nz=nz: (1 - e) * p + e * nz)
            with torch.no_grad():
                r_root, _, r_value = ref.run(obs)
            r_vis = np.array([r_root.children[a]["node"].visit_count if r_root.children[a]["node"] else 0
                              for a in range(A)])
            np.testing.assert_array_equal(t["visits"], r_vis, err_msg=f"game {g} move {mv}")
            assert t["root_n"] == r_root.visit_count == S
            assert abs(t["value"] - r_value) < 1e-5, (g, mv, t["value"], r_value)
            assert abs(hists[g].values[mv] - r_value) < 1e-5

    # (1) the bench's exact path: Dirichlet noise sampled on the device; the
    # sample each root drew is recorded (test hook) and the oracle re-searches
    # the sampled roots with it
    drawn = torch.zeros(G, M, A, dtype=torch.float64, device="cuda")
    hists, trees, c = _play(net, G, S, check, record=drawn)
    _replay_all(hists, N, S, c)
    drawn = drawn.cpu().numpy()
    for g, h in enumerate(hists):                  # a Dirichlet sample per move played
        rows = drawn[g, :len(h)]
        assert (rows > 0).all() and np.allclose(rows.sum(1), 1.0, atol=1e-12), g
    for (g, mv), t in trees.items():
        assert t["root_n"] == S and int(t["visits"].sum()) == S, (g, mv)
    against_oracle(hists, trees, drawn)

    # (2) injected noise (the counter-stream uniforms of oracle.rng): the same comparison
    noise = _noise_table(G, M, A)
    hists, trees, c = _play(net, G, S, check, noise=noise)
    _replay_all(hists, N, S, c)
    against_oracle(hists, trees, noise)


@pytest.mark.timeout(600)
def test_refill_streams_equal_one_engine():
    """bench.py --refill R (the epoch-tail configuration) runs R
    engines of G slots with game_base r * G, each on its own HIP stream, so
    their k_selfplay_move launches overlap on the GPU.  Concurrent engines
    must not interfere (no shared device state between engines), and a
    game's identity is its global id game_base + slot: engines (base 0, G)
    and (base G, G) played concurrently must leave byte-identical records to
    slots [0, G) and [G, 2G) of one engine of 2G slots played alone."""
    import mzgo
    N, G, S, epoch = 9, 128, 200, 5
    net = _net(N)
    big = mzgo.SelfPlay(net, 2 * G, S, seed=SEED)
    M = big.max_moves
    big.reset(epoch=epoch)
    big.move(M)
    torch.cuda.synchronize()
    ref, ra = _records(big.engine)
    parts = [mzgo.SelfPlay(net, G, S, seed=SEED, game_base=r * G) for r in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    for sp, st in zip(parts, streams):
        with torch.cuda.stream(st):
            sp.reset(epoch=epoch)
            sp.move(M)
    torch.cuda.synchronize()
    for r, sp in enumerate(parts):
        recs, pa = _records(sp.engine)
        np.testing.assert_array_equal(pa["status"], ra["status"][r * G:(r + 1) * G])
        np.testing.assert_array_equal(pa["final"].view(np.uint64), ra["final"][r * G:(r + 1) * G].view(np.uint64))
        for g in range(G):
            a, b = recs[g], ref[r * G + g]
            assert a["length"] == b["length"], (r, g)
            for k in ("stones", "invd", "flags", "action"):
                np.testing.assert_array_equal(a[k], b[k], err_msg=f"engine {r} game {g} {k}")
            for k in ("value", "policy", "reward"):
                np.testing.assert_array_equal(a[k].view(np.uint64), b[k].view(np.uint64),
                                              err_msg=f"engine {r} game {g} {k}")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("epoch", [5, 6])
def test_tail_helpers_do_not_change_records(epoch, monkeypatch):
    """The 9x9 epoch tail (tail_help / conv_tail): in a whole-game launch, the
    workgroups of ended games serve running games' parent convs.  At the
    bench's own size (9x9 / 256 / 200, whole epoch in one launch) the records
    and counters are byte for byte those of the same launch without it
    (MZGO_TAIL_HELPERS=0), and the tail jobs did run."""
    N, G, S = 9, 256, 200
    net = _net(N)
    sp = __import__("mzgo").SelfPlay(net, G, S, seed=SEED)
    eng = sp.engine
    out = {}
    monkeypatch.setenv("MZGO_MOVE_PARALLEL", "0")     # (the game-per-workgroup launch has the tail)
    for on in ("1", "0"):
        monkeypatch.setenv("MZGO_TAIL_HELPERS", on)
        c0 = eng.counters()
        sp.reset(epoch=epoch)
        sp.move(sp.max_moves)
        c1 = eng.counters()
        recs, arrays = _records(eng)
        out[on] = (recs, arrays, {k: c1[k] - c0[k] for k in c1 if k != "playing"})
    (ra, aa, ca), (rb, ab, cb) = out["1"], out["0"]
    assert ca["tail_convs"] > 0 and cb["tail_convs"] == 0, (ca, cb)
    assert {k: v for k, v in ca.items() if k not in ("tail_convs", "tail_wait_expiries")} == {k: v for k, v in cb.items() if k not in ("tail_convs", "tail_wait_expiries")}
    for k in aa:
        np.testing.assert_array_equal(aa[k].view(np.uint8), ab[k].view(np.uint8), err_msg=k)


@pytest.mark.timeout(300)
def test_tail_helpers_games_above_cu_count(monkeypatch):
    """More games than CUs (9x9: one workgroup per CU): the host leaves the
    epoch tail off by default -- ended workgroups would hold CUs that games
    not yet dispatched wait for (tail_enabled) --; forced on
    (MZGO_TAIL_HELPERS=2) the kernel's own guards (a helper joins only games
    whose workgroup has started, and exits when its bounded wait expires)
    still finish the launch, with records byte-identical to the tail off."""
    import mzgo
    N, S = 9, 8
    G = torch.cuda.get_device_properties(0).multi_processor_count + 44
    net = _net(N)
    sp = mzgo.SelfPlay(net, G, S, seed=SEED)
    eng = sp.engine
    out = {}
    monkeypatch.setenv("MZGO_MOVE_PARALLEL", "0")
    for mode in ("1", "2", "0"):
        monkeypatch.setenv("MZGO_TAIL_HELPERS", mode)
        c0 = eng.counters()
        sp.reset(epoch=2)
        sp.move(sp.max_moves)
        c1 = eng.counters()
        recs, arrays = _records(eng)
        out[mode] = (arrays, {k: c1[k] - c0[k] for k in c1 if k != "playing"})
    assert out["1"][1]["tail_convs"] == 0 and out["0"][1]["tail_convs"] == 0, (out["1"][1], out["0"][1])
    assert out["1"][1]["games_finished"] == G
    for mode in ("1", "2"):
        a, c = out[mode]
        assert {k: v for k, v in c.items() if k not in ("tail_convs", "tail_wait_expiries")} == \
            {k: v for k, v in out["0"][1].items() if k not in ("tail_convs", "tail_wait_expiries")}
        for k in a:
            np.testing.assert_array_equal(a[k].view(np.uint8), out["0"][0][k].view(np.uint8), err_msg=f"{mode} {k}")


MP_CASES = [
    # N, G, S, moves per launch (0: the whole game), epoch, MZGO_QUEUE_HELPERS
    (9, 256, 200, 0, 4, "0"),       # the headline's own launch
    (9, None, 8, 16, 2, "0"),       # more games than CUs (the queue's grid is the CU count), chunked launches
    (5, 64, 50, 0, 1, "0"),
    (5, 64, 50, 7, 3, "inject"),    # injected Dirichlet samples (the oracle tests' hook), chunked launches
    (19, 16, 96, 0, 1, "0"),        # 19x19: a tree slot per CU (k_search_queue) vs 3 helper workgroups per game
    (19, 16, 96, 0, 2, "1"),        # 19x19: every searching workgroup with a helper (jobs per tree slot)
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("N,G,S,per,epoch,qh", MP_CASES, ids=["9x9_g256_s200", "9x9_gcu44_s8_chunk16", "5x5_g64_s50",
                                                            "5x5_g64_s50_injected", "19x19_g16_s96",
                                                            "19x19_g16_s96_qh1"])
def test_move_parallel_epoch_equals_game_per_workgroup(N, G, S, per, epoch, qh, monkeypatch):
    """The move-parallel epoch (compat "reference"; k_selfplay_boards,
    then k_search_queue: every recorded move's search claimed from one queue by
    a grid of one workgroup per CU, each in its own tree slot) against the
    game-per-workgroup launch (MZGO_MOVE_PARALLEL=0): byte-identical records
    (observations, actions, root values, policies, rewards, lengths, status),
    the same Dirichlet sample at every root (test hook) and the same counters
    -- the same searches under the same keys, only scheduled differently."""
    import mzgo
    if G is None:
        G = torch.cuda.get_device_properties(0).multi_processor_count + 44
    net = _net(N)
    sp = mzgo.SelfPlay(net, G, S, seed=SEED)
    eng = sp.engine
    M = sp.max_moves
    out = {}
    inject = qh == "inject"
    monkeypatch.setenv("MZGO_QUEUE_HELPERS", "0" if inject else qh)
    if inject:
        eng.inject_noise(np.random.default_rng(7).dirichlet(np.full(eng.A, 0.3), size=(G, M)))
    for mode in ("1", "0"):
        monkeypatch.setenv("MZGO_MOVE_PARALLEL", mode)
        monkeypatch.setenv("MZGO_TAIL_HELPERS", "0")
        drawn = torch.zeros(G, M, eng.A, dtype=torch.float64, device="cuda")
        eng.record_noise(drawn)
        c0 = eng.counters()
        sp.reset(epoch=epoch)
        step = per or M
        for j in range(0, M, step):
            sp.move(min(step, M - j))
        c1 = eng.counters()
        eng.record_noise(None)
        recs, arrays = _records(eng)
        out[mode] = (arrays, drawn.cpu().numpy(),
                     {k: c1[k] - c0[k] for k in c1 if k not in ("playing", "tail_wait_expiries")})
    if inject:
        eng.inject_noise(None)
    (aa, da, ca), (ab, db, cb) = out["1"], out["0"]
    if N == 19:
        # prior_rows counts the rows a game's own workgroup forms; with helper
        # workgroups (the game-per-workgroup launch at 19x19) the batch
        # expansions' rows are formed by job and not counted there
        ca.pop("prior_rows"), cb.pop("prior_rows")
    assert ca == cb, (ca, cb)
    assert ca["games_finished"] == G and ca["simulations"] == ca["moves"] * S
    for k in aa:
        np.testing.assert_array_equal(aa[k].view(np.uint8), ab[k].view(np.uint8), err_msg=k)
    np.testing.assert_array_equal(da.view(np.uint64), db.view(np.uint64))
    assert (aa["meta"][:, 3] > 0).all()
