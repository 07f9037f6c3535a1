"""Generate tests/golden/ by importing the reference (TEST INFRASTRUCTURE ONLY).

Runs ONLY in the build container, where the reference snapshot is mounted at
/root/reference.  Nothing here travels to the GPU box: the outputs are small
data fixtures (inputs and expected outputs) committed under tests/golden/.

The reference ``self_play.py`` imports ``gym``, ``gym_go`` and ``wandb``,
none of which is installed; minimal stand-ins are written to a temporary
directory at run time: ``gym.make`` raises, ``govars``
holds the six plane indices, ``gogame``/``rendering`` are empty and ``wandb``
is a no-op.  Nothing from the reference is copied; its classes are called.

Fixtures:
  net_N{5,9,19}.npz    reference MuZeroNet (self_play.py:115-128) outputs for
                       deterministic weights (oracle/weights.py, seed 0, C=96)
  mcts_*.npz           reference MCTS.run (self_play.py:148-237) with
                       random.choice and the Dirichlet draw replaced by the
                       counter streams of oracle/rng.py: true root-child
                       visits, root value, root priors, nodes per depth
  game_5x5_*.npz/json  a reference run_self_play_game (self_play.py:453) over
                       oracle.goenv.GoEnv, (a) with counter-stream hooks and
                       (b) with the reference's own seeded RNGs
  mctsmain_*.npz       main.py's MCTS.run (main.py:246-368) under the same hooks
  train_5x5_c32.npz    main.py's MuZeroAgent.train (main.py:381-522), two
                       batches on synthetic trajectories with fixed start
                       indices: losses, priorities, lr, final weights
  arena_5x5_s16.npz    main.py's SelfPlayEvaluator (main.py:526-611) games
                       between two networks under the same hooks
Usage:  python -m oracle.make_golden   (from the repo root)
"""
import json
import os
import random
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
REFERENCE = "/root/reference"

_STUBS = {
    "gym/__init__.py": "def make(*a, **k):\n    raise RuntimeError('gym is not installed')\n",
    "gym_go/__init__.py": "",
    "gym_go/govars.py": "BLACK=0\nWHITE=1\nTURN_CHNL=2\nINVD_CHNL=3\nPASS_CHNL=4\nDONE_CHNL=5\nNUM_CHNLS=6\n",
    "gym_go/gogame.py": "",
    "gym_go/rendering.py": "",
    "wandb/__init__.py": "run = None\n" + "".join(
        f"def {f}(*a, **k):\n    return None\n" for f in ("init", "log", "save", "finish")),
}


def import_reference():
    stub_dir = tempfile.mkdtemp(prefix="mzgo_stubs_")
    for rel, text in _STUBS.items():
        path = os.path.join(stub_dir, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(text)
    sys.dont_write_bytecode = True
    sys.path[:0] = [stub_dir, REFERENCE]
    import self_play as sp  # noqa: E402  (the reference module)
    return sp


def _ref_net(sp, sd, C, A):
    net = sp.MuZeroNet(C, A)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return net.eval()


def make_net(sp, N, B, C=96, seed=0):
    from oracle.positions import random_position
    from oracle.weights import deterministic_state_dict
    A = N * N + 1
    sd = deterministic_state_dict(C, A, seed)
    net = _ref_net(sp, sd, C, A)
    rng = np.random.default_rng(1000 + N)
    obs = np.stack([random_position(N, int(rng.integers(0, N * N)), 7 * N + b) for b in range(B)])
    act = rng.integers(0, A, size=B).astype(np.int64)
    with torch.no_grad():
        lat, v0, lg0 = net.initial_inference(torch.FloatTensor(obs))
        nl, r1, v1, lg1 = net.recurrent_inference(lat, torch.from_numpy(act))
        # fp64 truth of the same computation (tolerance reasoning only)
        net64 = _ref_net(sp, sd, C, A).double()
        lat64, v064, lg064 = net64.initial_inference(torch.from_numpy(obs))
        nl64, r164, v164, lg164 = net64.recurrent_inference(lat.double(), torch.from_numpy(act))
    out = dict(obs=obs.astype(np.float64), action=act, latent=lat.numpy(), value0=v0.numpy(),
               logits0=lg0.numpy(), next_latent=nl.numpy(), reward1=r1.numpy(), value1=v1.numpy(),
               logits1=lg1.numpy(), latent_f64=lat64.numpy(), value0_f64=v064.numpy(),
               logits0_f64=lg064.numpy(), next_latent_f64=nl64.numpy(), reward1_f64=r164.numpy(),
               value1_f64=v164.numpy(), logits1_f64=lg164.numpy(), seed=np.int64(seed), C=np.int64(C))
    np.savez_compressed(os.path.join(GOLDEN, f"net_N{N}.npz"), **out)
    print("net", N, {k: v.shape for k, v in out.items()})


class _Hooked:
    """Counter-stream hooks installed into the reference module."""

    def __init__(self, sp, seed, game):
        from oracle.rng import SearchHooks
        self.sp, self.seed, self.game = sp, seed, game
        self.move, self.sim, self.in_search = 0, -1, False
        self.hooks = SearchHooks(seed, game, 0)
        self.saved = (sp.random.choice, sp.np.random.choice, sp.apply_dirichlet_noise,
                      sp.MCTS.select_leaf, sp.MCTS.run, sp.MuZeroAgent.select_action)

    def install(self, eps_noise=True):
        from oracle.rng import SearchHooks, injected_noise
        sp, me = self.sp, self
        orig_choice, orig_npchoice, _, orig_select, orig_run, orig_act = self.saved

        def choice(seq):
            if me.in_search:
                return seq[me.hooks.choice_index(len(seq), me.sim)]
            return seq[me.hooks.action_index(len(seq))]

        def np_choice(a, p=None, **kw):
            from oracle.selfplay import inverse_cdf
            return inverse_cdf(np.asarray(p), me.hooks.action_uniform())

        def noise(policy, alpha, epsilon):
            d = injected_noise(me.seed, me.game, me.move, len(policy))
            return (1 - epsilon) * policy + epsilon * d

        def select_leaf(self_, node, valid_mask):
            me.sim += 1
            return orig_select(self_, node, valid_mask)

        def run(self_, observation):
            me.in_search, me.sim = True, -1
            try:
                return orig_run(self_, observation)
            finally:
                me.in_search = False

        def select_action(self_, observation, temperature):
            me.hooks = SearchHooks(me.seed, me.game, me.move)
            try:
                return orig_act(self_, observation, temperature)
            finally:
                me.move += 1

        sp.random.choice = choice
        sp.np.random.choice = np_choice
        sp.apply_dirichlet_noise = noise
        sp.MCTS.select_leaf = select_leaf
        sp.MCTS.run = run
        sp.MuZeroAgent.select_action = select_action
        return self

    def restore(self):
        sp = self.sp
        (sp.random.choice, sp.np.random.choice, sp.apply_dirichlet_noise,
         sp.MCTS.select_leaf, sp.MCTS.run, sp.MuZeroAgent.select_action) = self.saved


def _configure(sp, N, S):
    sp.config.board_size = N
    sp.config.max_action_size = N * N + 1
    sp.config.mcts_simulations = S


def make_mcts(sp, name, N, S, n_moves, seed=11, game=3, move=5, C=96):
    from oracle.mcts import tree_summary
    from oracle.positions import random_position
    from oracle.weights import deterministic_state_dict
    A = N * N + 1
    _configure(sp, N, S)
    sd = deterministic_state_dict(C, A, 0)
    net = _ref_net(sp, sd, C, A)
    obs = random_position(N, n_moves, seed=500 + n_moves)
    h = _Hooked(sp, seed, game)
    h.move = move
    h.install()
    try:
        from oracle.rng import SearchHooks
        h.hooks = SearchHooks(seed, game, move)
        mcts = sp.MCTS(net, A, S)
        with torch.no_grad():
            root, vc, rv = mcts.run(obs)
    finally:
        h.restore()
    visits, depth = tree_summary(root, A)
    priors = np.array([root.children[a]["prior"] for a in range(A)], dtype=np.float64)
    out = dict(obs=obs, visits=visits, root_value=np.float64(rv), root_n=np.int64(root.visit_count),
               returned_visit_counts=np.asarray(vc), root_priors=priors,
               depth_hist=np.array(depth, dtype=np.int64), seed=np.int64(seed), game=np.int64(game),
               move=np.int64(move), S=np.int64(S), N=np.int64(N), C=np.int64(C))
    np.savez_compressed(os.path.join(GOLDEN, f"mcts_{name}.npz"), **out)
    print("mcts", name, "root N", root.visit_count, "value", rv, "depth", depth)


def make_mcts_main(mn, name, N, S, n_moves, seed=13, game=4, move=6, C=96):
    """main.py's MCTS (main.py:246-368; trainer self-play and arena), same
    counter-stream hooks: random.choice -> TAG_SELECT per simulation (the
    simulation index counted by wrapping select_leaf, called once per
    simulation at :290), apply_dirichlet_noise -> injected sample."""
    from oracle.mcts import tree_summary
    from oracle.positions import random_position
    from oracle.rng import SearchHooks, injected_noise
    from oracle.weights import deterministic_state_dict
    A = N * N + 1
    mn.config.board_size = N
    mn.config.max_action_size = A
    sd = deterministic_state_dict(C, A, 0)
    net = mn.MuZeroNet(C, A)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    net.eval()
    obs = random_position(N, n_moves, seed=700 + n_moves)
    hooks = SearchHooks(seed, game, move)
    state = {"sim": -1}
    saved = (mn.random.choice, mn.apply_dirichlet_noise, mn.MCTS.select_leaf)
    orig_select = mn.MCTS.select_leaf

    def select_leaf(self_, node):
        state["sim"] += 1
        return orig_select(self_, node)

    def noise(policy, alpha, epsilon):
        return (1 - epsilon) * policy + epsilon * injected_noise(seed, game, move, len(policy))
    mn.random.choice = lambda seq: seq[hooks.choice_index(len(seq), state["sim"])]
    mn.apply_dirichlet_noise = noise
    mn.MCTS.select_leaf = select_leaf
    try:
        with torch.no_grad():
            root = mn.MCTS(net, A, S).run(obs)
    finally:
        mn.random.choice, mn.apply_dirichlet_noise, mn.MCTS.select_leaf = saved
    visits, depth = tree_summary(root, A)
    priors = np.array([float(root.children[a]["prior"]) for a in range(A)], dtype=np.float64)
    out = dict(obs=obs, visits=visits, root_value=np.float64(root.value()), root_n=np.int64(root.visit_count),
               root_priors=priors, depth_hist=np.array(depth, dtype=np.int64), seed=np.int64(seed),
               game=np.int64(game), move=np.int64(move), S=np.int64(S), N=np.int64(N), C=np.int64(C),
               c_puct=np.float64(2.0), pass_epsilon=np.float64(mn.config.pass_epsilon),
               dirichlet_epsilon=np.float64(mn.config.dirichlet_epsilon), discount=np.float64(mn.config.discount))
    np.savez_compressed(os.path.join(GOLDEN, f"mctsmain_{name}.npz"), **out)
    print("mcts(main.py)", name, "root N", root.visit_count, "value", root.value(), "depth", depth)


def synthetic_trajectories(N, B, seed):
    """main.py-format trajectories (main.py:636-713) from random legal
    playouts on the oracle GoEnv rules: observations T+2, actions T,
    policies T (random distributions), rewards T+1 (0 per move, a winner)."""
    from oracle import gogame
    A = N * N + 1
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(B):
        T = int(rng.integers(4, 16))
        st = gogame.init_state(N)
        obs, acts, pols, rews = [st.copy()], [], [], []
        for _t in range(T):
            legal = np.flatnonzero(gogame.invalid_moves(st) == 0)
            a = int(rng.choice(legal)) if rng.random() > 0.1 else N * N
            st = gogame.next_state(st, a)
            p = rng.random(A)
            acts.append(a)
            pols.append(p / p.sum())
            rews.append(0.0)
            obs.append(st.copy())
            if gogame.game_ended(st):
                break
        rews.append(float(rng.choice([-1.0, 1.0])))
        obs.append(st.copy())
        out.append(dict(observations=obs, actions=acts, rewards=rews, policies=pols))
    return out


def pack_trajectories(trajs):
    lens = np.array([len(t["actions"]) for t in trajs], dtype=np.int64)
    return dict(traj_len=lens,
                traj_obs=np.concatenate([np.stack(t["observations"]) for t in trajs]),
                traj_actions=np.concatenate([np.array(t["actions"], dtype=np.int64) for t in trajs]),
                traj_rewards=np.concatenate([np.array(t["rewards"], dtype=np.float64) for t in trajs]),
                traj_policies=np.concatenate([np.stack(t["policies"]) for t in trajs]))


def make_train(mn, N=5, C=32, B=4, seed=5, batches=2):
    """main.py's MuZeroAgent.train (main.py:381-522) on synthetic
    trajectories: random.randint (the start index, :395) replaced by a fixed
    sequence, the replay buffer by a stub that returns the whole batch.
    Records the returned losses, the priorities handed back, the lr and the
    weights after ``batches`` steps."""
    from oracle.weights import deterministic_state_dict
    A = N * N + 1
    mn.config.board_size = N
    mn.config.max_action_size = A
    mn.config.latent_dim = C
    trajs = synthetic_trajectories(N, B, seed)
    rng = np.random.default_rng(seed + 1)
    starts = [int(rng.integers(0, len(t["actions"]))) for _ in range(batches) for t in trajs]
    agent = mn.MuZeroAgent(N, C, A, 4)
    agent.net.load_state_dict({k: torch.from_numpy(v) for k, v in deterministic_state_dict(C, A, seed).items()})
    it = iter(starts)
    prios = []

    class Buf:
        def sample(self, bs):
            return trajs, list(range(bs))

        def update_priorities(self, idx, p):
            prios.append(list(p))

    saved = mn.random.randint
    mn.random.randint = lambda lo, hi: next(it)
    try:
        losses = [agent.train(Buf(), B) for _ in range(batches)]
    finally:
        mn.random.randint = saved
    sd = {f"w_{k}": v.detach().numpy().astype(np.float32) for k, v in agent.net.state_dict().items()}
    np.savez_compressed(os.path.join(GOLDEN, f"train_{N}x{N}_c{C}.npz"), N=np.int64(N), C=np.int64(C),
                        B=np.int64(B), seed=np.int64(seed), starts=np.array(starts, dtype=np.int64),
                        losses=np.array(losses, dtype=np.float64), priorities=np.array(prios, dtype=np.float64),
                        lr=np.float64(agent.optimizer.param_groups[0]["lr"]), **pack_trajectories(trajs), **sd)
    print("train", N, C, "losses", losses)


def _pack_record(rec):
    types = {
        "rewards": [type(r).__name__ for r in rec["rewards"]],
        "returns": [type(r).__name__ for r in rec["returns"]],
        "values": [type(v).__name__ for v in rec["values"]],
        "actions": [type(a).__name__ for a in rec["actions"]],
        "final_reward": type(rec["final_reward"]).__name__,
        "observations": sorted({f"{o.dtype}{o.shape}" for o in rec["observations"]}),
        "policies": sorted({f"{p.dtype}{p.shape}" for p in rec["policies"]}),
        "keys": list(rec.keys()),
    }
    arrays = dict(
        observations=np.stack(rec["observations"]),
        actions=np.array(rec["actions"], dtype=np.int64),
        policies=np.stack(rec["policies"]),
        values=np.array(rec["values"], dtype=np.float64),
        rewards=np.array(rec["rewards"], dtype=np.float64),
        returns=np.array(rec["returns"], dtype=np.float64),
        final_reward=np.float64(rec["final_reward"]),
    )
    return arrays, types


def make_game(sp, name, N=5, S=25, C=96, seed=1234, game=0, hooked=True):
    from oracle.goenv import GoEnv
    from oracle.weights import deterministic_state_dict
    A = N * N + 1
    _configure(sp, N, S)
    sd = deterministic_state_dict(C, A, 0)
    agent = sp.MuZeroAgent(N, C, A, S)
    agent.net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    agent.net.eval()
    env = GoEnv(N, komi=0, reward_method="real")
    h = None
    if hooked:
        h = _Hooked(sp, seed, game).install()
    else:
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
    import contextlib
    import io
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            hist = sp.run_self_play_game(agent, env, sp.config)
    finally:
        if h:
            h.restore()
    rec = {
        "observations": hist.observations, "actions": hist.actions, "policies": hist.policies,
        "values": hist.values, "rewards": hist.rewards, "returns": hist.calculate_returns(),
        "final_reward": hist.final_reward,
    }
    arrays, types = _pack_record(rec)
    arrays.update(seed=np.int64(seed), game=np.int64(game), S=np.int64(S), N=np.int64(N), C=np.int64(C))
    np.savez_compressed(os.path.join(GOLDEN, f"game_{name}.npz"), **arrays)
    with open(os.path.join(GOLDEN, f"game_{name}.json"), "w") as f:
        json.dump(types, f, indent=1)
    print("game", name, "moves", len(hist), "final", hist.final_reward)


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    sys.path.insert(0, REPO)
    sp = import_reference()
    torch.set_num_threads(1)
    make_net(sp, 5, 4)
    make_net(sp, 9, 4)
    make_net(sp, 19, 2)
    make_mcts(sp, "5x5_s25_empty", 5, 25, 0)
    make_mcts(sp, "5x5_s25_mid", 5, 25, 9)
    make_mcts(sp, "9x9_s200_empty", 9, 200, 0)
    make_mcts(sp, "9x9_s200_mid", 9, 200, 30)
    make_mcts(sp, "9x9_s400_mid", 9, 400, 45)
    make_mcts(sp, "19x19_s800_mid", 19, 800, 120)
    make_game(sp, "5x5_s25_hooked", hooked=True)
    make_game(sp, "5x5_s25_seeded", hooked=False)
    import main as mn  # noqa: E402  (the reference trainer module, same stubs)
    make_mcts_main(mn, "5x5_s25_mid", 5, 25, 7)
    make_mcts_main(mn, "9x9_s200_empty", 9, 200, 0)
    make_mcts_main(mn, "9x9_s200_mid", 9, 200, 26)
    make_train(mn)


def make_arena(mn, N=5, S=16, G=4, C=96, seed=21, seeds=(3, 4)):
    """main.py's SelfPlayEvaluator (main.py:526-611): G games between two
    main.py MuZeroNets (deterministic weights, seeds[0] = current,
    seeds[1] = best) on oracle.goenv.GoEnv, game i started by the current
    agent iff i is even (evaluate, :597-600).  Hooks per (game i, move m):
    MCTS's random.choice -> TAG_SELECT draw of the simulation, the Dirichlet
    draw -> injected_noise(seed, i, m), the evaluator's random.choice(valid
    actions) -> TAG_ACTION draw (SearchHooks.action_index).  Records every
    game's actions, env.winner(), play_game's result, and evaluate's win
    rate and Elo."""
    from oracle.goenv import GoEnv
    from oracle.rng import SearchHooks, injected_noise
    from oracle.weights import deterministic_state_dict
    A = N * N + 1
    mn.config.board_size = N
    mn.config.max_action_size = A
    mn.config.max_game_moves = int(N * N * 1.5)

    class _Agent:
        def __init__(self, s):
            self.net = mn.MuZeroNet(C, A)
            self.net.load_state_dict({k: torch.from_numpy(v) for k, v in deterministic_state_dict(C, A, s).items()})
            self.net.eval()
            self.action_size = A
            self.mcts_simulations = S

    cur, best = _Agent(seeds[0]), _Agent(seeds[1])
    st = {"game": 0, "move": 0, "sim": -1, "in_search": False, "hooks": None}
    saved = (mn.random.choice, mn.apply_dirichlet_noise, mn.MCTS.select_leaf, mn.MCTS.run)
    orig_select, orig_run = mn.MCTS.select_leaf, mn.MCTS.run

    def run(self_, obs):
        st["hooks"] = SearchHooks(seed, st["game"], st["move"])
        st["sim"], st["in_search"] = -1, True
        try:
            return orig_run(self_, obs)
        finally:
            st["in_search"] = False
            st["move"] += 1

    def select_leaf(self_, node):
        st["sim"] += 1
        return orig_select(self_, node)

    def choice(seq):
        h = st["hooks"]
        if st["in_search"]:
            return seq[h.choice_index(len(seq), st["sim"])]
        # the evaluator's fallback, drawn for the move just searched
        return seq[SearchHooks(seed, st["game"], st["move"] - 1).action_index(len(seq))]

    def noise(policy, alpha, epsilon):
        return (1 - epsilon) * policy + epsilon * injected_noise(seed, st["game"], st["move"], len(policy))
    mn.random.choice, mn.apply_dirichlet_noise = choice, noise
    mn.MCTS.select_leaf, mn.MCTS.run = select_leaf, run
    env = GoEnv(N)
    ev = mn.SelfPlayEvaluator(cur, best, env, num_games=G)
    actions, winners, results = [], [], []
    orig_step = env.step
    try:
        for i in range(G):
            st["game"], st["move"] = i, 0
            acts = []

            def step(a, _acts=acts):
                _acts.append(int(a))
                return orig_step(a)
            env.step = step
            with torch.no_grad():
                results.append(ev.play_game(starting_player=i % 2))
            winners.append(float(env.winner()))
            actions.append(acts)
        # evaluate()'s scoring of the same games (:597-611)
        wins = sum((1 - r) if i % 2 == 1 else r for i, r in enumerate(results))
        win_rate = wins / G
        expected = 1 / (1 + 10 ** ((ev.best_elo - ev.current_elo) / 400))
        elo = ev.current_elo
        if win_rate > mn.config.evaluation_win_threshold:
            elo = ev.current_elo + mn.config.elo_k * (win_rate - expected)
    finally:
        mn.random.choice, mn.apply_dirichlet_noise, mn.MCTS.select_leaf, mn.MCTS.run = saved
        env.step = orig_step
    L = max(len(a) for a in actions)
    pad = np.full((G, L), -1, np.int64)
    for i, a in enumerate(actions):
        pad[i, :len(a)] = a
    out = dict(actions=pad, lengths=np.array([len(a) for a in actions], np.int64),
               winners=np.array(winners, np.float64), results=np.array(results, np.int64),
               win_rate=np.float64(win_rate), elo=np.float64(elo), initial_elo=np.float64(mn.config.initial_elo),
               seed=np.int64(seed), seeds=np.array(seeds, np.int64), N=np.int64(N), S=np.int64(S),
               G=np.int64(G), C=np.int64(C), max_moves=np.int64(mn.config.max_game_moves))
    np.savez_compressed(os.path.join(GOLDEN, f"arena_{N}x{N}_s{S}.npz"), **out)
    print("arena", N, "lengths", out["lengths"], "winners", winners, "results", results, "win_rate", win_rate)


def arena_only():
    """Regenerate only the arena fixture (``python -m oracle.make_golden arena``)."""
    os.makedirs(GOLDEN, exist_ok=True)
    sys.path.insert(0, REPO)
    import_reference()
    torch.set_num_threads(1)
    import main as mn  # noqa: E402
    make_arena(mn)


def train_only():
    """Regenerate only the trainer fixture (``python -m oracle.make_golden train``)."""
    os.makedirs(GOLDEN, exist_ok=True)
    sys.path.insert(0, REPO)
    import_reference()
    torch.set_num_threads(1)
    import main as mn  # noqa: E402
    make_train(mn)


def main_only():
    """Regenerate only the main.py MCTS fixtures (``python -m oracle.make_golden main``)."""
    os.makedirs(GOLDEN, exist_ok=True)
    sys.path.insert(0, REPO)
    import_reference()
    torch.set_num_threads(1)
    import main as mn  # noqa: E402
    make_mcts_main(mn, "5x5_s25_mid", 5, 25, 7)
    make_mcts_main(mn, "9x9_s200_empty", 9, 200, 0)
    make_mcts_main(mn, "9x9_s200_mid", 9, 200, 26)


if __name__ == "__main__":
    {"main": main_only, "train": train_only, "arena": arena_only}.get(sys.argv[1] if sys.argv[1:] else "", main)()
