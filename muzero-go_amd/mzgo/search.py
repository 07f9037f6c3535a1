"""``MCTS`` and ``MuZeroAgent`` drop-ins backed by the device search.

Reference: ``MCTS`` (self_play.py:142-343) and ``MuZeroAgent``
(self_play.py:347-412).  ``MCTS.run`` runs the whole search on the GPU
(``mzgo_search``: representation, root priors, S simulations of select /
fused dynamics+prediction / expand / backup) and returns a read-only view of
the device tree shaped like the reference's ``MCTSNode`` graph.

Randomness: the reference's ``random.choice`` / ``np.random`` draws are
replaced by the counter-based streams keyed by (seed, game, move) that the
batched engine uses (SURVEY.md §7 "RNG parity").
"""
import numpy as np
import torch

from .engine import EngineConfig
from .net import MuZeroNet
from .resnet import ResMuZeroNet


class TreeNode:
    """Read-only view of one device tree node with MCTSNode's attributes."""

    __slots__ = ("_t", "_i", "_children")

    def __init__(self, tree, index):
        self._t = tree
        self._i = index
        self._children = None

    @property
    def visit_count(self):
        return int(self._t["visits"][self._i])

    @property
    def value_sum(self):
        return float(self._t["value_sum"][self._i])

    @property
    def terminal(self):
        return False

    def value(self):
        n = self.visit_count
        return self.value_sum / n if n > 0 else 0

    @property
    def children(self):
        if self._children is None:
            t, i = self._t, self._i
            A = t["child"].shape[1]
            row = t["child"][i]
            pri = t["root_prior"] if i == 0 else t["prior"][i]
            cast = np.float64 if i == 0 else np.float32
            self._children = {
                a: {"node": TreeNode(t, int(row[a])) if row[a] >= 0 else None,
                    "prior": cast(pri[a]), "visit_count": 0, "value_sum": 0, "action": a}
                for a in range(A)
            }
        return self._children


class MCTS:
    def __init__(self, muzero_net, action_size, num_simulations, c_puct=2.5, *, compat="reference",
                 seed=1234, game=0, dirichlet_alpha=0.15, dirichlet_epsilon=0.02, discount=0.99,
                 pass_epsilon=0.01, dynamics="factored"):
        if not isinstance(muzero_net, (MuZeroNet, ResMuZeroNet)):
            raise TypeError("mzgo.MCTS searches with an mzgo.MuZeroNet or ResMuZeroNet (HIP engine); got "
                            f"{type(muzero_net).__name__}")
        if action_size != muzero_net.board_size ** 2 + 1:
            raise ValueError("action_size must be the board's N*N+1 actions")
        self.net = muzero_net
        self.action_size = action_size
        self.num_simulations = num_simulations
        self.c_puct = c_puct
        self.cfg = dict(c_puct=c_puct, compat=compat, seed=seed, game_base=game,
                        dirichlet_alpha=dirichlet_alpha, dirichlet_epsilon=dirichlet_epsilon,
                        discount=discount, pass_epsilon=pass_epsilon, dynamics=dynamics)
        self.compat = compat
        self.root_child_visits = None

    def run(self, observation, move_index=0, noise=None):
        N = self.net.board_size
        obs = torch.as_tensor(np.asarray(observation), dtype=torch.float32).reshape(1, 6, N, N)
        eng = self.net.engine(num_games=1, num_simulations=self.num_simulations, **self.cfg)
        visits, value = eng.search(obs, noise=noise, move_index=move_index)
        tree = eng.tree(0)
        root = TreeNode(tree, 0)
        self.root_child_visits = visits[0].cpu().numpy().astype(np.int64)
        if self.compat == "reference":
            visit_counts = np.zeros(self.action_size, dtype=np.int64)  # self_play.py:233-235
        else:
            visit_counts = self.root_child_visits.copy()
        return root, visit_counts, float(value[0].item())


class MainMCTS:
    """main.py's MCTS (main.py:246-368; the trainer's self-play and the arena
    evaluator) on the device search: ``MainMCTS(net, A, S, c_puct=2).run(obs)
    -> root``.  Defaults are main.py's Config (:37-52): Dirichlet(0.03) with
    epsilon 0.25, pass prior 0.05, discount 0.99."""

    def __init__(self, muzero_net, action_size, num_simulations, c_puct=2, *, seed=1234, game=0,
                 dirichlet_alpha=0.03, dirichlet_epsilon=0.25, discount=0.99, pass_epsilon=0.05):
        self._m = MCTS(muzero_net, action_size, num_simulations, c_puct, compat="fixed", seed=seed, game=game,
                       dirichlet_alpha=dirichlet_alpha, dirichlet_epsilon=dirichlet_epsilon,
                       discount=discount, pass_epsilon=pass_epsilon)
        self._m.cfg["search_variant"] = "main"
        self.net, self.action_size, self.num_simulations = muzero_net, action_size, num_simulations

    @property
    def root_child_visits(self):
        return self._m.root_child_visits

    def run(self, observation, move_index=0, noise=None):
        root, _visits, value = self._m.run(observation, move_index=move_index, noise=noise)
        self.root_value = value
        return root


def valid_mask_of(observation, pass_epsilon=0.01):
    """valid_mask of self_play.py:363-370 (float64, pass last)."""
    valid_board = (np.asarray(observation)[3].flatten() == 0).astype(np.float32)
    pass_prior = pass_epsilon if valid_board.sum() > 0 else 1.0
    return np.concatenate([valid_board, np.array([pass_prior])])


class MuZeroAgent:
    """Single-game agent (self_play.py:347-412) on the device search.

    Action choice follows select_action's formulas on the host with the
    engine's counter RNG (draw (seed, game, move, TAG_ACTION, 0)).
    """

    def __init__(self, board_size, latent_dim, env_action_size, num_simulations, *, compat="reference",
                 seed=1234, game=0, device="cuda"):
        self.board_size = board_size
        self.action_size = env_action_size
        self.net = MuZeroNet(latent_dim, board_size * board_size + 1).to(device)
        self.net.eval()
        self.mcts_simulations = num_simulations
        self.compat = compat
        self.seed = seed
        self.game = game
        self.move = 0

    def select_action(self, observation, temperature):
        from .weights import _mix
        valid_mask = valid_mask_of(observation)
        mcts = MCTS(self.net, self.action_size, self.mcts_simulations, compat=self.compat,
                    seed=self.seed, game=self.game)
        root, visit_counts, root_value = mcts.run(observation, move_index=self.move)
        key = _mix(_mix(self.seed) ^ ((self.game << 32) | self.move))
        h = _mix(key ^ (3 << 56))
        self.move += 1

        visit_counts = visit_counts * valid_mask
        policy_target = (visit_counts / visit_counts.sum() if visit_counts.sum() > 0
                         else valid_mask / valid_mask.sum())
        if temperature == 0:
            if visit_counts.sum() > 0:
                action = int(np.argmax(visit_counts))
            else:
                valid = np.where(valid_mask > 0)[0]
                action = int(valid[((h >> 32) * len(valid)) >> 32])
        else:
            vt = visit_counts ** (1.0 / temperature) * valid_mask
            s = vt.sum()
            p = vt / s if s > 0 else valid_mask / valid_mask.sum()
            cdf = p.cumsum()
            cdf /= cdf[-1]
            action = int(cdf.searchsorted(float(h >> 11) * 2.0 ** -53, side="right"))
        return action, policy_target, root_value

    def load_weights(self, weight_file):
        state_dict = torch.load(weight_file, map_location="cpu", weights_only=True)
        self.net.load_state_dict(state_dict)
        self.net.eval()
        print(f"Loaded weights from {weight_file}")


__all__ = ["MCTS", "MuZeroAgent", "TreeNode", "EngineConfig", "valid_mask_of"]
