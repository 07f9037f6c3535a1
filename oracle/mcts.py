"""MCTS of self_play.py restated with injection hooks (TEST INFRASTRUCTURE ONLY).

Follows self_play.py:36-39 (``apply_dirichlet_noise``), :131-140
(``MCTSNode``), :148-237 (``MCTS.run``), :239-335 (``select_leaf``) and
:337-343 (``backpropagate``) operation for operation, keeping numpy's dtype
chain (root priors float64, child priors float32, Q/U/scores
float64).  With the default hooks it is the reference algorithm itself;
``tests/test_oracle_golden.py`` checks it against trees recorded from the
reference.

Hooks (all optional):

``choice(seq, sim)``      replaces ``random.choice`` (:287)
``noise(policy, alpha, eps)``    replaces ``apply_dirichlet_noise`` (:166)
``softmax(logits) -> f32[A]``    replaces ``torch.softmax(...).numpy()[0]``
                                 (:151, :204) -- used by replay tests that feed
                                 the engine's own softmax outputs
"""
import random

import numpy as np
import torch

from . import gogame
from .npsum import pairwise_sum  # noqa: F401  (documented order; np.sum used)


def apply_dirichlet_noise(policy, alpha, epsilon):
    noise = np.random.dirichlet([alpha] * len(policy))
    return (1 - epsilon) * policy + epsilon * noise


def root_valid_mask(observation, pass_epsilon=0.01):
    """valid_mask of self_play.py:152-158 / :363-370 (float64, pass last)."""
    valid_board = (observation[gogame.INVD_CHNL].flatten() == 0).astype(np.float32)
    pass_prior = pass_epsilon if valid_board.sum() > 0 else 1.0
    return np.concatenate([valid_board, np.array([pass_prior])])


def _default_softmax(logits):
    return torch.softmax(logits, dim=1).detach().cpu().numpy()[0]


class Node:
    """MCTSNode (self_play.py:131-140): children map a -> {'node','prior',...}."""

    __slots__ = ("latent", "prior", "visit_count", "value_sum", "children", "terminal")

    def __init__(self, latent, prior, terminal=False):
        self.latent = latent
        self.prior = prior
        self.visit_count = 0
        self.value_sum = 0
        self.children = {}
        self.terminal = terminal

    def value(self):
        return self.value_sum / self.visit_count if self.visit_count > 0 else 0


def _fill_children(node, priors, valid_mask, action_size):
    for a in range(action_size):
        node.children[a] = {
            "node": None,
            "prior": priors[a] if valid_mask[a] > 0 else 0.0,
            "visit_count": 0,
            "value_sum": 0,
            "action": a,
        }


def _normalise_masked(p, valid_mask):
    """:159-164 / :169-174 / :210-215 -- mask in place, renormalise, fallback."""
    p *= valid_mask
    s = p.sum()
    if s > 0:
        p /= s
        return p
    if valid_mask.sum() > 0:
        return np.ones_like(p) * valid_mask / valid_mask.sum()
    return np.ones_like(p) / len(p)


class MCTS:
    def __init__(self, muzero_net, action_size, num_simulations, c_puct=2.5,
                 dirichlet_alpha=0.15, dirichlet_epsilon=0.02, discount=0.99,
                 pass_epsilon=0.01, choice=None, noise=None, softmax=None,
                 device="cpu"):
        self.net = muzero_net
        self.action_size = action_size
        self.num_simulations = num_simulations
        self.c_puct = c_puct
        self.alpha = dirichlet_alpha
        self.epsilon = dirichlet_epsilon
        self.discount = discount
        self.pass_epsilon = pass_epsilon
        self.choice = choice or (lambda seq, sim: random.choice(seq))
        self.noise = noise or apply_dirichlet_noise
        self.softmax = softmax or _default_softmax
        self.device = device
        self._sim = 0

    def root_priors(self, observation, logits):
        """Root prior vector (float64) of :151-174."""
        valid_mask = root_valid_mask(observation, self.pass_epsilon)
        policy = self.softmax(logits)
        policy = _normalise_masked(policy, valid_mask)
        policy = self.noise(policy, self.alpha, self.epsilon)
        policy = _normalise_masked(policy, valid_mask)
        return policy, valid_mask

    def run(self, observation):
        obs = torch.FloatTensor(observation).unsqueeze(0).to(self.device)
        latent, _value, logits = self.net.initial_inference(obs)
        policy, valid_mask = self.root_priors(observation, logits)

        root = Node(latent[0], prior=0)
        _fill_children(root, policy, valid_mask, self.action_size)

        for sim in range(self.num_simulations):
            self._sim = sim
            path, action = self.select_leaf(root, valid_mask)
            leaf = path[-1]
            if leaf.terminal:
                self.backpropagate(path, 0)
                continue
            if action is None:
                self.backpropagate(path, leaf.value())
                continue
            act = torch.LongTensor([action]).to(self.device)
            with torch.no_grad():
                nxt, reward, value, child_logits = self.net.recurrent_inference(
                    leaf.latent.unsqueeze(0), act)
            pc = self.softmax(child_logits)
            pc = _normalise_masked(pc, valid_mask)         # ROOT mask (:210)
            child = Node(nxt[0], prior=0, terminal=False)
            _fill_children(child, pc, valid_mask, self.action_size)
            backup = reward.item() + self.discount * value.item()
            leaf.children[action]["node"] = child
            self.backpropagate(path + [child], backup)

        # :233-235 reads the never-updated per-child dict field: always zeros
        visit_counts = np.array([c["visit_count"] for _, c in root.children.items()])
        return root, visit_counts, root.value()

    def select_leaf(self, node, valid_mask):
        path = [node]
        while node.children:
            if node.visit_count > 0 and not any(c["prior"] > 0 for _, c in node.children.items()):
                node.terminal = True
                return path, None

            stats = {}
            q_expanded = []
            expanded = []
            for a, c in node.children.items():
                if valid_mask[a] > 0 and c["prior"] > 0:
                    ch = c["node"]
                    q = ch.value() if (ch is not None and ch.visit_count > 0) else 0.0
                    stats[a] = (q, c["prior"], ch.visit_count if ch is not None else 0)
                    if ch is not None:
                        q_expanded.append(q)
                        expanded.append(a)
            if not stats:
                node.terminal = True
                return path, None

            lo, hi = (min(q_expanded), max(q_expanded)) if q_expanded else (0, 0)
            best, best_score = None, -float("inf")
            unexpanded = [a for a, c in node.children.items()
                          if valid_mask[a] > 0 and c["prior"] > 0 and c["node"] is None]
            if unexpanded:
                best = self.choice(unexpanded, self._sim)
            else:
                n_parent = max(1, node.visit_count)
                for a in expanded:
                    q, prior, n = stats[a]
                    qn = (q - lo) / (hi - lo) if hi > lo else q
                    score = qn + self.c_puct * prior * np.sqrt(n_parent) / (1 + n)
                    if score > best_score:
                        best_score, best = score, a
            if best is None:
                node.terminal = True
                return path, None
            nxt = node.children[best]["node"]
            if nxt is None:
                return path, best
            node = nxt
            path.append(node)
        return path, None

    @staticmethod
    def backpropagate(path, value):
        for i, node in enumerate(reversed(path)):
            node.visit_count += 1
            node.value_sum += value * ((-1) ** i)


def tree_summary(root, action_size):
    """Per-root-child true visit counts, and nodes per depth (parity record)."""
    visits = np.zeros(action_size, dtype=np.int64)
    for a, c in root.children.items():
        if c["node"] is not None:
            visits[a] = c["node"].visit_count
    depth = []
    frontier = [root]
    while frontier:
        depth.append(len(frontier))
        nxt = []
        for n in frontier:
            nxt.extend(c["node"] for c in n.children.values() if c["node"] is not None)
        frontier = nxt
    return visits, depth
