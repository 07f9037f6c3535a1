"""The trainer-side MCTS of main.py restated (TEST INFRASTRUCTURE ONLY).

main.py:246-368 runs its own MCTS variant for self-play and for the arena
evaluator (main.py:526-611); SURVEY.md §8(f) item 3.  It differs from
self_play.py's (oracle/mcts.py) in:

* root (:256-287): softmax x valid_mask (in place, f32), normalised only if
  the sum is positive (no uniform fallback), Dirichlet noise, and no re-mask
  / renormalisation afterwards; root prior = p[a] if valid_mask[a] > 0;
* child priors (:299-309): softmax(child logits)[a] if valid_mask[a] > 0 --
  not renormalised;
* select (:318-364): no terminal test; unexpanded = prior > 0 and no node;
  PUCT u = c_puct * P * sqrt(N + 1) / (1 + n) with c_puct = 2; when no child
  has a positive prior the walk stops with no action, and the simulation
  does nothing (:296 ``if not leaf.terminal and action is not None``);
* backup (:366-368): every node on the path gets +value (no sign flip).

Hooks as in oracle/mcts.py: ``choice(seq, sim)``, ``noise(policy, alpha,
eps)``, ``softmax(logits)``.
"""
import random

import numpy as np
import torch

from .mcts import Node, _default_softmax, root_valid_mask


def apply_dirichlet_noise(policy, alpha, epsilon):
    noise = np.random.dirichlet([alpha] * len(policy))
    return (1 - epsilon) * policy + epsilon * noise


class MCTSMain:
    def __init__(self, muzero_net, action_size, num_simulations, c_puct=2,
                 dirichlet_alpha=0.03, dirichlet_epsilon=0.25, discount=0.99,
                 pass_epsilon=0.05, choice=None, noise=None, softmax=None, device="cpu"):
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
        valid_mask = root_valid_mask(observation, self.pass_epsilon)
        policy = self.softmax(logits)            # f32
        policy *= valid_mask                     # in place: stays f32 (:268)
        s = policy.sum()
        if s > 0:
            policy /= s
        policy = self.noise(policy, self.alpha, self.epsilon)   # -> f64 (:276)
        return policy, valid_mask

    def run(self, observation):
        obs = torch.FloatTensor(observation).unsqueeze(0).to(self.device)
        latent, _value, logits = self.net.initial_inference(obs)
        policy, valid_mask = self.root_priors(observation, logits)
        root = Node(latent[0], prior=0)
        for a in range(self.action_size):
            root.children[a] = {"node": None, "prior": policy[a] if valid_mask[a] > 0 else 0,
                                "visit_count": 0, "value_sum": 0, "action": a}
        for sim in range(self.num_simulations):
            self._sim = sim
            path, action = self.select_leaf(root)
            leaf = path[-1]
            if leaf.terminal or action is None:
                continue
            act = torch.LongTensor([action]).to(self.device)
            with torch.no_grad():
                nxt, reward, value, child_logits = self.net.recurrent_inference(leaf.latent.unsqueeze(0), act)
            pc = self.softmax(child_logits)
            child = Node(nxt[0], prior=0, terminal=False)
            for a in range(self.action_size):
                child.children[a] = {"node": None, "prior": pc[a] if valid_mask[a] > 0 else 0,
                                     "visit_count": 0, "value_sum": 0, "action": a}
            backup = reward.item() + self.discount * value.item()
            leaf.children[action]["node"] = child
            self.backpropagate(path + [child], backup)
        return root

    def select_leaf(self, node):
        path = [node]
        while node.children:
            unexpanded = [a for a, c in node.children.items() if c["prior"] > 0 and c["node"] is None]
            if unexpanded:
                return path, self.choice(unexpanded, self._sim)
            q_values = []
            for a, c in node.children.items():
                if c["prior"] <= 0:
                    continue
                ch = c["node"]
                q_values.append(ch.value() if (ch is not None and ch.visit_count > 0) else 0.0)
            lo, hi = (min(q_values), max(q_values)) if q_values else (0, 0)
            best_score, best = -float("inf"), None
            for a, c in node.children.items():
                if c["prior"] <= 0:
                    continue
                ch = c["node"]
                q = ch.value() if (ch is not None and ch.visit_count > 0) else 0.0
                qn = (q - lo) / (hi - lo) if hi > lo else q
                n = ch.visit_count if ch is not None else 0
                score = qn + self.c_puct * c["prior"] * np.sqrt(node.visit_count + 1) / (1 + n)
                if score > best_score:
                    best_score, best = score, a
            if best is None:
                break
            node = node.children[best]["node"]
            path.append(node)
        return path, None

    @staticmethod
    def backpropagate(path, value):
        for node in reversed(path):
            node.visit_count += 1
            node.value_sum += value
