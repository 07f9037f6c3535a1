"""Agent, game record and self-play loop of self_play.py restated (TEST INFRASTRUCTURE ONLY).

Follows ``MuZeroAgent.select_action`` (self_play.py:357-402), ``GameHistory``
(:415-450), ``run_self_play_game`` (:453-526) and the batch writer in
``main`` (:554-583).  Board printing (:466-476, :519-524) is I/O only and is
omitted.

RNG: with ``hooks=None`` the draws are the reference's own (CPython
``random.choice``, numpy's global ``RandomState``); with a hooks factory
(``oracle.rng.SearchHooks``) every draw comes from the engine's counter
streams, which is how engine and oracle are made to play the same game.

``compat``:
* ``"reference"`` -- the visit counts MCTS.run returns are the never-updated
  dict field, i.e. zeros, so the policy target is
  ``valid_mask / sum`` and the move is a uniform draw over legal moves;
* ``"fixed"`` -- the same formulas with the true child visit counts
  (``child['node'].visit_count``, as main.py:666-669 reads them).
"""
import os
import pickle
import random

import numpy as np
import torch

from .mcts import MCTS, root_valid_mask


class Agent:
    def __init__(self, net, board_size, action_size, num_simulations, compat="reference",
                 c_puct=2.5, dirichlet_alpha=0.15, dirichlet_epsilon=0.02, discount=0.99,
                 pass_epsilon=0.01, noise=None):
        if compat not in ("reference", "fixed"):
            raise ValueError(compat)
        self.net = net
        self.board_size = board_size
        self.action_size = action_size
        self.num_simulations = num_simulations
        self.compat = compat
        self.kw = dict(c_puct=c_puct, dirichlet_alpha=dirichlet_alpha,
                       dirichlet_epsilon=dirichlet_epsilon, discount=discount,
                       pass_epsilon=pass_epsilon, noise=noise)
        self.pass_epsilon = pass_epsilon
        self.last_root = None

    def select_action(self, observation, temperature, hooks=None):
        valid_mask = root_valid_mask(observation, self.pass_epsilon)
        choice = None
        if hooks is not None:
            choice = lambda seq, sim: seq[hooks.choice_index(len(seq), sim)]  # noqa: E731
        mcts = MCTS(self.net, self.action_size, self.num_simulations, choice=choice, **self.kw)
        with torch.no_grad():
            root, visit_counts, root_value = mcts.run(observation)
        self.last_root = root
        if self.compat == "fixed":
            visit_counts = np.array([c["node"].visit_count if c["node"] is not None else 0
                                     for _, c in root.children.items()])

        visit_counts = visit_counts * valid_mask
        policy_target = (visit_counts / visit_counts.sum() if visit_counts.sum() > 0
                         else valid_mask / valid_mask.sum())

        if temperature == 0:
            if visit_counts.sum() > 0:
                action = int(np.argmax(visit_counts))
            else:
                valid_actions = np.where(valid_mask > 0)[0]
                if hooks is None:
                    action = int(random.choice(valid_actions))
                else:
                    action = int(valid_actions[hooks.action_index(len(valid_actions))])
        else:
            vt = visit_counts ** (1.0 / temperature)
            vt = vt * valid_mask
            s = vt.sum()
            probabilities = vt / s if s > 0 else valid_mask / valid_mask.sum()
            if hooks is None:
                action = int(np.random.choice(self.action_size, p=probabilities))
            else:
                action = inverse_cdf(probabilities, hooks.action_uniform())
        return action, policy_target, root_value


def inverse_cdf(p, u):
    """numpy RandomState.choice(a, p=p) given its uniform draw u."""
    cdf = p.cumsum()
    cdf /= cdf[-1]
    return int(cdf.searchsorted(u, side="right"))


class GameHistory:
    def __init__(self, board_size, discount):
        self.board_size = board_size
        self.discount = discount
        self.observations, self.actions, self.rewards = [], [], []
        self.policies, self.values, self.dones = [], [], []
        self.final_reward = 0

    def add_step(self, obs, action, reward, done, policy, value):
        self.observations.append(obs)
        self.actions.append(action)
        self.rewards.append(reward)
        self.dones.append(done)
        self.policies.append(policy)
        self.values.append(value)

    def calculate_returns(self):
        """G_t back from the end, seeded with final_reward (:435-447)."""
        acc = self.final_reward
        out = []
        for r in reversed(self.rewards):
            acc = r + self.discount * acc
            out.append(acc)
        return list(reversed(out))

    def __len__(self):
        return len(self.actions)

    def to_record(self):
        """The dict written per game by self_play.py:569-578."""
        return {
            "observations": self.observations,
            "actions": self.actions,
            "policies": self.policies,
            "values": self.values,
            "rewards": self.rewards,
            "returns": self.calculate_returns(),
            "final_reward": self.final_reward,
        }


def run_self_play_game(agent, env, board_size, discount=0.99, temperature=1.0,
                       temperature_moves=15, hooks_factory=None):
    obs = env.reset()
    if isinstance(obs, tuple):
        obs = obs[0]
    done = False
    moves = 0
    history = GameHistory(board_size, discount)
    while not done and moves < board_size * board_size:
        temp = temperature if moves < temperature_moves else 0
        hooks = hooks_factory(moves) if hooks_factory else None
        action, policy, root_value = agent.select_action(obs, temp, hooks)
        result = env.step(action)
        if len(result) == 5:
            nobs, reward, terminated, truncated, _ = result
            done = terminated or truncated
        elif len(result) == 4:
            nobs, reward, done, _ = result
        else:
            raise ValueError(f"Unexpected number of return values from env.step: {len(result)}")
        if isinstance(nobs, tuple):
            nobs = nobs[0]
        history.add_step(obs, action, reward, done, policy, root_value)
        obs = nobs
        moves += 1
        if done:
            history.final_reward = env.winner()
            break
    if not done:
        history.final_reward = env.winner()
    return history


def save_batches(histories, output_dir, save_interval=10):
    """The periodic writer of self_play.py:554-583, slice quirk included.

    After game i (1-based) with i % save_interval == 0 or i == len(histories),
    writes ``self_play_batch_{i}.pkl`` holding the records of
    ``histories[i - save_interval:]`` *as they stood after game i* (the
    reference slices its growing list with a possibly negative start).
    """
    os.makedirs(output_dir, exist_ok=True)
    written = []
    n = len(histories)
    for i in range(n):
        if (i + 1) % save_interval == 0 or (i + 1) == n:
            sofar = histories[: i + 1]
            batch = [h.to_record() for h in sofar[i + 1 - save_interval:]]
            path = os.path.join(output_dir, f"self_play_batch_{i + 1}.pkl")
            with open(path, "wb") as f:
                pickle.dump(batch, f)
            written.append(path)
    return written
