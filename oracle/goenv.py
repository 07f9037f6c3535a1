"""GymGo ``GoEnv`` restated (TEST INFRASTRUCTURE ONLY; parity unpinned, see gogame).

Mirrors upstream ``gym_go/envs/go_env.py`` as the reference drives it:
``gym.make("gym_go:go-v0", size=N, komi=0, reward_method='real')``
(self_play.py:544), ``reset`` (:455), ``step`` returning the 4-tuple
(:479-488), ``winner`` (:502, :513).
"""
import numpy as np

from . import gogame


class GoEnv:
    def __init__(self, size, komi=0, reward_method="real"):
        if reward_method not in ("real", "heuristic"):
            raise ValueError(reward_method)
        self.size = size
        self.komi = komi
        self.reward_method = reward_method
        self.state_ = gogame.init_state(size)
        self.done = False

    def reset(self):
        self.state_ = gogame.init_state(self.size)
        self.done = False
        return np.copy(self.state_)

    def step(self, action):
        assert not self.done
        if isinstance(action, (tuple, list, np.ndarray)):
            assert 0 <= action[0] < self.size
            assert 0 <= action[1] < self.size
            action = self.size * action[0] + action[1]
        elif action is None:
            action = self.size ** 2
        self.state_ = gogame.next_state(self.state_, action, canonical=False)
        self.done = gogame.game_ended(self.state_)   # int 0/1 as upstream
        return np.copy(self.state_), self.reward(), self.done, self.info()

    def game_ended(self):
        return gogame.game_ended(self.state_)

    def winning(self):
        return gogame.winning(self.state_, self.komi)

    def winner(self):
        if self.game_ended():
            return self.winning()
        return 0

    def reward(self):
        if self.reward_method == "real":
            return self.winner()
        black, white = gogame.areas(self.state_)
        diff = black - white - self.komi
        if self.game_ended():
            return (1 if diff > 0 else -1) * self.size ** 2
        return diff

    def info(self):
        return {
            "turn": gogame.turn(self.state_),
            "invalid_moves": gogame.invalid_moves(self.state_),
            "prev_player_passed": gogame.prev_player_passed(self.state_),
        }
