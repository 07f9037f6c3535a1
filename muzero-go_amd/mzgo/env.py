"""``GoEnv`` drop-in whose board lives on the GPU (bit-exact integer kernels).

Replaces ``gym.make("gym_go:go-v0", size=N, komi=0, reward_method='real')``
as self_play.py:544 creates it and :455/:479/:502/:513 drive it: ``reset``,
``step`` (4-tuple; ``AssertionError`` on an invalid move or a step after the
end, like GymGo), ``winner``.  The rules are upstream GymGo's (SURVEY.md
Appendix B); they run in ``mzgo_board_step`` (muzero-go_amd/csrc/mzgo_board.hpp).
"""
import numpy as np
import torch

from .engine import Engine, EngineConfig

_BOARD_ERRORS = {1: "step after the game ended", 2: "Invalid move", 3: "action out of range"}


class GoEnv:
    def __init__(self, size, komi=0, reward_method="real", device=0):
        if reward_method != "real":
            raise ValueError("only reward_method='real' is used by self_play.py:544")
        self.size = size
        self.komi = komi
        self.reward_method = reward_method
        self._eng = Engine(EngineConfig(board_size=size, latent_dim=0, num_games=1,
                                        num_simulations=0, komi=float(komi), device=device))
        self.done = False
        self._winner = 0
        self.state_ = None
        self.reset()

    def _pull(self):
        self.state_ = self._eng.board_planes()[0].cpu().numpy()
        return np.copy(self.state_)

    def reset(self):
        self._eng.board_reset()
        self.done = False
        self._winner = 0
        return self._pull()

    def step(self, action):
        assert not self.done
        if isinstance(action, (tuple, list, np.ndarray)):
            assert 0 <= action[0] < self.size
            assert 0 <= action[1] < self.size
            action = self.size * action[0] + action[1]
        elif action is None:
            action = self.size ** 2
        status, winner = self._eng.board_step(torch.tensor([int(action)], dtype=torch.int32))
        if status[0] != 0:
            r, c = divmod(int(action), self.size)
            raise AssertionError((_BOARD_ERRORS.get(int(status[0]), "board error"), (r, c)))
        obs = self._pull()
        self.done = int(self.state_[5].max() == 1)
        self._winner = np.float64(winner[0]) if self.done else 0
        return obs, self.reward(), self.done, self.info()

    def game_ended(self):
        return int(self.state_[5].max() == 1)

    def winner(self):
        return self._winner if self.game_ended() else 0

    def reward(self):
        return self.winner()

    def info(self):
        invalid = (np.zeros(self.size ** 2 + 1) if self.game_ended()
                   else np.append(self.state_[3].flatten(), 0))
        return {"turn": int(self.state_[2].max()), "invalid_moves": invalid,
                "prev_player_passed": bool(self.state_[4].max() == 1)}
