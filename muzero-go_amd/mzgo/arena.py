"""The trainer's arena evaluator (main.py:526-611) on the device.

``SelfPlayEvaluator(current, best, num_games).evaluate() -> (win_rate, elo)``
plays all games at once: one ``mzgo_arena_move`` launch advances every game
by one move, the side to move searching with its own network (main.py's
MCTS variant, ``search_variant="main"``) and moving by main.py's rule
(argmax of valid child visit counts, else a random valid action).

Kept from the reference: game i starts with the current agent iff i is even;
``play_game``'s result is flipped a second time in ``evaluate`` for games the
best agent started (main.py:597-600), so a current-agent win in those games
counts as a loss -- the win rate is the reference's number, quirk included;
truncated games have winner 0 (upstream ``winner()`` is 0 unless the game
ended); the Elo update is :603-606.  Randomness: counter streams keyed by
(seed, game id, move) as everywhere in the engine (not Python's RNG).
"""
import numpy as np
import torch

from .selfplay import history_from_device


def _net_of(x):
    return getattr(x, "net", x)


class SelfPlayEvaluator:
    def __init__(self, current_agent, best_agent, env=None, num_games=20, *, num_simulations=None,
                 initial_elo=1000, elo_k=32, win_threshold=0.55, max_moves=None, seed=1234,
                 c_puct=2.0, dirichlet_alpha=0.03, dirichlet_epsilon=0.25, pass_epsilon=0.05,
                 discount=0.99, komi=0.0):
        self.current, self.best = _net_of(current_agent), _net_of(best_agent)
        if (self.current.board_size, self.current.latent_dim) != (self.best.board_size, self.best.latent_dim):
            raise ValueError("arena networks differ in board size / latent_dim")
        N = self.current.board_size
        self.num_games = num_games
        self.S = num_simulations or getattr(current_agent, "mcts_simulations", 256)
        self.max_moves = max_moves or int(N * N * 1.5)          # main.py:53
        self.current_elo = float(initial_elo)
        self.best_elo = float(initial_elo)
        self.elo_k, self.win_threshold = elo_k, win_threshold
        self.discount = discount
        self.epoch = 0
        self.cfg = dict(search_variant="main", compat="fixed", c_puct=c_puct, dirichlet_alpha=dirichlet_alpha,
                        dirichlet_epsilon=dirichlet_epsilon, pass_epsilon=pass_epsilon, discount=discount,
                        max_moves=self.max_moves, komi=float(komi), seed=seed)

    def play(self, noise=None):
        """Play all games; returns the per-game winner (+1 black, -1 white, 0).
        noise: test hook, Dirichlet samples float64 [num_games, max_moves, A]
        in place of the counter-RNG draws (Engine.inject_noise)."""
        eng = self.current.engine(self.num_games, self.S, **self.cfg)
        opp = self.best.engine(self.num_games, self.S, **self.cfg)
        eng.inject_noise(noise)
        eng.selfplay_reset(self.epoch)
        eng.arena_move(opp, self.max_moves)          # whole games, one launch
        if noise is not None:
            torch.cuda.synchronize(eng.device)       # the launch reads the samples until it ends
            eng.inject_noise(None)
        self.epoch += 1
        N = self.current.board_size
        return np.array([float(history_from_device(eng.record(g), N, self.discount).final_reward)
                         for g in range(self.num_games)])

    @staticmethod
    def win_rate(winners):
        """main.py:583-601 on per-game winners (+1 black, -1 white, 0)."""
        current_wins = 0
        for i, w in enumerate(winners):
            starting_player = i % 2
            result = (1 if w == 1 else 0) if starting_player == 0 else (1 if w == -1 else 0)
            if starting_player == 1:
                result = 1 - result                                  # main.py:599-600, kept
            current_wins += result
        return current_wins / len(winners)

    def evaluate(self):
        win_rate = self.win_rate(self.play())
        expected = 1 / (1 + 10 ** ((self.best_elo - self.current_elo) / 400))
        if win_rate > self.win_threshold:
            self.current_elo += self.elo_k * (win_rate - expected)
            self.best_elo += self.elo_k * ((1 - win_rate) - (1 - expected))
        return win_rate, self.current_elo
