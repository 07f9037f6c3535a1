"""Interactive play against the engine (play.py).

The reference's play.py (351 lines) pits a human against a MuZero agent on
a GymGo board.  Here the agent's search is the device MCTS in main.py's
variant (``search_variant="main"``: play.py:113-231 is the same algorithm --
root softmax x valid mask normalised once, Dirichlet mixed in, no re-mask;
child priors = softmax where the root mask is positive, not renormalised;
unexpanded-first; PUCT ``c_puct * P * sqrt(N + 1) / (1 + n)``; backup
without sign alternation) with play.py's constants (play.py:16-23, :111:
c_puct 10, Dirichlet(0.01) at 0.02, pass prior 0.01, 64 simulations), and
the board is the device ``GoEnv``.

Kept from the reference: the network's embedding table has int(1.5 N^2)
rows (play.py:193; only the first N^2 + 1 are ever used), the move rule
(argmax of the masked child visit counts, else a random valid action,
play.py:196-212), the coordinate format (column letter, 1-based row,
``pass``; play.py:226-245), the human/agent loop with a 2 N^2 move cap
(play.py:297-333) and the outcome message.  An illegal human move raises
``AssertionError`` from ``GoEnv.step`` as in the reference.  Randomness is
the engine's counter stream (seed, game, move) instead of Python's RNG.
"""
import sys
from dataclasses import dataclass

import numpy as np
import torch

from .env import GoEnv
from .net import MuZeroNet
from .search import MainMCTS, valid_mask_of
from .weights import _mix


@dataclass
class PlayConfig:                 # play.py:16-23, c_puct from MCTS (play.py:111)
    board_size: int = 6
    latent_dim: int = 64
    mcts_simulations: int = 64
    dirichlet_epsilon: float = 0.02
    dirichlet_alpha: float = 0.01
    discount: float = 0.99
    pass_epsilon: float = 0.01
    c_puct: float = 10.0


class PlayAgent:
    """play.py's ``MuZeroAgent`` (play.py:188-212) on the device search."""

    def __init__(self, board_size, latent_dim, env_action_size, num_simulations, *, config=None, seed=1234,
                 game=0, device="cuda"):
        self.config = config or PlayConfig(board_size=board_size, latent_dim=latent_dim,
                                           mcts_simulations=num_simulations)
        self.board_size = board_size
        self.action_size = env_action_size
        self.net = MuZeroNet(latent_dim, int(board_size * board_size * 1.5), board_size=board_size).to(device)
        self.net.eval()
        self.mcts_simulations = num_simulations
        self.seed, self.game, self.move = seed, game, 0

    def search(self, observation, noise=None):
        """The root after play.py's MCTS.run (play.py:113-183); visit counts of
        the root's children in ``root_child_visits``."""
        c = self.config
        m = MainMCTS(self.net, self.action_size, self.mcts_simulations, c_puct=c.c_puct, seed=self.seed,
                     game=self.game, dirichlet_alpha=c.dirichlet_alpha, dirichlet_epsilon=c.dirichlet_epsilon,
                     discount=c.discount, pass_epsilon=c.pass_epsilon)
        m.run(observation, move_index=self.move, noise=noise)
        return m

    def select_action(self, observation, noise=None):
        valid_mask = valid_mask_of(observation, self.config.pass_epsilon)
        m = self.search(observation, noise)
        visits = np.where(valid_mask > 0, np.asarray(m.root_child_visits), 0)
        key = _mix(_mix(self.seed) ^ ((self.game << 32) | self.move))
        self.move += 1
        if visits.sum() > 0:
            return int(np.argmax(visits))
        valid = np.nonzero(valid_mask)[0]
        h = _mix(key ^ (3 << 56))
        return int(valid[((h >> 32) * len(valid)) >> 32])

    def load_weights(self, weight_file):
        self.net.load_state_dict(torch.load(weight_file, map_location="cpu", weights_only=True))
        self.net.eval()


def board_text(obs, board_size):
    """The board as play.py's print_board prints it (play.py:215-224)."""
    lines = ["   " + " ".join(chr(ord("A") + j) for j in range(board_size))]
    for i in range(board_size):
        row = ["B" if obs[0, i, j] == 1 else ("W" if obs[1, i, j] == 1 else ".") for j in range(board_size)]
        lines.append(f"{i + 1:2d} " + " ".join(row))
    return "\n".join(lines)


def print_board(obs, board_size):
    print(board_text(obs, board_size))


def action_to_coord(action, board_size):
    if action == board_size * board_size:
        return "pass"
    row, col = divmod(action, board_size)
    return f"{chr(ord('A') + col)}{row + 1}"


def coord_to_action(coord, board_size):
    if coord.lower() == "pass":
        return board_size * board_size
    coord = coord.strip().upper()
    try:
        row = int(coord[1:]) - 1
    except Exception:
        raise ValueError("Invalid coordinate format")
    return row * board_size + (ord(coord[0]) - ord("A"))


def play(agent, env, human_is_black, read=input, write=print):
    """play.py:297-341: returns (outcome, final reward).  ``read`` / ``write``
    stand in for input() / print()."""
    N = agent.board_size
    observation = env.reset()
    done, reward = False, 0
    move_count, max_moves = 0, N * N * 2
    human_turn = human_is_black
    while not done and move_count < max_moves:
        write(board_text(observation, N))
        if human_turn:
            move = read("Your move (e.g., A1 or 'pass'): ")
            try:
                action = coord_to_action(move, N)
            except Exception:
                write("Invalid move format. Try again.")
                continue
        else:
            action = agent.select_action(observation)
            write(f"Agent move: {action_to_coord(action, N)}")
        observation, reward, done, _info = env.step(action)
        human_turn = not human_turn
        move_count += 1
    if not done:
        write(f"Reached max moves {move_count}, forcing game end.")
    write(board_text(observation, N))
    write("Game over!")
    if reward > 0:
        outcome = "win" if human_is_black else "loss"
    elif reward < 0:
        outcome = "loss" if human_is_black else "win"
    else:
        outcome = "draw"
    write(f"Final outcome: {outcome}. Final reward: {reward}")
    return outcome, reward


def main(argv=None, read=input, write=print):
    argv = sys.argv[1:] if argv is None else argv
    c = PlayConfig()
    N = c.board_size
    env = GoEnv(N, komi=0, reward_method="real")
    agent = PlayAgent(N, c.latent_dim, N * N + 1, c.mcts_simulations, config=c)
    weight_file = argv[0] if argv else "muzero_model_final.pth"
    try:
        agent.load_weights(weight_file)
        write(f"Loaded weights from {weight_file}")
    except Exception as e:
        write(f"Error loading weight file: {e}")
        return None
    while True:
        user_color = read("Do you want to play as Black (B) or White (W)? ").strip().upper()
        if user_color in ("B", "W"):
            break
        write("Invalid input. Please enter 'B' or 'W'.")
    return play(agent, env, user_color == "B", read, write)


if __name__ == "__main__":
    main()
