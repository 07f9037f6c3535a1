"""Batched self-play: G concurrent games resident on one GPU, and the
reference's game-record format.

Reference: ``GameHistory`` (self_play.py:415-450), ``run_self_play_game``
(:453-526) and ``main``'s pickle writer (:529-596).  Every move of every
unfinished game is one iteration of the ``k_selfplay_move`` kernel on the
device: observation recorded, MCTS (S simulations), action choice, board step,
result recorded; one launch plays any number of moves of every game (whole
games by default) -- the host only harvests finished records.

CLI (replaces ``python self_play.py``)::

    python -m mzgo.selfplay --weights W.pth --num_games 64 --simulations 200 \
        --board-size 9 --output_dir self_play_data [--random-init SEED] [--parallel-games G]
"""
import argparse
import os
import pickle
import sys
import time

import numpy as np
import torch

from .net import MuZeroNet
from .weights import deterministic_state_dict


class GameHistory:
    """The reference's per-game record (self_play.py:415-450)."""

    def __init__(self, board_size, discount):
        self.board_size = board_size
        self.discount = discount
        self.observations, self.actions, self.rewards = [], [], []
        self.policies, self.values, self.dones = [], [], []
        self.final_reward = 0

    def calculate_returns(self):
        acc = self.final_reward
        out = []
        for r in reversed(self.rewards):
            acc = r + self.discount * acc
            out.append(acc)
        return list(reversed(out))

    def __len__(self):
        return len(self.actions)

    def to_record(self):
        return {
            "observations": self.observations,
            "actions": self.actions,
            "policies": self.policies,
            "values": self.values,
            "rewards": self.rewards,
            "returns": self.calculate_returns(),
            "final_reward": self.final_reward,
        }


def history_from_device(rec, board_size, discount):
    """Rebuild the reference's Python objects from an engine record.

    Types follow the reference: observations float64 [6,N,N]; actions int;
    policies float64 [A]; values float; rewards int 0 except the final step
    of a game that ended by double pass (np.float64 winner); final_reward
    np.float64 winner if ended, else int 0 (env.winner() of an unfinished
    game, self_play.py:513).
    """
    N = board_size
    L = rec["length"]
    h = GameHistory(N, discount)
    pass_a = N * N
    acts = [int(a) for a in rec["action"]]
    ended = L >= 2 and acts[-1] == pass_a and acts[-2] == pass_a
    for t in range(L):
        o = np.zeros((6, N, N))
        s = rec["stones"][t].reshape(N, N)
        f = int(rec["flags"][t])
        o[0] = s == 1
        o[1] = s == 2
        o[2] = f & 1
        o[3] = rec["invd"][t].reshape(N, N)
        o[4] = (f >> 1) & 1
        o[5] = (f >> 2) & 1
        last = t == L - 1
        h.observations.append(o)
        h.actions.append(acts[t])
        h.policies.append(np.array(rec["policy"][t], dtype=np.float64))
        h.values.append(float(rec["value"][t]))
        h.rewards.append(np.float64(rec["reward"][t]) if (ended and last) else 0)
        h.dones.append(int(ended and last))
    h.final_reward = np.float64(rec["final_reward"]) if ended else 0
    return h


class SelfPlay:
    """G self-play games advanced in lockstep on one GPU."""

    def __init__(self, net, num_games, num_simulations, *, seed=1234, compat="reference",
                 max_moves=0, temperature=1.0, temperature_moves=15, komi=0.0, game_base=0,
                 discount=0.99, c_puct=2.5, dirichlet_alpha=0.15, dirichlet_epsilon=0.02,
                 pass_epsilon=0.01, search_variant="self_play", dynamics="factored"):
        self.net = net
        self.N = net.board_size
        self.G = num_games
        self.S = num_simulations
        self.discount = discount
        self.engine = net.engine(num_games, num_simulations, seed=seed, compat=compat,
                                 max_moves=max_moves, temperature=temperature,
                                 temperature_moves=temperature_moves, komi=float(komi),
                                 game_base=game_base, discount=discount, c_puct=c_puct,
                                 dirichlet_alpha=dirichlet_alpha,
                                 dirichlet_epsilon=dirichlet_epsilon, pass_epsilon=pass_epsilon,
                                 search_variant=search_variant, dynamics=dynamics)
        self.max_moves = self.engine.M
        self.epoch = 0

    def reset(self, epoch=None):
        if epoch is not None:
            self.epoch = epoch
        self.engine.selfplay_reset(self.epoch)

    def move(self, moves=1):
        """Enqueue ``moves`` moves for every unfinished game, one launch
        (asynchronous).  Tower engines (ResMuZeroNet) enqueue a move as a
        sequence of launches and, for moves > 4, BLOCK every 4 moves to read
        the games' status (mzgo_selfplay_moves): they stop once every game has
        ended, with the records of ``moves`` single-move calls."""
        self.engine.selfplay_move(moves)

    def play(self):
        """Play all G games to the end (one launch); returns their GameHistory objects."""
        self.reset()
        self.move(self.max_moves)
        if self.engine.counters()["playing"] != 0:
            raise RuntimeError("games still playing after max_moves moves")
        hist = self.histories()
        self.epoch += 1
        return hist

    def histories(self):
        return [history_from_device(self.engine.record(g), self.N, self.discount) for g in range(self.G)]


def save_batches(histories, output_dir, save_interval=10):
    """self_play.py:554-583's periodic writer, slice quirk included."""
    os.makedirs(output_dir, exist_ok=True)
    written = []
    n = len(histories)
    for i in range(n):
        if (i + 1) % save_interval == 0 or (i + 1) == n:
            batch = [h.to_record() for h in histories[: i + 1][i + 1 - save_interval:]]
            path = os.path.join(output_dir, f"self_play_batch_{i + 1}.pkl")
            with open(path, "wb") as f:
                pickle.dump(batch, f)
            written.append(path)
            print(f"Saved batch of {len(batch)} games to {path}")
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(description="MuZero-Go self-play on the MI355X engine.")
    ap.add_argument("--weights", type=str, default=None, help="state_dict (.pth) of the reference MuZeroNet")
    ap.add_argument("--random-init", type=int, default=None, help="use deterministic weights with this seed")
    ap.add_argument("--num_games", type=int, default=1)
    ap.add_argument("--output_dir", type=str, default="self_play_data")
    ap.add_argument("--simulations", type=int, default=128)
    ap.add_argument("--board-size", type=int, default=6, help="self_play.py:20 uses 6")
    ap.add_argument("--latent-dim", type=int, default=96)
    ap.add_argument("--parallel-games", type=int, default=256, help="games resident on the GPU at once")
    ap.add_argument("--compat", choices=["reference", "fixed"], default="reference")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--save-interval", type=int, default=10)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher N > 1 starts N child processes")
    args = ap.parse_args(argv)
    if (args.weights is None) == (args.random_init is None):
        ap.error("give exactly one of --weights or --random-init (self_play.py:531's default path is cluster-only)")
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # nothing has touched the GPU yet: one fresh process per rank
        from .launch import spawn_ranks
        sys.exit(spawn_ranks(args.gpus, [sys.executable, "-m", "mzgo.selfplay",
                                         *(sys.argv[1:] if argv is None else argv)]))
    if args.gpus is not None and int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')}")

    # one process per GPU under torchrun: games sharded by global id, weights
    # broadcast from rank 0, finished games gathered to rank 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one-GPU rehearsal (as bench.py): every rank on cuda:0, gloo for RCCL
    if os.environ.get("MZGO_SHARE_DEVICE") == "1":
        local = 0
    if world > 1:
        import torch.distributed as dist

        from . import distributed as mdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        backend = os.environ.get("MZGO_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    N = args.board_size
    net = MuZeroNet(args.latent_dim, N * N + 1).to(f"cuda:{local}").eval()
    if rank == 0:
        if args.weights:
            net.load_state_dict(torch.load(args.weights, map_location="cpu", weights_only=True))
            print(f"Loaded weights from {args.weights}")
        else:
            net.load_state_dict(deterministic_state_dict(args.latent_dim, N * N + 1, args.random_init))
    if world > 1:
        mdist.broadcast_weights(net)

    # every rank plays the same number of games per round (gathers need equal
    # buffers): ``per`` ids per rank, ids >= num_games are dropped on rank 0
    per = -(-args.num_games // world)
    base = rank * per
    histories = []
    t0 = time.time()
    done = 0
    while done < per:
        G = min(args.parallel_games, per - done)
        sp = SelfPlay(net, G, args.simulations, seed=args.seed, compat=args.compat, game_base=base + done)
        if world == 1:
            histories.extend((base + done + g, h) for g, h in enumerate(sp.play()))
        else:
            sp.play()
            got = mdist.gather_histories(sp.engine, N, sp.discount)
            if rank == 0:
                histories.extend((r * per + done + g, got[r * G + g]) for r in range(world) for g in range(G))
        done += G
        if rank == 0:
            print(f"{min(done * world, args.num_games)}/{args.num_games} games done")
    histories = [h for gid, h in sorted(histories, key=lambda x: x[0]) if gid < args.num_games]
    dt = time.time() - t0
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        save_batches(histories, args.output_dir, args.save_interval)
        print(f"Finished {args.num_games} games in {dt:.2f} seconds.")
        print(f"Average time per game: {dt / max(1, args.num_games):.2f} seconds.")


if __name__ == "__main__":
    main()
