"""Engine: one ``mzgo_engine`` (include/mzgo.h) holding G game slots on one GPU.

The engine owns the device-resident state of the hot path: latent pools and
search trees for every slot, the Go boards and the self-play records.  Caller
tensors (inputs/outputs of inference and search) are torch CUDA tensors.
"""
import ctypes
from dataclasses import dataclass, fields

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_of


@dataclass
class EngineConfig:
    """Engine parameters; defaults are the reference's (self_play.py:19-33, :143, :544)."""

    board_size: int = 9
    latent_dim: int = 96
    num_games: int = 1
    num_simulations: int = 128
    max_moves: int = 0            # 0 = N*N (self_play.py:461)
    compat: str = "reference"     # "reference" (zero visit counts, §0.6) or "fixed"
    temperature_moves: int = 15
    search_variant: str = "self_play"   # "self_play" (self_play.py MCTS) or "main" (main.py:246-368)
    c_puct: float = 2.5
    discount: float = 0.99
    dirichlet_alpha: float = 0.15
    dirichlet_epsilon: float = 0.02
    pass_epsilon: float = 0.01
    temperature: float = 1.0
    komi: float = 0.0
    seed: int = 1234
    game_base: int = 0
    device: int = 0
    dynamics: str = "factored"    # "factored" (conv once per parent, mzgo_expand.hpp) or "direct"
    tower: int = 0                # 1: the residual-tower network (BASELINE config 5, mzgo.resnet)
    res_blocks: int = 0           # its residual blocks per network

    def to_c(self):
        c = _lib.Config()
        lib.mzgo_default_config(ctypes.byref(c), self.board_size)
        for f in fields(self):
            v = getattr(self, f.name)
            if f.name == "compat":
                if v not in ("reference", "fixed"):
                    raise ValueError(f"compat must be 'reference' or 'fixed', not {v!r}")
                v = 0 if v == "reference" else 1
            if f.name == "search_variant":
                if v not in ("self_play", "main"):
                    raise ValueError(f"search_variant must be 'self_play' or 'main', not {v!r}")
                v = 0 if v == "self_play" else 1
            if f.name == "dynamics":
                if v not in ("factored", "direct"):
                    raise ValueError(f"dynamics must be 'factored' or 'direct', not {v!r}")
                c.direct_dynamics = 0 if v == "factored" else 1
                continue
            setattr(c, f.name, v)
        return c


class Engine:
    def __init__(self, config: EngineConfig):
        self.config = config
        self.N = config.board_size
        self.C = config.latent_dim
        self.A = self.N * self.N + 1
        self.G = config.num_games
        self.S = config.num_simulations
        self.M = config.max_moves or self.N * self.N
        self.device = torch.device("cuda", config.device)
        if not torch.cuda.is_available():
            raise RuntimeError("mzgo needs a ROCm GPU (MI355X); no CPU fallback exists")
        torch.cuda.init()
        h = ctypes.c_void_p()
        check(lib.mzgo_engine_create(ctypes.byref(config.to_c()), ctypes.byref(h)))
        self._h = h
        self._weights_key = None

    def close(self):
        if getattr(self, "_h", None):
            lib.mzgo_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def device_bytes(self):
        return int(lib.mzgo_engine_device_bytes(self._h))

    # ---- weights ----
    def set_state_dict(self, state_dict):
        """Load reference state_dict tensors (any device/dtype -> host f32)."""
        for key, t in state_dict.items():
            a = np.ascontiguousarray(torch.as_tensor(t).detach().to("cpu", torch.float32).numpy())
            if key == "dynamics.action_embedding.weight" and a.ndim == 2 and a.shape[0] > self.A:
                a = np.ascontiguousarray(a[:self.A])      # rows past the board's actions (play.py:193)
            shape = (ctypes.c_int64 * a.ndim)(*a.shape)
            check(lib.mzgo_set_weights(self._h, key.encode(), ptr(a), shape, a.ndim))
        if not lib.mzgo_weights_ready(self._h):
            check(_lib.MZGO_ENOWEIGHTS)

    # ---- network protocol ----
    def initial_inference(self, obs):
        B = obs.shape[0]
        obs = obs.to(self.device, torch.float32).contiguous()
        lat = torch.empty(B, self.C, self.N, self.N, device=self.device)
        val = torch.empty(B, 1, device=self.device)
        logits = torch.empty(B, self.A, device=self.device)
        check(lib.mzgo_initial_inference(self._h, ptr(obs), B, ptr(lat), ptr(val), ptr(logits),
                                         stream_of(self.device)))
        return lat, val, logits

    def recurrent_inference(self, latent, action, check_range=False):
        B = latent.shape[0]
        latent = latent.to(self.device, torch.float32).contiguous()
        action = action.to(self.device, torch.int64).reshape(B).contiguous()
        nlat = torch.empty(B, self.C, self.N, self.N, device=self.device)
        rew = torch.empty(B, 1, device=self.device)
        val = torch.empty(B, 1, device=self.device)
        logits = torch.empty(B, self.A, device=self.device)
        check(lib.mzgo_recurrent_inference(self._h, ptr(latent), ptr(action), B, ptr(nlat), ptr(rew),
                                           ptr(val), ptr(logits), stream_of(self.device)))
        if check_range:
            check(lib.mzgo_check_inference_errors(self._h, stream_of(self.device)))
        return nlat, rew, val, logits

    # ---- search ----
    def search(self, root_obs, noise=None, move_index=0):
        """MCTS.run for the first G = root_obs.shape[0] slots.

        Returns (root child visits int32 [G, A], root value float64 [G]) on the GPU.
        """
        G = root_obs.shape[0]
        root_obs = root_obs.to(self.device, torch.float32).contiguous()
        if noise is not None:
            noise = torch.as_tensor(noise, dtype=torch.float64).to(self.device).reshape(G, self.A).contiguous()
        visits = torch.empty(G, self.A, dtype=torch.int32, device=self.device)
        value = torch.empty(G, dtype=torch.float64, device=self.device)
        check(lib.mzgo_search(self._h, ptr(root_obs), ptr(noise), G, move_index, ptr(visits),
                              ptr(value), stream_of(self.device)))
        return visits, value

    def tree(self, g=0):
        """Host copy of slot g's last search tree (dict of numpy arrays)."""
        n1 = self.S + 1
        nn = ctypes.c_int32()
        child = np.empty((n1, self.A), np.int32)
        visits = np.empty(n1, np.int32)
        wsum = np.empty(n1, np.float64)
        prior = np.empty((n1, self.A), np.float32)
        rprior = np.empty(self.A, np.float64)
        check(lib.mzgo_tree_export(self._h, g, ctypes.byref(nn), ptr(child), ptr(visits), ptr(wsum),
                                   ptr(prior), ptr(rprior), stream_of(self.device)))
        n = nn.value
        return dict(n=n, child=child[:n], visits=visits[:n], value_sum=wsum[:n], prior=prior[:n],
                    root_prior=rprior)

    # ---- boards ----
    def board_reset(self):
        check(lib.mzgo_board_reset(self._h, stream_of(self.device)))

    def board_step(self, actions):
        """actions: int sequence/tensor [G] (-1 = skip). Returns (status, winner) on the host."""
        a = torch.as_tensor(actions, dtype=torch.int32).to(self.device).reshape(self.G).contiguous()
        status = torch.empty(self.G, dtype=torch.int32, device=self.device)
        winner = torch.empty(self.G, dtype=torch.float64, device=self.device)
        check(lib.mzgo_board_step(self._h, ptr(a), ptr(status), ptr(winner), stream_of(self.device)))
        return status.cpu().numpy(), winner.cpu().numpy()

    def board_planes(self):
        planes = torch.empty(self.G, 6, self.N, self.N, dtype=torch.float64, device=self.device)
        check(lib.mzgo_board_planes(self._h, ptr(planes), stream_of(self.device)))
        return planes

    def board_set(self, g, state):
        """Load a GymGo float64 [6,N,N] state into slot g."""
        st = np.asarray(state)
        stones = (st[0] > 0).astype(np.int8) + 2 * (st[1] > 0).astype(np.int8)
        stones = np.ascontiguousarray(stones.reshape(-1))
        invd = np.ascontiguousarray((st[3] > 0).astype(np.uint8).reshape(-1))
        meta = np.array([int(st[2].max()), int(st[4].max() == 1), int(st[5].max() == 1), 0], np.int32)
        check(lib.mzgo_board_set(self._h, g, ptr(stones), ptr(invd), ptr(meta), stream_of(self.device)))

    # ---- self-play ----
    def selfplay_reset(self, epoch=0):
        check(lib.mzgo_selfplay_reset(self._h, epoch, stream_of(self.device)))

    def selfplay_move(self, moves=1):
        """``moves`` moves of every unfinished game in one launch (mzgo_selfplay_moves)."""
        check(lib.mzgo_selfplay_moves(self._h, int(moves), stream_of(self.device)))

    def arena_move(self, opponent, moves=1):
        """``moves`` moves of every unfinished arena game in one launch: this
        engine's network plays turn 0, ``opponent``'s turn 1 (mzgo_arena_moves)."""
        check(lib.mzgo_arena_moves(self._h, opponent.handle, int(moves), stream_of(self.device)))

    def inject_noise(self, noise):
        """Test hook: Dirichlet samples float64 [G, max_moves, A] on the GPU (None = sample)."""
        if noise is not None:
            noise = torch.as_tensor(noise, dtype=torch.float64).to(self.device).contiguous()
            assert noise.shape == (self.G, self.M, self.A)
        self._noise = noise      # keep it alive while moves use it
        check(lib.mzgo_selfplay_inject_noise(self._h, ptr(noise)))

    def record_noise(self, buf):
        """Test hook: every self-play root's normalised Dirichlet sample into
        ``buf`` (float64 [G, max_moves, A] on the GPU; None = off)."""
        if buf is not None:
            assert buf.dtype == torch.float64 and buf.is_cuda and buf.is_contiguous()
            assert tuple(buf.shape) == (self.G, self.M, self.A)
        self._noise_out = buf
        check(lib.mzgo_selfplay_record_noise(self._h, ptr(buf)))

    def record_nodes(self, buf):
        """Test hook (tower engines): every node the searches evaluate into
        ``buf`` (float32 [G, S+1, A+2] on the GPU: logits, reward, value;
        node 0 the root's logits and value; None = off)."""
        if buf is not None:
            assert buf.dtype == torch.float32 and buf.is_cuda and buf.is_contiguous()
            assert tuple(buf.shape) == (self.G, self.S + 1, self.A + 2)
        self._nodes_out = buf
        check(lib.mzgo_tower_record_nodes(self._h, ptr(buf)))

    def tower_timing(self, enable):
        """Tower engines: (ms, towers) spent in dynamics towers since the last
        call (synchronises), then timing on/off (mzgo_tower_timing)."""
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(lib.mzgo_tower_timing(self._h, int(enable), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def launch_timing(self, enable):
        """Move-parallel epochs (mzgo_selfplay_launch_times): the (boards, queue)
        launch durations in ms of every multi-move call since the last read
        (synchronises; empty lists when none ran), then timing on/off."""
        cap = 4096
        b = np.zeros(cap, np.float32)
        q = np.zeros(cap, np.float32)
        n = ctypes.c_int()
        check(lib.mzgo_selfplay_launch_times(self._h, ptr(b), ptr(q), cap, ctypes.byref(n)))
        check(lib.mzgo_selfplay_set_timing(self._h, int(enable)))
        k = min(n.value, cap)
        return b[:k].tolist(), q[:k].tolist()

    def counters(self):
        out = np.zeros(9, np.uint64)
        check(lib.mzgo_selfplay_counters(self._h, ptr(out), stream_of(self.device)))
        return dict(simulations=int(out[0]), moves=int(out[1]), games_finished=int(out[2]),
                    playing=int(out[3]), dynamics_convs=int(out[4]), tail_convs=int(out[5]),
                    prior_rows=int(out[6]), workgroups_started=int(out[7]), tail_wait_expiries=int(out[8]))

    def wait_started(self, target, stream=None):
        """Diagnostic (scripts/rccl_standin.py; bench.py does not use it):
        enqueue on ``stream`` (default: the current one) a gate that completes
        once ``counters()['workgroups_started'] >= target``: a collective
        queued behind it cannot displace a self-play workgroup of the launch
        that brings the count there (mzgo_stream_wait_started; reference
        network engines only; a gate that gives up is reported by the next
        counters() call)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        check(lib.mzgo_stream_wait_started(self._h, int(target), ctypes.c_void_p(s.cuda_stream)))

    def record(self, g):
        """Host copy of slot g's game record (numpy arrays)."""
        M, CELLS, A = self.M, self.N * self.N, self.A
        length = ctypes.c_int32()
        status = ctypes.c_int32()
        stones = np.empty((M, CELLS), np.int8)
        invd = np.empty((M, CELLS), np.uint8)
        flags = np.empty(M, np.uint8)
        action = np.empty(M, np.int32)
        value = np.empty(M, np.float64)
        policy = np.empty((M, A), np.float64)
        reward = np.empty(M, np.float64)
        final = np.zeros(1, np.float64)
        check(lib.mzgo_records_export(self._h, g, ctypes.byref(length), ctypes.byref(status), ptr(stones),
                                      ptr(invd), ptr(flags), ptr(action), ptr(value), ptr(policy),
                                      ptr(reward), ptr(final), stream_of(self.device)))
        L = length.value
        return dict(length=L, status=status.value, stones=stones[:L], invd=invd[:L], flags=flags[:L],
                    action=action[:L], value=value[:L], policy=policy[:L], reward=reward[:L],
                    final_reward=float(final[0]))
