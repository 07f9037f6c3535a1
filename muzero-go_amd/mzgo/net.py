"""``MuZeroNet`` drop-in: the reference module's parameters and state_dict keys,
with ``initial_inference`` / ``recurrent_inference`` executed by the HIP
engine (fused MFMA conv + heads kernels).

Reference: self_play.py:63-128 (RepresentationNetwork, DynamicsNetwork,
PredictionNetwork, MuZeroNet).  The torch sub-modules below only *hold* the
parameters so that ``state_dict`` / ``load_state_dict`` / ``.to()`` /
``.parameters()`` behave like the reference's; no torch op computes the
network.  Outputs are inference-only (no autograd graph); ``mzgo.trainer``
(main.py's training step) differentiates through these
same parameters.
"""
import torch
import torch.nn as nn

from .engine import Engine, EngineConfig


class _Representation(nn.Module):
    def __init__(self, latent_dim):
        super().__init__()
        self.conv1 = nn.Conv2d(6, 64, kernel_size=3, padding=1)
        self.conv2 = nn.Conv2d(64, 64, kernel_size=3, padding=1)
        self.conv3 = nn.Conv2d(64, latent_dim, kernel_size=3, padding=1)


class _Dynamics(nn.Module):
    def __init__(self, latent_dim, max_action_size):
        super().__init__()
        self.action_embedding = nn.Embedding(max_action_size, latent_dim)
        self.conv = nn.Conv2d(latent_dim, latent_dim, kernel_size=3, padding=1)
        self.reward_conv = nn.Conv2d(latent_dim, 1, kernel_size=1)
        self.fc_reward_hidden = nn.Linear(1, 16)
        self.fc_reward_output = nn.Linear(16, 1)


class _Prediction(nn.Module):
    def __init__(self, latent_dim):
        super().__init__()
        self.value_conv = nn.Conv2d(latent_dim, 1, kernel_size=1)
        self.value_fc = nn.Linear(1, 1)
        self.policy_conv = nn.Conv2d(latent_dim, 1, kernel_size=1)
        self.pass_logit = nn.Parameter(torch.zeros(1))


def board_size_of(action_size):
    n = int(round((action_size - 1) ** 0.5))
    if n * n + 1 != action_size:
        raise ValueError(f"max_action_size {action_size} is not N*N+1 (self_play.py:22 quirk); "
                         "the engine needs the board's exact action count")
    return n


class MuZeroNet(nn.Module):
    """``board_size``: for networks whose embedding table is larger than the
    board's N*N+1 actions (play.py:193 sizes it int(1.5 N^2)); the extra rows
    are kept in the state_dict and never reach the engine (actions >= N*N+1
    do not exist on the board)."""

    def __init__(self, latent_dim, max_action_size, board_size=None):
        super().__init__()
        self.latent_dim = latent_dim
        self.max_action_size = max_action_size
        if board_size is None:
            self.board_size = board_size_of(max_action_size)
        else:
            if max_action_size < board_size * board_size + 1:
                raise ValueError(f"max_action_size {max_action_size} < {board_size}*{board_size}+1 actions")
            self.board_size = board_size
        self.representation = _Representation(latent_dim)
        self.dynamics = _Dynamics(latent_dim, max_action_size)
        self.prediction = _Prediction(latent_dim)
        self._engines = {}

    # -- engine plumbing --
    def _version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def engine(self, num_games=1, num_simulations=1, **cfg):
        """A HIP engine with this net's current weights (cached per shape/config)."""
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("MuZeroNet runs on the GPU only: call .to('cuda') first")
        key = (num_games, num_simulations, tuple(sorted(cfg.items())), dev.index or 0)
        eng = self._engines.get(key)
        if eng is None:
            conf = EngineConfig(board_size=self.board_size, latent_dim=self.latent_dim,
                                num_games=num_games, num_simulations=num_simulations,
                                device=dev.index or 0, **cfg)
            eng = Engine(conf)
            eng._weights_key = None
            self._engines[key] = eng
        v = self._version()
        if eng._weights_key != v:
            eng.set_state_dict(self.state_dict())
            eng._weights_key = v
        return eng

    def _apply(self, fn, *args, **kwargs):
        self._engines = {}
        return super()._apply(fn, *args, **kwargs)

    # -- the reference protocol (self_play.py:121-128) --
    @torch.no_grad()
    def initial_inference(self, observation):
        return self.engine().initial_inference(observation)

    @torch.no_grad()
    def recurrent_inference(self, latent, action):
        return self.engine().recurrent_inference(latent, action)

    def forward(self, observation):
        return self.initial_inference(observation)
