"""``ResMuZeroNet``: the residual-tower MuZero network of BASELINE config 5
(19x19, 20-block residual nets, 1600 simulations per move).

The reference has no such network (its representation is three convs and
its dynamics ONE conv, self_play.py:63-128); config 5 names the regime, and
this module fixes the architecture, keeping the reference's protocol and
heads:

* representation: conv_in 3x3 6->C + ReLU, then ``blocks`` residual blocks
  x = relu(x + conv2(relu(conv1(x))));
* dynamics: latent + embedding[action] broadcast over the board (as
  self_play.py:88-90), conv_in 3x3 C->C + ReLU, ``blocks`` residual blocks;
  the reward head of self_play.py:91-94;
* prediction: the heads of self_play.py:104-113.

The torch sub-modules only hold the parameters (state_dict keys below); the
network runs on the HIP engine (``res_blocks`` > 0: ``k_tconv``, bf16 MFMA
with fp32 accumulation, activations stored in bf16).  ``oracle/resnet.py``
is the torch restatement the parity tests compare with.
"""
import torch
import torch.nn as nn

from .engine import Engine, EngineConfig
from .net import _Prediction, board_size_of


def _conv3(cin, cout):
    return nn.Conv2d(cin, cout, kernel_size=3, padding=1)


class _Block(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv1 = _conv3(c, c)
        self.conv2 = _conv3(c, c)


class _ResRepresentation(nn.Module):
    def __init__(self, c, blocks):
        super().__init__()
        self.conv_in = _conv3(6, c)
        self.blocks = nn.ModuleList([_Block(c) for _ in range(blocks)])


class _ResDynamics(nn.Module):
    def __init__(self, c, max_action_size, blocks):
        super().__init__()
        self.action_embedding = nn.Embedding(max_action_size, c)
        self.conv_in = _conv3(c, c)
        self.blocks = nn.ModuleList([_Block(c) for _ in range(blocks)])
        self.reward_conv = nn.Conv2d(c, 1, kernel_size=1)
        self.fc_reward_hidden = nn.Linear(1, 16)
        self.fc_reward_output = nn.Linear(16, 1)


class ResMuZeroNet(nn.Module):
    """Same protocol as ``mzgo.MuZeroNet`` (initial_inference /
    recurrent_inference / engine); defaults are config 5's C=256, 20 blocks."""

    def __init__(self, latent_dim=256, max_action_size=362, blocks=20):
        super().__init__()
        if latent_dim % 64:
            raise ValueError("the tower engine needs latent_dim a multiple of 64")
        self.latent_dim = latent_dim
        self.max_action_size = max_action_size
        self.board_size = board_size_of(max_action_size)
        self.blocks = blocks
        self.representation = _ResRepresentation(latent_dim, blocks)
        self.dynamics = _ResDynamics(latent_dim, max_action_size, blocks)
        self.prediction = _Prediction(latent_dim)
        self._engines = {}

    def _version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def engine(self, num_games=1, num_simulations=1, **cfg):
        """A HIP tower engine with this net's current weights (cached per shape/config)."""
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("ResMuZeroNet runs on the GPU only: call .to('cuda') first")
        key = (num_games, num_simulations, tuple(sorted(cfg.items())), dev.index or 0)
        eng = self._engines.get(key)
        if eng is None:
            conf = EngineConfig(board_size=self.board_size, latent_dim=self.latent_dim, num_games=num_games,
                                num_simulations=num_simulations, device=dev.index or 0, tower=1,
                                res_blocks=self.blocks,
                                **cfg)
            eng = Engine(conf)
            self._engines[key] = eng
        v = self._version()
        if eng._weights_key != v:
            eng.set_state_dict(self.state_dict())
            eng._weights_key = v
        return eng

    def _apply(self, fn, *args, **kwargs):
        self._engines = {}
        return super()._apply(fn, *args, **kwargs)

    @torch.no_grad()
    def initial_inference(self, observation):
        return self.engine().initial_inference(observation)

    @torch.no_grad()
    def recurrent_inference(self, latent, action):
        return self.engine().recurrent_inference(latent, action)

    def forward(self, observation):
        return self.initial_inference(observation)
