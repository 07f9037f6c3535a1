"""mzgo -- MI355X-native MuZero-Go self-play engine (host side).

Drop-in counterparts of the reference's hot path (Sir-Teo/MuZero-Go
self_play.py), all executed by libmzgo.so's HIP kernels:

* ``MuZeroNet``   -- same parameters/state_dict keys; initial/recurrent inference on MFMA
* ``ResMuZeroNet`` -- BASELINE config 5's residual-tower network (bf16 MFMA tower engine)
* ``MCTS``, ``MuZeroAgent`` -- device search (select / expand / backup kernels)
* ``MainMCTS`` -- main.py's MCTS variant (trainer self-play / arena) on the same kernels
* ``GoEnv``       -- GymGo rules as bit-exact integer kernels
* ``SelfPlay``    -- G concurrent games per GPU, one fused kernel step per move
* ``SelfPlayEvaluator`` -- main.py's arena (two networks, all games at once)
* ``GameHistory``, ``save_batches`` -- the reference's record / pickle format
* ``mzgo.play`` -- play.py's interactive human-vs-agent loop (``python -m mzgo.play weights.pth``)
"""
from ._lib import MzgoError
from .arena import SelfPlayEvaluator
from .engine import Engine, EngineConfig
from .env import GoEnv
from .net import MuZeroNet
from .resnet import ResMuZeroNet
from .search import MCTS, MainMCTS, MuZeroAgent
from .selfplay import GameHistory, SelfPlay, history_from_device, save_batches
from .weights import deterministic_res_state_dict, deterministic_state_dict

__all__ = ["Engine", "EngineConfig", "GoEnv", "MuZeroNet", "MCTS", "MainMCTS", "MuZeroAgent", "SelfPlay",
           "GameHistory", "history_from_device", "save_batches", "deterministic_state_dict", "SelfPlayEvaluator",
           "ResMuZeroNet", "deterministic_res_state_dict", "MzgoError"]
