"""Trainer ingestion: main.py's MuZero training step
over trajectories produced by the device self-play.

The reference trains in main.py (``MuZeroAgent.train``, main.py:381-501;
``compute_target_value``, :503-522) on trajectory dicts built by its own
self-play loop (main.py:636-713): ``observations`` T+2 (the initial
observation, one per move, the terminal one again), ``actions`` T,
``policies`` T (child-visit distributions) and ``rewards`` T+1 (the env
rewards, -0.5 added to the last one when the game hit the move cap, then the
winner).  This module produces exactly that format from the engine's records
(``trajectory_from_record``, ``MainSelfPlay`` -- main.py's MCTS and move rule
on the device, every game of a batch at once) and trains on it:

* ``mode="reference"`` -- main.py's step, quirks included: ``zero_grad`` once
  per batch but ``backward`` + ``clip_grad_norm_`` + ``optimizer.step`` per
  trajectory, so gradients accumulate across the batch;
  bootstrap values with the weights of that moment; every priority set to the
  batch's mean loss; ``StepLR`` stepped once per batch.  Pinned by a step
  recorded from the reference (``tests/golden/train_*``).
* ``mode="batched"`` -- the same losses for all B trajectories in one unroll
  (B x 10 recurrent steps, each one launch for all B) and ONE optimizer step
  on their summed gradient; the bootstrap values of every (trajectory, unroll
  step) pair come from one batched ``initial_inference`` on the HIP engine.
  With ``hip_forward=True`` the unroll's forward runs on the HIP kernels
  (``initial_inference_hip`` / ``recurrent_inference_hip``: the engine's
  k_initial_inference / k_recurrent_inference for the 3x3 convs, autograd
  Functions whose backward is the HIP kernels of csrc/mzgo_train.hip for every
  3x3 conv -- the dynamics conv from its saved input and output, the
  representation's three after recomputing its two hidden activations on the
  same kernels); the 1x1 heads stay torch ops on the engine's latents.  The
  default is torch's ops (MIOpen), measured 8 % faster at main.py's sizes.

``initial_inference_torch`` / ``recurrent_inference_torch`` restate
main.py:72-144 with torch ops on the module's own parameters (reference
mode, and the CPU).  Replay buffers restate main.py:158-244.
"""
import ctypes
import random
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from .net import MuZeroNet
from .selfplay import SelfPlay


# ---------------------------------------------------------------------------
# configuration (main.py:27-53, the trainer's part)
# ---------------------------------------------------------------------------
@dataclass
class TrainConfig:
    learning_rate: float = 1e-4
    unroll_steps: int = 10
    discount: float = 0.99
    value_loss_weight: float = 1.0
    policy_loss_weight: float = 1.0
    reward_loss_weight: float = 1.0
    use_value_transform: bool = True
    lr_step_size: int = 1000          # StepLR(step_size=1000, gamma=0.9), main.py:379
    lr_gamma: float = 0.9
    max_grad_norm: float = 1.0        # main.py:481


def reward_value_transform(x, epsilon=0.001):
    """h(x) = sign(x) (sqrt(|x| + 1) - 1) + eps x (main.py:66-69)."""
    return torch.sign(x) * (torch.sqrt(torch.abs(x) + 1) - 1) + epsilon * x


# ---------------------------------------------------------------------------
# differentiable forward (main.py:72-144), on the MuZeroNet's parameters
# ---------------------------------------------------------------------------
def _prediction(net, latent):
    p = net.prediction
    value = p.value_fc(p.value_conv(latent).mean(dim=[2, 3]))
    policy_map = p.policy_conv(latent)
    b = policy_map.size(0)
    logits = torch.cat([policy_map.view(b, -1), p.pass_logit.expand(b, 1)], dim=1)
    return value, logits


def initial_inference_torch(net, observation):
    r = net.representation
    x = F.relu(r.conv1(observation))
    x = F.relu(r.conv2(x))
    latent = F.relu(r.conv3(x))
    value, logits = _prediction(net, latent)
    return latent, value, logits


def recurrent_inference_torch(net, latent, action):
    d = net.dynamics
    b = latent.shape[0]
    emb = d.action_embedding(action).view(b, latent.shape[1], 1, 1).expand_as(latent)
    x = F.relu(d.conv(latent + emb))
    reward = d.fc_reward_output(F.relu(d.fc_reward_hidden(d.reward_conv(x).mean(dim=[2, 3]))))
    value, logits = _prediction(net, x)
    return x, reward, value, logits


# ---------------------------------------------------------------------------
# the same networks with the forward on the HIP engine (SURVEY.md §8(f) 1:
# "forward only through HIP, backward via torch")
# ---------------------------------------------------------------------------
def conv3x3_forward_hip(x, weight, bias):
    """relu(conv3x3(x) + bias), padding 1, on the HIP fp32-MFMA kernel
    (mzgo_conv3x3_relu_forward): the representation's hidden activations
    recomputed for its backward (main.py:72-84)."""
    from ._lib import check, lib, ptr, stream_of
    B, Cin, N, _ = x.shape
    Cout = weight.shape[0]
    dev = x.device
    f = [t.detach().to(dev, torch.float32).contiguous() for t in (x, weight, bias)]
    y = torch.empty(B, Cout, N, N, device=dev)
    check(lib.mzgo_conv3x3_relu_forward(ptr(f[0]), None, None, ptr(f[1]), ptr(f[2]), B, Cin, Cout, N, ptr(y),
                                        stream_of(dev)))
    return y


def conv3x3_backward_hip(g, out, x, weight, action=None, emb=None, need_input_grad=True):
    """Backward of out = relu(conv3x3(x') + b), x' = x (+ emb[action] broadcast),
    on the HIP kernels (mzgo_conv3x3_backward: fp32 MFMA implicit GEMMs,
    deterministic; replaces torch.nn.grad.conv2d_input / conv2d_weight): with
    gp = g * [out > 0], returns (d x or None, d weight, d bias)."""
    from ._lib import check, lib, ptr, stream_of
    B, Cin, N, _ = x.shape
    Cout = weight.shape[0]
    dev = x.device
    f = [t.detach().to(dev, torch.float32).contiguous() for t in (g, out, x, weight)]
    e = emb.detach().to(dev, torch.float32).contiguous() if emb is not None else None
    act = action.to(dev, torch.int64).contiguous() if action is not None else None
    ws = ctypes.c_int64()
    check(lib.mzgo_conv3x3_backward_workspace(B, Cin, Cout, ctypes.byref(ws)))
    work = torch.empty(ws.value, dtype=torch.uint8, device=dev)
    gx = torch.empty_like(f[2]) if need_input_grad else None
    gw = torch.empty_like(f[3])
    gb = torch.empty(Cout, device=dev)
    check(lib.mzgo_conv3x3_backward(ptr(f[0]), ptr(f[1]), ptr(f[2]), ptr(act), ptr(e), ptr(f[3]), B, Cin, Cout, N,
                                    ptr(gx), ptr(gw), ptr(gb), ptr(work), ws.value, stream_of(dev)))
    return gx, gw, gb


def dyn_conv_backward_hip(g, nxt, latent, action, emb, weight):
    """The dynamics conv's backward on the HIP kernels (mzgo_dyn_conv_backward,
    csrc/mzgo_train.hip): with gp = g * [nxt > 0], returns (d latent, d weight,
    d bias) of nxt = relu(conv3x3(latent + emb[action]) + bias), main.py:97-103."""
    from ._lib import check, lib, ptr, stream_of
    B, C, N, _ = latent.shape
    dev = latent.device
    f = [t.detach().to(dev, torch.float32).contiguous() for t in (g, nxt, latent, emb, weight)]
    act = action.to(dev, torch.int64).contiguous()
    ws = ctypes.c_int64()
    check(lib.mzgo_dyn_conv_backward_workspace(B, C, ctypes.byref(ws)))
    work = torch.empty(ws.value, dtype=torch.uint8, device=dev)
    gx = torch.empty_like(f[2])
    gw = torch.empty_like(f[4])
    gb = torch.empty(C, device=dev)
    check(lib.mzgo_dyn_conv_backward(ptr(f[0]), ptr(f[1]), ptr(f[2]), ptr(act), ptr(f[3]), ptr(f[4]), B, C, N,
                                     ptr(gx), ptr(gw), ptr(gb), ptr(work), ws.value, stream_of(dev)))
    return gx, gw, gb


class _HipDynamicsConv(torch.autograd.Function):
    """x' = relu(conv3x3(latent + emb[a]) + b) (main.py:97-103) with the
    forward on the engine's k_recurrent_inference and the backward on the
    HIP backward kernels from the saved input and output (ReLU mask = x' > 0;
    dyn_conv_backward_hip); the embedding's gradient = the input gradient
    summed over the board, added into row a."""

    @staticmethod
    def forward(ctx, latent, action, weight, bias, emb, net):
        nxt, _, _, _ = net.engine().recurrent_inference(latent.detach(), action)
        ctx.save_for_backward(latent, action, weight, emb, nxt)
        return nxt

    @staticmethod
    def backward(ctx, g):
        latent, action, weight, emb, nxt = ctx.saved_tensors
        gx, gw, gb = dyn_conv_backward_hip(g, nxt, latent, action, emb, weight)
        gemb = torch.zeros_like(emb).index_add_(0, action, gx.sum(dim=(2, 3)))
        return gx, None, gw, gb, gemb, None


class _HipRepresentation(torch.autograd.Function):
    """The representation (main.py:72-84) with the forward on the engine's
    k_initial_inference and the backward on the HIP kernels: the two hidden
    activations recomputed (mzgo_conv3x3_relu_forward; the engine keeps them
    on chip), then each conv's input / weight / bias gradients from the saved
    input and output (mzgo_conv3x3_backward), conv3 -> conv2 -> conv1."""

    @staticmethod
    def forward(ctx, obs, w1, b1, w2, b2, w3, b3, net):
        lat, _, _ = net.engine().initial_inference(obs.detach())
        ctx.save_for_backward(obs, w1, b1, w2, b2, w3, b3, lat)
        return lat

    @staticmethod
    def backward(ctx, g):
        obs, w1, b1, w2, b2, w3, b3, lat = ctx.saved_tensors
        x1 = conv3x3_forward_hip(obs, w1, b1)
        x2 = conv3x3_forward_hip(x1, w2, b2)
        g2, gw3, gb3 = conv3x3_backward_hip(g, lat, x2, w3)
        g1, gw2, gb2 = conv3x3_backward_hip(g2, x2, x1, w2)
        _, gw1, gb1 = conv3x3_backward_hip(g1, x1, obs, w1, need_input_grad=False)
        return None, gw1, gb1, gw2, gb2, gw3, gb3, None


def initial_inference_hip(net, observation):
    r = net.representation
    latent = _HipRepresentation.apply(observation.contiguous(), r.conv1.weight, r.conv1.bias, r.conv2.weight,
                                      r.conv2.bias, r.conv3.weight, r.conv3.bias, net)
    value, logits = _prediction(net, latent)
    return latent, value, logits


def recurrent_inference_hip(net, latent, action):
    d = net.dynamics
    x = _HipDynamicsConv.apply(latent.contiguous(), action.contiguous(), d.conv.weight, d.conv.bias,
                               d.action_embedding.weight, net)
    reward = d.fc_reward_output(F.relu(d.fc_reward_hidden(d.reward_conv(x).mean(dim=[2, 3]))))
    value, logits = _prediction(net, x)
    return x, reward, value, logits


# ---------------------------------------------------------------------------
# replay buffers (main.py:158-244)
# ---------------------------------------------------------------------------
class PrioritizedReplayBuffer:
    def __init__(self, capacity):
        self.capacity = capacity
        self.buffer = []
        self.priorities = []

    def add(self, trajectory):
        if len(self.buffer) >= self.capacity:
            self.buffer.pop(0)
            self.priorities.pop(0)
        self.buffer.append(trajectory)
        self.priorities.append(1.0)

    def sample(self, batch_size):
        priorities = np.array(self.priorities)
        probs = priorities / priorities.sum()
        indices = np.random.choice(len(self.buffer), batch_size, replace=False, p=probs)
        return [self.buffer[i] for i in indices], indices

    def update_priorities(self, indices, new_priorities):
        for i, p in zip(indices, new_priorities):
            self.priorities[i] = p


class MultiVersionReplayBuffer:
    """Buffers of the last ``num_versions`` model versions, sampled jointly."""

    def __init__(self, capacity, num_versions=1, prioritized=True):
        from collections import deque
        self.capacity = capacity
        self.prioritized = prioritized
        self.buffers = deque(maxlen=num_versions)
        self.add_version()

    def add_version(self):
        from collections import deque
        self.buffers.append(PrioritizedReplayBuffer(self.capacity) if self.prioritized
                            else deque(maxlen=self.capacity))

    def add(self, trajectory):
        if self.prioritized:
            self.buffers[-1].add(trajectory)
        else:
            self.buffers[-1].append(trajectory)

    def sample(self, batch_size):
        if not self.prioritized:
            combined = [t for buf in self.buffers for t in buf]
            if len(combined) < batch_size:
                return [], []
            return random.sample(combined, batch_size), None
        combined, combined_p, owner = [], [], []
        for b, buf in enumerate(self.buffers):
            combined.extend(buf.buffer)
            combined_p.extend(buf.priorities)
            owner.extend((b, i) for i in range(len(buf.buffer)))
        if len(combined) < batch_size:
            return [], []
        probs = np.array(combined_p) / sum(combined_p)
        indices = np.random.choice(len(combined), batch_size, replace=False, p=probs)
        return [combined[i] for i in indices], [owner[i] for i in indices]

    def update_priorities(self, mapping, new_priorities):
        if not self.prioritized or mapping is None:
            return
        for (b, i), p in zip(mapping, new_priorities):
            if b < len(self.buffers):
                self.buffers[b].priorities[i] = p


# ---------------------------------------------------------------------------
# trajectories in main.py's format
# ---------------------------------------------------------------------------
def _planes(stones, invd, flags, N):
    o = np.zeros((6, N, N))
    s = np.asarray(stones).reshape(N, N)
    o[0] = s == 1
    o[1] = s == 2
    o[2] = flags & 1
    o[3] = np.asarray(invd).reshape(N, N)
    o[4] = (flags >> 1) & 1
    o[5] = (flags >> 2) & 1
    return o


def trajectory_from_record(rec, final_obs, board_size, max_moves):
    """main.py:636-713's trajectory from an engine record (``Engine.record``)
    and the board after the game's last move (``final_obs``, f64 [6,N,N]):
    observations T+2, actions T, policies T, rewards T+1."""
    N = board_size
    L = int(rec["length"])
    acts = [int(a) for a in rec["action"][:L]]
    obs = [_planes(rec["stones"][t], rec["invd"][t], int(rec["flags"][t]), N) for t in range(L)]
    final_obs = np.asarray(final_obs, dtype=np.float64)
    done = bool(final_obs[5].max() > 0)
    rewards = [float(r) for r in rec["reward"][:L]]
    if not done and L >= max_moves and rewards:
        rewards[-1] += -0.5                      # main.py:699-702 (move cap)
    winner = float(rec["final_reward"]) if done else 0.0   # env.winner(): 0 unless ended
    return {
        "observations": obs + [final_obs, final_obs],
        "actions": acts,
        "rewards": rewards + [winner],
        "policies": [np.array(p, dtype=np.float64) for p in rec["policy"][:L]],
    }


class MainSelfPlay:
    """main.py's self-play loop (main.py:636-713) for G games at once: its MCTS
    (``search_variant="main"``: c_puct 2, Dirichlet(0.03) at 0.25, pass prior
    0.05), its move rule (argmax of child visits, main.py:660-673) and its
    move cap int(1.5 N^2) (main.py:51).  ``play()`` returns main.py
    trajectories."""

    def __init__(self, net, num_games, num_simulations, *, seed=1234, game_base=0, dynamics="factored"):
        N = net.board_size
        self.max_moves = int(N * N * 1.5)
        self.N = N
        self.sp = SelfPlay(net, num_games, num_simulations, seed=seed, compat="fixed", max_moves=self.max_moves,
                           game_base=game_base, c_puct=2.0, dirichlet_alpha=0.03, dirichlet_epsilon=0.25,
                           pass_epsilon=0.05, search_variant="main", dynamics=dynamics)

    def play(self):
        sp = self.sp
        sp.reset()
        for _ in range(self.max_moves):
            sp.move()
        eng = sp.engine
        if eng.counters()["playing"] != 0:
            raise RuntimeError("games still playing after max_moves moves")
        finals = eng.board_planes().cpu().numpy()
        out = [trajectory_from_record(eng.record(g), finals[g], self.N, self.max_moves) for g in range(sp.G)]
        sp.epoch += 1
        return out


# ---------------------------------------------------------------------------
# the training step (main.py:381-522)
# ---------------------------------------------------------------------------
class MuZeroTrainer:
    """main.py's ``MuZeroAgent`` training half: Adam + StepLR on ``net``'s
    parameters, ``train(replay_buffer, batch_size)`` as main.py:381-501.

    ``start_index(trajectory_length)`` draws a trajectory's start (main.py:395
    ``random.randint(0, T - 1)``; tests pass a fixed sequence)."""

    def __init__(self, net: MuZeroNet, config: TrainConfig = None, mode="reference", start_index=None,
                 hip_forward=None):
        if mode not in ("reference", "batched"):
            raise ValueError(f"mode must be 'reference' or 'batched', not {mode!r}")
        self.net = net
        # batched mode: the unroll's forward and 3x3-conv backward on the HIP
        # kernels (hip_forward=True) or on torch's ops (MIOpen convs, the
        # default): measured at main.py's 6x6 / C=128 / batch 128 x unroll 10,
        # the network part takes 10.49 ms on the HIP kernels and 9.71 ms on
        # MIOpen, the whole step 22.1 vs 21.0 ms (scripts/trainer_timing.py,
        # profiles/r5_trainer_step.json), so the faster one is the default
        self.hip_forward = False if hip_forward is None else hip_forward
        self.config = config or TrainConfig()
        self.mode = mode
        self.action_size = net.board_size ** 2 + 1
        self.optimizer = torch.optim.Adam(net.parameters(), lr=self.config.learning_rate)
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=self.config.lr_step_size,
                                                         gamma=self.config.lr_gamma)
        self.start_index = start_index or (lambda T: random.randint(0, T - 1))
        self.last = {}

    @property
    def device(self):
        return next(self.net.parameters()).device

    # -- targets ------------------------------------------------------------
    def _discounted(self, trajectory, index):
        """The reward part of compute_target_value (main.py:503-515) and the
        bootstrap position (or None)."""
        c = self.config
        target, factor = 0.0, 1.0
        rewards = trajectory["rewards"]
        T = len(rewards)
        for k in range(c.unroll_steps):
            j = index + k
            if j >= T:
                break
            target += factor * rewards[j]
            factor *= c.discount
        boot = index + c.unroll_steps if index + c.unroll_steps < T else None
        return target, factor, boot

    def compute_target_value(self, trajectory, index, unroll_steps=None):
        """main.py:503-522 (bootstrap value from the current weights)."""
        target, factor, boot = self._discounted(trajectory, index)
        if boot is not None:
            obs = torch.as_tensor(np.asarray(trajectory["observations"][boot]), dtype=torch.float32,
                                  device=self.device).unsqueeze(0)
            with torch.no_grad():
                _, value, _ = initial_inference_torch(self.net, obs)
            target += factor * value.item()
        return target

    def _policy_target(self, trajectory, i):
        pol = trajectory["policies"]
        return pol[i] if i < len(pol) else np.ones(self.action_size) / self.action_size

    def _value_loss(self, value, target):
        if self.config.use_value_transform:
            return F.mse_loss(reward_value_transform(value), reward_value_transform(target), reduction="none")
        return F.mse_loss(value, target, reduction="none")

    # -- main.py's step -------------------------------------------------------
    def train(self, replay_buffer, batch_size):
        batch, indices = replay_buffer.sample(batch_size)
        if not batch or len(batch) < batch_size:
            return None
        avg = self._train_reference(batch) if self.mode == "reference" else self._train_batched(batch)
        if indices is not None:
            replay_buffer.update_priorities(indices, [avg] * len(indices))
        self.scheduler.step()
        return avg

    def _train_reference(self, batch):
        c, dev, net = self.config, self.device, self.net
        A = self.action_size
        loss_total = tot_v = tot_p = tot_r = 0.0
        self.optimizer.zero_grad()                       # once per batch (main.py:391)
        for trajectory in batch:
            T = len(trajectory["actions"])
            start = self.start_index(T)
            obs = torch.as_tensor(np.asarray(trajectory["observations"][start]), dtype=torch.float32,
                                  device=dev).unsqueeze(0)
            latent, value, logits = initial_inference_torch(net, obs)
            tv = torch.tensor(self.compute_target_value(trajectory, start), dtype=torch.float32, device=dev)
            tp = torch.tensor(self._policy_target(trajectory, start), dtype=torch.float32, device=dev)
            v_loss = self._value_loss(value.squeeze(), tv)
            p_loss = F.kl_div(F.log_softmax(logits, dim=1), tp, reduction="batchmean")
            step_loss = c.value_loss_weight * v_loss + c.policy_loss_weight * p_loss
            tot_v += c.value_loss_weight * v_loss.item()
            tot_p += c.policy_loss_weight * p_loss.item()
            for k in range(1, c.unroll_steps + 1):
                j = start + k - 1
                a = trajectory["actions"][j] if j < T else A - 1          # pass past the end
                latent, reward, value, logits = recurrent_inference_torch(
                    net, latent, torch.tensor([a], dtype=torch.long, device=dev))
                tr = trajectory["rewards"][j] if j < len(trajectory["rewards"]) else 0.0
                tr = torch.tensor(tr, dtype=torch.float32, device=dev)
                tv = torch.tensor(self.compute_target_value(trajectory, start + k), dtype=torch.float32, device=dev)
                tp = torch.tensor(self._policy_target(trajectory, start + k), dtype=torch.float32, device=dev)
                r_loss = F.mse_loss(reward.squeeze(), tr)
                v_loss = self._value_loss(value.squeeze(), tv)
                p_loss = F.kl_div(F.log_softmax(logits, dim=1), tp, reduction="batchmean")
                step_loss = step_loss + (c.reward_loss_weight * r_loss + c.value_loss_weight * v_loss
                                         + c.policy_loss_weight * p_loss)
                tot_r += c.reward_loss_weight * r_loss.item()
                tot_v += c.value_loss_weight * v_loss.item()
                tot_p += c.policy_loss_weight * p_loss.item()
            step_loss.backward()
            torch.nn.utils.clip_grad_norm_(net.parameters(), max_norm=c.max_grad_norm)
            self.optimizer.step()
            loss_total += step_loss.item()
        n = len(batch)
        self.last = dict(training_loss=loss_total / n, value_loss=tot_v / n, policy_loss=tot_p / n,
                         reward_loss=tot_r / n, lr=self.optimizer.param_groups[0]["lr"])
        return loss_total / n

    def _train_batched(self, batch):
        c, dev, net = self.config, self.device, self.net
        A, K, B = self.action_size, c.unroll_steps, len(batch)
        starts = [self.start_index(len(t["actions"])) for t in batch]
        # targets: rewards, policies and the discounted part of every value
        # target; all bootstrap positions in one inference
        t_val = np.zeros((B, K + 1))
        t_rew = np.zeros((B, K))
        t_pol = np.zeros((B, K + 1, A))
        acts = np.full((B, K), A - 1, dtype=np.int64)
        boot_obs, boot_at = [], []
        for b, (tr, s) in enumerate(zip(batch, starts)):
            T = len(tr["actions"])
            for k in range(K + 1):
                val, factor, boot = self._discounted(tr, s + k)
                t_val[b, k] = val
                if boot is not None:
                    boot_obs.append(np.asarray(tr["observations"][boot]))
                    boot_at.append((b, k, factor))
                t_pol[b, k] = self._policy_target(tr, s + k)
            for k in range(K):
                j = s + k
                if j < T:
                    acts[b, k] = tr["actions"][j]
                t_rew[b, k] = tr["rewards"][j] if j < len(tr["rewards"]) else 0.0
        if boot_obs:
            obs = torch.as_tensor(np.stack(boot_obs), dtype=torch.float32, device=dev)
            with torch.no_grad():
                if dev.type == "cuda":
                    _, v, _ = net.initial_inference(obs)      # HIP engine, one launch
                else:
                    _, v, _ = initial_inference_torch(net, obs)
            v = v.squeeze(1).double().cpu().numpy()
            for (b, k, factor), vb in zip(boot_at, v):
                t_val[b, k] += factor * float(np.float32(vb))
        f32 = lambda x: torch.as_tensor(x, dtype=torch.float32, device=dev)
        t_val, t_rew, t_pol = f32(t_val), f32(t_rew), f32(t_pol)
        obs0 = f32(np.stack([np.asarray(tr["observations"][s]) for tr, s in zip(batch, starts)]))
        self.optimizer.zero_grad()
        fwd0, fwd = ((initial_inference_hip, recurrent_inference_hip) if self.hip_forward
                     else (initial_inference_torch, recurrent_inference_torch))
        latent, value, logits = fwd0(net, obs0)
        kl = lambda lg, tp: F.kl_div(F.log_softmax(lg, dim=1), tp, reduction="none").sum(dim=1)
        v_l = c.value_loss_weight * self._value_loss(value.squeeze(1), t_val[:, 0])
        p_l = c.policy_loss_weight * kl(logits, t_pol[:, 0])
        per = v_l + p_l
        tot_v, tot_p, tot_r = v_l.sum().item(), p_l.sum().item(), 0.0
        acts_t = torch.as_tensor(acts, device=dev)
        for k in range(1, K + 1):
            latent, reward, value, logits = fwd(net, latent, acts_t[:, k - 1])
            r_l = c.reward_loss_weight * F.mse_loss(reward.squeeze(1), t_rew[:, k - 1], reduction="none")
            v_l = c.value_loss_weight * self._value_loss(value.squeeze(1), t_val[:, k])
            p_l = c.policy_loss_weight * kl(logits, t_pol[:, k])
            per = per + r_l + v_l + p_l
            tot_r += r_l.sum().item()
            tot_v += v_l.sum().item()
            tot_p += p_l.sum().item()
        loss = per.sum()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), max_norm=c.max_grad_norm)
        self.optimizer.step()
        self.last = dict(training_loss=loss.item() / B, value_loss=tot_v / B, policy_loss=tot_p / B,
                         reward_loss=tot_r / B, lr=self.optimizer.param_groups[0]["lr"])
        return loss.item() / B
