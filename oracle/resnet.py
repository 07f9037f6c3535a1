"""The residual-tower network of BASELINE config 5, restated functionally in
torch (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Config 5 (19x19, 20-block residual nets, 1600 simulations) has no reference
counterpart: the architecture is the build's own
``mzgo.resnet.ResMuZeroNet`` and this module is its parity reference:

* representation: relu(conv_in(obs)), then per block
  x = relu(x + conv2(relu(conv1(x)))) (3x3, padding 1);
* dynamics: x = latent + embedding[action] broadcast (self_play.py:88-90),
  relu(conv_in(x)), the same blocks; the reward head of self_play.py:91-94;
* prediction: the heads of self_play.py:104-113 (oracle/net.py).

``bf16=False``: the network in fp32 (the architecture's definition).
``bf16=True``: the engine's rounding points, computed in float64 -- conv
weights rounded to bf16, every stored activation (each conv's output after
bias / residual / ReLU, and a latent entering the dynamics) rounded to bf16,
the dynamics' embedding added through the conv of the embedding plane (the
engine's region table, mzgo_expand.hpp), the heads in high precision on the
rounded latent.  What remains between it and the engine is the engine's fp32
accumulation order (rarely a different bf16 rounding of one element).
Duck-type compatible with oracle.mcts.MCTS (initial_inference /
recurrent_inference).
"""
import torch
import torch.nn.functional as F


class OracleResNet:
    def __init__(self, state_dict, blocks, bf16=False):
        self.blocks = blocks
        self.bf16 = bf16
        self.dt = torch.float64 if bf16 else torch.float32
        p = {}
        for k, v in state_dict.items():
            t = torch.as_tensor(v).detach().to(torch.float32)
            if bf16 and k.endswith(".weight") and t.dim() == 4 and t.shape[-1] == 3:
                t = t.to(torch.bfloat16).to(torch.float32)          # the MFMA operands
            p[k] = t.to(self.dt)
        self.p = p
        self.latent_dim = p["dynamics.conv_in.weight"].shape[0]
        self.action_size = p["dynamics.action_embedding.weight"].shape[0]

    def eval(self):
        return self

    def _store(self, x):
        return x.to(torch.bfloat16).to(self.dt) if self.bf16 else x

    def _conv(self, x, key):
        return F.conv2d(x, self.p[key + ".weight"], self.p[key + ".bias"], padding=1)

    def _tower(self, x, net):
        for i in range(self.blocks):
            h = self._store(F.relu(self._conv(x, f"{net}.blocks.{i}.conv1")))
            x = self._store(F.relu(self._conv(h, f"{net}.blocks.{i}.conv2") + x))
        return x

    def representation(self, obs):
        x = self._store(F.relu(self._conv(obs.to(self.dt), "representation.conv_in")))
        return self._tower(x, "representation")

    def dynamics(self, latent, action):
        p = self.p
        emb = p["dynamics.action_embedding.weight"][action.long()]
        x = self._store(latent.to(self.dt))
        B, C, N, _ = x.shape
        if self.bf16:
            # conv(x + emb) = conv(x) + conv(emb plane) under zero padding (the engine's E table)
            plane = emb[:, :, None, None].expand(B, C, N, N)
            y = self._conv(x, "dynamics.conv_in") + F.conv2d(plane, p["dynamics.conv_in.weight"], padding=1)
        else:
            y = self._conv(x + emb[:, :, None, None], "dynamics.conv_in")
        x = self._tower(self._store(F.relu(y)), "dynamics")
        r = F.conv2d(x, p["dynamics.reward_conv.weight"], p["dynamics.reward_conv.bias"]).mean(dim=[2, 3])
        r = F.relu(F.linear(r, p["dynamics.fc_reward_hidden.weight"], p["dynamics.fc_reward_hidden.bias"]))
        r = F.linear(r, p["dynamics.fc_reward_output.weight"], p["dynamics.fc_reward_output.bias"])
        return x, r

    def prediction(self, x):
        p = self.p
        v = F.conv2d(x, p["prediction.value_conv.weight"], p["prediction.value_conv.bias"]).mean(dim=[2, 3])
        v = F.linear(v, p["prediction.value_fc.weight"], p["prediction.value_fc.bias"])
        logits = F.conv2d(x, p["prediction.policy_conv.weight"], p["prediction.policy_conv.bias"])
        logits = logits.reshape(x.shape[0], -1)
        pass_col = p["prediction.pass_logit"].reshape(1, 1).expand(x.shape[0], 1)
        return v, torch.cat([logits, pass_col], dim=1)

    # the protocol (outputs f32 like the engine's; bf16 latents are exact in f32)
    def initial_inference(self, obs):
        latent = self.representation(obs)
        v, logits = self.prediction(latent)
        return latent.float(), v.float(), logits.float()

    def recurrent_inference(self, latent, action):
        nxt, r = self.dynamics(latent, action)
        v, logits = self.prediction(nxt)
        return nxt.float(), r.float(), v.float(), logits.float()
