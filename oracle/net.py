"""MuZeroNet restated functionally in torch fp32 (TEST INFRASTRUCTURE ONLY).

Restates self_play.py:63-128 over a plain state_dict (same keys as the
reference module, see ``oracle/weights.py``):

* representation (:70-74): three 3x3/pad-1 convolutions 6->64->64->C, ReLU
  after each;
* dynamics (:85-95): ``latent + embedding[action]`` broadcast over the board,
  3x3 conv C->C + ReLU; reward = fc_out(relu(fc_hidden(mean(reward_conv(x)))));
* prediction (:104-113): value = value_fc(mean(value_conv(x))); logits =
  flatten(policy_conv(x)) ++ pass_logit.

The object is duck-type compatible with the reference ``MuZeroNet`` as used by
``MCTS`` (``initial_inference`` / ``recurrent_inference``; self_play.py:150,202).
"""
import torch
import torch.nn.functional as F


def _t(sd, key, dtype):
    v = sd[key]
    if not torch.is_tensor(v):
        v = torch.as_tensor(v)
    return v.to(dtype)


class OracleNet:
    def __init__(self, state_dict, dtype=torch.float32):
        self.dtype = dtype
        self.p = {k: _t(state_dict, k, dtype) for k in state_dict}
        self.latent_dim = self.p["dynamics.conv.weight"].shape[0]
        self.action_size = self.p["dynamics.action_embedding.weight"].shape[0]

    def eval(self):
        return self

    # -- the three networks --
    def representation(self, obs):
        p = self.p
        x = obs.to(self.dtype)
        for i in (1, 2, 3):
            x = F.relu(F.conv2d(x, p[f"representation.conv{i}.weight"],
                                p[f"representation.conv{i}.bias"], padding=1))
        return x

    def dynamics(self, latent, action):
        p = self.p
        emb = p["dynamics.action_embedding.weight"][action.long()]
        x = latent.to(self.dtype) + emb[:, :, None, None]
        x = F.relu(F.conv2d(x, p["dynamics.conv.weight"], p["dynamics.conv.bias"], padding=1))
        r = F.conv2d(x, p["dynamics.reward_conv.weight"], p["dynamics.reward_conv.bias"])
        r = r.mean(dim=[2, 3])
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

    # -- the protocol MCTS consumes --
    def initial_inference(self, obs):
        latent = self.representation(obs)
        v, logits = self.prediction(latent)
        return latent, v, logits

    def recurrent_inference(self, latent, action):
        nxt, r = self.dynamics(latent, action)
        v, logits = self.prediction(nxt)
        return nxt, r, v, logits
