"""Config-5 tower: inference error against the oracle per tower depth.

Measures ResMuZeroNet (19x19, C=256; bf16 MFMA operands, fp32 accumulation,
bf16 activations) against oracle/resnet.py at 2, 5, 10 and 20 residual
blocks: vs OracleResNet(bf16=True) (the engine's rounding points in float64)
and vs OracleResNet(bf16=False) (the architecture in fp32).  Prints one JSON
line per depth; tests/test_gpu_tower.py's per-depth bounds come from these.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def errs(got, want):
    d = (got - want).abs()
    return dict(max=d.max().item(), mean=d.mean().item(), ref_mean=want.abs().mean().item(),
                ref_max=want.abs().max().item())


def main():
    import mzgo
    from oracle.positions import random_position
    from oracle.resnet import OracleResNet
    torch.set_num_threads(16)
    N, C, B = 19, 256, 4
    A = N * N + 1
    depths = [int(x) for x in (sys.argv[1:] or ["2", "5", "10", "20"])]
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(np.stack([random_position(N, int(rng.integers(0, N * N // 2)), int(rng.integers(1 << 30)))
                                     for _ in range(B)]).astype(np.float32))
    act = torch.tensor([0, A - 1, 3, A // 2])
    for blocks in depths:
        t0 = time.time()
        sd = mzgo.deterministic_res_state_dict(C, A, blocks, 0)
        net = mzgo.ResMuZeroNet(C, A, blocks).to("cuda").eval()
        net.load_state_dict(sd)
        lat, v, lg = net.initial_inference(obs.cuda())
        nl, r, v2, lg2 = net.recurrent_inference(lat, act.cuda())
        out = {"blocks": blocks}
        for name, bf in (("bf16", True), ("f32", False)):
            o = OracleResNet(sd, blocks, bf16=bf)
            with torch.no_grad():
                el, ev, elg = o.initial_inference(obs)
                enl, er, ev2, elg2 = o.recurrent_inference(lat.cpu(), act)
            out[name] = dict(latent=errs(lat.cpu(), el), value=errs(v.cpu(), ev), logits=errs(lg.cpu(), elg),
                             next_latent=errs(nl.cpu(), enl), reward=errs(r.cpu(), er),
                             value1=errs(v2.cpu(), ev2), logits1=errs(lg2.cpu(), elg2))
        out["s"] = time.time() - t0
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
