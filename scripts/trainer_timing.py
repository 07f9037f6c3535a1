"""The batched trainer step (main.py:381-501's losses, mzgo.trainer
mode="batched") at main.py's configuration -- 6x6 board, latent_dim 128,
batch 128 trajectories x unroll 10 -- with the unroll's forward and every 3x3
conv backward on the HIP kernels (csrc/mzgo_train.hip; hip_forward=True)
against torch's ops (MIOpen convs; hip_forward=False, MuZeroTrainer's default
since round 5, when MIOpen measured faster).
Same trajectories, same start indices, alternating, same process.

Usage (GPU box): python scripts/trainer_timing.py [tag] -> one JSON line
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


class _Buf:
    def __init__(self, trajs):
        self.trajs = trajs

    def sample(self, n):
        return self.trajs[:n], None


def main():
    import mzgo
    from mzgo.trainer import MuZeroTrainer
    from oracle.make_golden import synthetic_trajectories
    N, C, B = 6, 128, 128
    A = N * N + 1
    steps, reps = int(os.environ.get("STEPS", 10)), int(os.environ.get("REPS", 3))
    trajs = synthetic_trajectories(N, B, seed=11)
    trainers = {}
    for hip in (True, False):
        net = mzgo.MuZeroNet(C, A).cuda()
        net.load_state_dict(mzgo.deterministic_state_dict(C, A, 7))
        trainers[hip] = MuZeroTrainer(net, mode="batched", start_index=lambda T: T // 3, hip_forward=hip)
    buf = _Buf(trajs)
    times = {True: [], False: []}
    for hip, tr in trainers.items():                  # warmup (MIOpen picks its kernels here)
        for _ in range(2):
            tr.train(buf, B)
    torch.cuda.synchronize()
    for _ in range(reps):
        for hip, tr in trainers.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                tr.train(buf, B)
            torch.cuda.synchronize()
            times[hip].append((time.perf_counter() - t0) / steps * 1e3)
    # the network part alone: forward unroll (initial + 10 recurrent) + a loss
    # over every output + backward, on fixed inputs (no targets, no optimizer)
    from mzgo.trainer import (initial_inference_hip, initial_inference_torch, recurrent_inference_hip,
                              recurrent_inference_torch)
    obs = torch.as_tensor(np.stack([t["observations"][0] for t in trajs]), dtype=torch.float32).cuda()
    acts = torch.randint(0, A, (10, B), device="cuda")
    fb = {True: [], False: []}

    def fwd_bwd(net, hip):
        f0, f = ((initial_inference_hip, recurrent_inference_hip) if hip
                 else (initial_inference_torch, recurrent_inference_torch))
        net.zero_grad()
        lat, v, lg = f0(net, obs)
        loss = (v ** 2).sum() + lg.logsumexp(1).sum()
        for k in range(10):
            lat, r, v, lg = f(net, lat, acts[k])
            loss = loss + (r ** 2).sum() + (v ** 2).sum() + lg.logsumexp(1).sum()
        loss.backward()

    for hip, tr in trainers.items():
        for _ in range(2):
            fwd_bwd(tr.net, hip)
    for _ in range(reps):
        for hip, tr in trainers.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                fwd_bwd(tr.net, hip)
            torch.cuda.synchronize()
            fb[hip].append((time.perf_counter() - t0) / steps * 1e3)
    out = {"what": "one batched trainer step (targets + bootstrap inference + forward unroll + backward + Adam), "
                   "ms; wall time over STEPS steps, best of REPS",
           "config": {"board_size": N, "latent_dim": C, "batch": B, "unroll": 10, "steps": steps, "reps": reps},
           "hip_ms": min(times[True]), "torch_miopen_ms": min(times[False]),
           "hip_all_ms": times[True], "torch_all_ms": times[False]}
    out["speedup_hip_over_torch"] = out["torch_miopen_ms"] / out["hip_ms"]
    out["network_fwd_bwd"] = {"what": "forward unroll (1 + 10 steps, B=128) + loss + backward only, ms (best of REPS)",
                              "hip_ms": min(fb[True]), "torch_miopen_ms": min(fb[False])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
