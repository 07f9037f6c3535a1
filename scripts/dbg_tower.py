"""Debug: per-board / per-channel-chunk error of the tower engine vs the bf16 oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]
import numpy as np, torch
import mzgo
from oracle.resnet import OracleResNet
from oracle.positions import random_position
for (N, C, blocks, B) in [(5, 64, 0, 6), (5, 64, 0, 8), (5, 64, 1, 6), (5, 64, 2, 6), (5, 128, 0, 6), (9, 128, 1, 6), (19, 256, 2, 8)]:
    A = N * N + 1
    sd = mzgo.deterministic_res_state_dict(C, A, blocks, 0)
    net = mzgo.ResMuZeroNet(C, A, blocks).to("cuda").eval(); net.load_state_dict(sd)
    emu = OracleResNet(sd, blocks, bf16=True)
    obs = torch.from_numpy(np.stack([random_position(N, 3 * b, b) for b in range(B)]).astype(np.float32))
    lat, v, lg = net.initial_inference(obs.cuda())
    elat, ev, elg = emu.initial_inference(obs)
    d = (lat.cpu() - elat).abs()
    per = d.reshape(B, C // 64, 64, -1).amax(dim=(2, 3))
    print(N, C, blocks, B, "lat max per board/chunk:", per.numpy().round(3).tolist(), "v", (v.cpu() - ev).abs().max().item(), "lg", (lg.cpu() - elg).abs().max().item())
    act = torch.arange(B) % A
    nl, r, v2, lg2 = net.recurrent_inference(lat, act.cuda())
    enl, er, ev2, elg2 = emu.recurrent_inference(lat.cpu(), act)
    d = (nl.cpu() - enl).abs()
    per = d.reshape(B, C // 64, 64, -1).amax(dim=(2, 3))
    print("   rec per board/chunk:", per.numpy().round(3).tolist(), "r", (r.cpu() - er).abs().max().item(), "v", (v2.cpu() - ev2).abs().max().item())
