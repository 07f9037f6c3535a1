"""Diagnostic (a -DMZGO_XCC_DIAG build): how many 19x19 helper job
acquisitions found the game's workgroup on another XCC (engine counter 4)
out of all acquisitions (counter 3's high bits), for per-move launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]
import torch  # noqa: E402

import mzgo  # noqa: E402

G, S, M = int(os.environ.get("G", 64)), int(os.environ.get("S", 800)), int(os.environ.get("M", 3))
net = mzgo.MuZeroNet(96, 362).cuda().eval()
net.load_state_dict(mzgo.deterministic_state_dict(96, 362, 0))
sp = mzgo.SelfPlay(net, G, S, seed=1234)
sp.reset(epoch=0)
c0 = sp.engine.counters()
for _ in range(M):
    sp.move()
torch.cuda.synchronize()
c1 = sp.engine.counters()
acq = (c1["dynamics_convs"] >> 40) - (c0["dynamics_convs"] >> 40)
print(f"G={G} S={S} moves={M}: acquisitions {acq}, game on another XCC {c1['tail_convs'] - c0['tail_convs']}")
