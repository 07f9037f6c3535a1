"""k_tconv phase split from a -DMZGO_TCONV_STAMPS build (diagnostic only):
MZGO_LIB=muzero-go_amd/mzgo/libmzgo_ts.so python scripts/tconv_stamps.py"""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]
import torch
import mzgo
from mzgo import _lib
N, C, B, G, S = 19, 256, 20, 64, 64
A = N * N + 1
net = mzgo.ResMuZeroNet(C, A, B).to("cuda").eval()
net.load_state_dict(mzgo.deterministic_res_state_dict(C, A, B, 0))
sp = mzgo.SelfPlay(net, G, S, seed=1234)
sp.reset()
sp.move()
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 128)()
f = _lib.lib.mzgo_debug_tconv_stamps
f.argtypes = [ctypes.c_void_p]
f(out)                       # zero after warmup
t0 = time.perf_counter()
sp.move()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
f(out)
n = out[6]
clk = [out[w * 16] / max(out[w * 16 + 8], 1) * 0.1 for w in range(8)]
names = ["total", "prologue", "vmcnt waits", "barriers", "MFMA steps", "epilogue", "", "epi: exchange", "",
         "epi: give", "epi: barrier + finish", "epi: heads"]
print(f"workgroup-launches {n}, move {dt*1e3:.1f} ms  (wave 0; other waves per column); in-kernel clock GHz per wave: " + " ".join(f"{c:.3f}" for c in clk))
for k, nm in enumerate(names):
    if not nm: continue
    per = " ".join(f"{out[w * 16 + k] / max(out[w * 16 + 6], 1):7.0f}" for w in range(8))
    print(f"  {nm:12s} {out[k] / max(n, 1):10.0f} cycles/launch  ({out[k] / max(out[0], 1) * 100:5.1f} %)  waves: {per}")
