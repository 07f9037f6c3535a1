"""Per-segment phase shares of a whole 9x9 self-play epoch (diagnostic,
-DMZGO_STAMPS build): the epoch is played in move segments (one launch per
segment; k moves per launch == k one-move launches, test_gpu_selfplay), the
stamps are read and reset after each, so every segment reports its phase
shares and the spread of its games' busy cycles (where the epoch's tail
builds up).  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so python scripts/phases_split.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd"), os.path.join(ROOT, "scripts")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from phases import PHASES, MOVE_SLOTS  # noqa: E402


def main():
    import mzgo
    from mzgo import _lib
    N, G, S, C = 9, 256, 200, 96
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    sp = mzgo.SelfPlay(net, G, S, seed=1234)
    fn = _lib.lib.mzgo_debug_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    buf = np.zeros((G, 96), np.uint64)
    sp.reset(epoch=0)
    sp.move(sp.max_moves)
    torch.cuda.synchronize()
    fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p))
    sp.reset(epoch=1)
    segs = [(0, 20), (20, 40), (40, 60), (60, 70), (70, 81)]
    rows = []
    tot_game = np.zeros(G)
    per = []
    slowest_rows = []
    for m0, m1 in segs:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        sp.move(m1 - m0)
        b.record()
        torch.cuda.synchronize()
        fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p))
        f = buf[:G].astype(np.float64)
        game = f[:, MOVE_SLOTS].sum(1)
        tot_game += game
        per.append(game)
        top = np.argsort(game)[-8:]                      # the segment's 8 slowest games
        rows_extra = {k: round(float(f[top][:, v].sum(1).mean()) / 1e6, 2) for k, v in PHASES.items()}
        rows_extra["convs"] = float(f[top, 59].mean())
        rows_extra["selects"] = float(f[top, 92].mean())
        rows_extra["leaf_depth_sum"] = float(f[top, 95].mean())
        rows_extra["slots"] = {int(i): round(float(f[top, i].mean()) / 1e6, 3) for i in range(96) if f[top, i].any()}
        slowest_rows.append(rows_extra)
        tot = {k: float(f[:, v].sum()) for k, v in PHASES.items()}
        alls = sum(tot.values()) or 1.0
        rows.append({"moves": [m0, m1], "ms": a.elapsed_time(b),
                     "shares": {k: round(v / alls, 4) for k, v in tot.items()},
                     "game_cycles_mean": float(game.mean()), "game_cycles_max": float(game.max()),
                     "idle_share_if_alone": float(1 - game.mean() / max(game.max(), 1)),
                     "convs_per_game": float(f[:, 59].mean()),
                     "playing_games": int((game > 0).sum())})
    per = np.array(per)
    slow = int(tot_game.argmax())
    out = {"segments": rows, "epoch_idle_share": float(1 - tot_game.mean() / tot_game.max()),
           "slowest_game_segments": [float(x) for x in per[:, slow]],
           "mean_game_segments": [float(x) for x in per.mean(1)],
           "slowest8_phase_Mcycles_per_segment": slowest_rows,
           "corr_segment_vs_total": [float(np.corrcoef(per[i], tot_game)[0, 1]) for i in range(len(segs))]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
