"""Whole-game launch vs per-move launches: where do the records differ?

Plays the same epoch several ways on one engine (19x19 / 64 / 800 by
default) and compares the records pairwise: games with any difference, the
largest value difference, the first differing move.  MZGO_HELPERS_PER_GAME
in the environment sets the helper workgroups (read at each launch).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import mzgo
    from mzgo.distributed import pack_engine, unpack
    N = int(os.environ.get("N", 19))
    G = int(os.environ.get("G", 64))
    S = int(os.environ.get("S", 800))
    A = N * N + 1
    net = mzgo.MuZeroNet(96, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(96, A, 0))
    sp = mzgo.SelfPlay(net, G, S, seed=1234)
    eng = sp.engine
    M = sp.max_moves

    def run(mode, helpers):
        os.environ["MZGO_HELPERS_PER_GAME"] = str(helpers)
        sp.reset(epoch=1)
        if mode == "per":
            for _ in range(M):
                sp.move()
        else:
            sp.move(M)
        torch.cuda.synchronize()
        return unpack(pack_engine(eng).cpu().numpy(), G, M, N)

    runs = {}
    for name, mode, h in [("whole_h3_a", "whole", 3), ("whole_h3_b", "whole", 3), ("per_h3_a", "per", 3),
                          ("per_h3_b", "per", 3), ("whole_h0", "whole", 0), ("per_h0", "per", 0)]:
        runs[name] = run(mode, h)

    def cmp(a, b):
        ra, rb = runs[a], runs[b]
        games, first, vmax = 0, [], 0.0
        for g in range(G):
            L = int(ra["meta"][g, 3])
            same_act = L == int(rb["meta"][g, 3]) and (ra["action"][g, :L] == rb["action"][g, :L]).all()
            va, vb = ra["value"][g, :L], rb["value"][g, :L]
            diff = np.flatnonzero(va.view(np.uint64) != vb.view(np.uint64)) if same_act else np.array([0])
            if not same_act or diff.size:
                games += 1
                first.append(int(diff[0]) if diff.size else -1)
                if same_act:
                    vmax = max(vmax, float(np.abs(va - vb).max()))
            if not same_act:
                first[-1] = -2
        return dict(games_differing=games, first_diff_moves=first[:12], max_value_abs_diff=vmax)

    names = list(runs)
    out = {f"{a}~{b}": cmp(a, b) for i, a in enumerate(names) for b in names[i + 1:]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
