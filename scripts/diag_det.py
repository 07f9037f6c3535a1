"""Determinism check of the helper path: the same 19x19 / 64 / 800 epoch
(one launch, 3 helper workgroups per game) played RUNS times; prints how many
games' records differ from the first run.  MZGO_LIB selects the build."""
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
    N, G, S = 19, 64, int(os.environ.get("S", 800))
    A = N * N + 1
    net = mzgo.MuZeroNet(96, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(96, A, 0))
    sp = mzgo.SelfPlay(net, G, S, seed=1234)
    eng = sp.engine
    M = sp.max_moves
    runs = []
    for _ in range(int(os.environ.get("RUNS", 3))):
        sp.reset(epoch=1)
        sp.move(M)
        torch.cuda.synchronize()
        runs.append(unpack(pack_engine(eng).cpu().numpy(), G, M, N))
    out = []
    for r in runs[1:]:
        bad = 0
        for g in range(G):
            L = int(runs[0]["meta"][g, 3])
            same = (L == int(r["meta"][g, 3]) and (runs[0]["action"][g, :L] == r["action"][g, :L]).all()
                    and (runs[0]["value"][g, :L].view(np.uint64) == r["value"][g, :L].view(np.uint64)).all())
            bad += not same
        out.append(bad)
    print(json.dumps({"lib": os.path.basename(os.environ.get("MZGO_LIB", "libmzgo.so")), "games_differing": out}))


if __name__ == "__main__":
    main()
