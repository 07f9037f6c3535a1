"""Helper-workgroup nondeterminism: play the same 19x19 / 64 / 800 epoch
twice, one launch per move with helpers, export the trees of a few games
after each of the first moves, and report the first tree element that
differs (node count, child ids, visits, value sums, prior rows, root priors).
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
    N, G, S = 19, 64, 800
    MOVES = int(os.environ.get("MOVES", 30))
    GAMES = [int(x) for x in os.environ.get("GAMES", "0,1,2,3").split(",")]
    A = N * N + 1
    net = mzgo.MuZeroNet(96, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(96, A, 0))
    sp = mzgo.SelfPlay(net, G, S, seed=1234)
    eng = sp.engine

    def run():
        sp.reset(epoch=1)
        trees = {}
        for mv in range(MOVES):
            sp.move()
            for g in GAMES:
                if eng.record(g)["length"] == mv + 1:
                    trees[(g, mv)] = eng.tree(g)
        return trees

    ta, tb = run(), run()
    out = []
    for key in sorted(ta):
        a, b = ta[key], tb.get(key)
        if b is None:
            out.append({"game_move": key, "missing": True})
            break
        diffs = {}
        if a["n"] != b["n"]:
            diffs["n"] = [a["n"], b["n"]]
        n = min(a["n"], b["n"])
        for k in ("child", "visits", "value_sum", "prior"):
            x, y = a[k][:n], b[k][:n]
            xb = x.view(np.uint64 if x.dtype == np.float64 else np.uint32) if x.dtype.kind == "f" else x
            yb = y.view(np.uint64 if y.dtype == np.float64 else np.uint32) if y.dtype.kind == "f" else y
            bad = np.argwhere(xb != yb)
            if bad.size:
                i = tuple(int(v) for v in bad[0])
                diffs[k] = {"count": int(len(bad)), "first": i, "a": float(x[i]), "b": float(y[i]),
                            "rows": sorted(set(int(r[0]) for r in bad))[:20]}
        if (a["root_prior"].view(np.uint64) != b["root_prior"].view(np.uint64)).any():
            diffs["root_prior"] = int((a["root_prior"] != b["root_prior"]).sum())
        if diffs:
            out.append({"game_move": key, **diffs})
            if len(out) >= 6:
                break
    print(json.dumps({"compared": len(ta), "first_differences": out}, indent=1, default=str))


if __name__ == "__main__":
    main()
