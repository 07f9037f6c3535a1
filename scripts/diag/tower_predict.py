"""Speculation study on the device's own config-5 tree (diagnostic):
one 19x19 search with the config-5 network (C=256, 20 blocks) on the tower
engine, the per-node tower outputs recorded (Engine.record_nodes), then the
oracle MCTS replays the search on those outputs (tests/test_gpu_tower.py's
_ReplayNet) while predictors of the next simulations' root children are
scored against what the replay does.  Also prints the engine's towers per
simulation for the same search at several MZGO_TOWER_SPEC values."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd"), os.path.join(ROOT, "tests")]

import mzgo  # noqa: E402
from oracle import gogame  # noqa: E402
from oracle.mcts import MCTS as OracleMCTS  # noqa: E402
from oracle.rng import SearchHooks  # noqa: E402
from test_gpu_tower import _ReplayNet  # noqa: E402

N, C, BL = 19, 256, int(os.environ.get("BLOCKS", "20"))
S = int(os.environ.get("SIMS", "1000"))
A = N * N + 1
net = mzgo.ResMuZeroNet(C, A, BL).to("cuda").eval()
net.load_state_dict(mzgo.deterministic_res_state_dict(C, A, BL, 0))
obs = gogame.init_state(N).astype(np.float64)
sseed, game, move = 1234, 3, 0
rs = np.random.RandomState(7)
noise = rs.dirichlet([0.15] * A)
m = mzgo.MCTS(net, A, S, seed=sseed, game=game)
eng = net.engine(num_games=1, num_simulations=S, **m.cfg)
out = {}
for spec in ("1", "16", "32"):
    os.environ["MZGO_TOWER_SPEC"] = spec
    c0 = eng.counters()
    m.run(obs, move_index=move, noise=torch.from_numpy(noise))
    c1 = eng.counters()
    out[f"towers_per_sim_spec{spec}"] = (c1["dynamics_convs"] - c0["dynamics_convs"]) / S
rec = torch.zeros(1, S + 1, A + 2, dtype=torch.float32, device="cuda")
eng.record_nodes(rec)
m.run(obs, move_index=move, noise=torch.from_numpy(noise))
eng.record_nodes(None)
t = eng.tree(0)
nodes = rec[0].cpu().numpy()
hooks = SearchHooks(sseed, game, move)
om = OracleMCTS(_ReplayNet(nodes, t["child"], A), A, S, choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
                noise=lambda p, a, e: (1 - e) * p + e * noise)
recs = []
orig = om.select_leaf


def snap(root, vm):
    ch = root.children
    el = [a for a, c in ch.items() if vm[a] > 0 and c["prior"] > 0]
    if not all(ch[a]["node"] is not None for a in el):
        return None
    P = np.array([ch[a]["prior"] for a in el])
    n = np.array([ch[a]["node"].visit_count for a in el], float)
    q = np.array([ch[a]["node"].value() if ch[a]["node"].visit_count > 0 else 0.0 for a in el])
    return (np.array(el), P, n, q, root.visit_count)


def sl(root, vm):
    s = snap(root, vm)
    path, a = orig(root, vm)
    ra = path[1] if len(path) > 1 else None
    act = [k for k, c in root.children.items() if c["node"] is ra][0] if ra is not None else None
    recs.append((s, act, len(path) - 1))
    return path, a


om.select_leaf = sl
oroot, _, _ = om.run(obs)


def predict(s, first, k, mode):
    el, P, n, q, Nv = s
    n, q = n.copy(), q.copy()
    i0 = list(el).index(first)

    def visit(i):
        nonlocal Nv
        if mode == "mean":
            q[i] = (q[i] * n[i] + np.mean(q)) / (n[i] + 1)
        n[i] += 1
        Nv += 1
    if mode == "static":
        lo, hi = q.min(), q.max()
        qn = (q - lo) / (hi - lo) if hi > lo else q
        sc = qn + 2.5 * P * np.sqrt(max(1, Nv)) / (1 + n)
        sc[i0] = -1e9
        return [first] + [int(el[j]) for j in np.argsort(-sc, kind="stable")[:k - 1]]
    visit(i0)
    res = [first]
    for _ in range(k - 1):
        lo, hi = q.min(), q.max()
        qn = (q - lo) / (hi - lo) if hi > lo else q
        sc = qn + 2.5 * P * np.sqrt(max(1, Nv)) / (1 + n)
        i = int(np.argmax(sc))
        res.append(int(el[i]))
        visit(i)
    return res


start = next(i for i, r in enumerate(recs) if r[0] is not None)
out["depth_hist"] = np.bincount([d for _, _, d in recs]).tolist()
runs, r = [], 1
for i in range(start + 1, len(recs)):
    if recs[i][1] == recs[i - 1][1]:
        r += 1
    else:
        runs.append(r)
        r = 1
out["same_root_child_run_mean"] = float(np.mean(runs)) if runs else None
qs = recs[-1][0][3] if recs[-1][0] is not None else None
if qs is not None:
    out["root_child_q_range"] = [float(qs.min()), float(qs.max())]
for mode in ("static", "fixed", "mean"):
    for Bp in (16, 32):
        hits, i = [], start
        while i < len(recs):
            s, first, _ = recs[i]
            pred = predict(s, first, Bp, mode)
            k = 0
            while k < Bp and i + k < len(recs) and recs[i + k][1] == pred[k]:
                k += 1
            hits.append(max(k, 1))
            i += max(k, 1)
        out[f"{mode}_B{Bp}_accepted"] = float(np.mean(hits))
print(json.dumps(out))
