"""Per-phase shares of a whole self-play epoch, from the
-DMZGO_STAMPS diagnostic build (scripts/build_stamps.sh; in the real kernel no
stamp executes).

Thread 0 of each game's workgroup adds shader-clock deltas between
consecutive stamps ("laps") into per-slot counters, so the lap slots of one
workgroup partition its time.  They are grouped into the phases below, summed
over every game of one epoch (9x9 / 256 games / 200 simulations by default,
bench.py's step), and reported as shares of the total, beside the epoch's
tail: each game's busy cycles against the slowest game's (the CU-time idle
while the last games finish).

Usage (GPU box):  MZGO_LIB=$PWD/muzero-go_amd/mzgo/libmzgo_stamps.so \
                  python scripts/phases.py <tag>   -> gpurun_out/<tag>_phases.json
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

# lap slots (mzgo_common.hpp's map) -> phase
PHASES = {
    "representation": [84],                                   # board planes + conv1-3 + heads (per move)
    "root": [85, 4],                                          # root priors + Dirichlet; root batch backups
    "select": [0, 22, 23, 24, 25, 26, 27, 32, 33, 35, 36, 37, 38, 39, 49],  # select_leaf walks (+ the barrier after
                                                              # them; 32/33 a lazy node's policy sums / resumed walk)
    "conv": [1, 6, 7, 20, 21, 29, 30, 52, 53, 54, 60, 81, 82],  # parent / root dynamics convs (Winograd)
    "expand": [2, 3, 5, 40, 41, 42, 43, 61, 62, 69, 70, 71],  # child expansions (heads, priors), picks, backups
    "replay": [63, 72, 73, 74, 75, 76, 77, 78, 79],           # verify_batch: the batch's replayed selects
    "board": [83, 87],                                        # board load + record, action choice + board step
}
MOVE_SLOTS = [83, 84, 85, 86, 87]


def _decile(f, game, sp):
    order = np.argsort(game)
    n = max(len(game) // 10, 1)
    slow, mid = order[-n:], order[len(game) // 2 - n // 2:len(game) // 2 - n // 2 + n]
    lens = np.array([sp.engine.record(int(g))["length"] for g in range(len(game))])

    def per(idx):
        return {k: float(f[idx][:, v].sum(1).mean()) for k, v in PHASES.items()}
    return {"games": int(n), "cycles_slowest": per(slow), "cycles_median_decile": per(mid),
            "moves_slowest": float(lens[slow].mean()), "moves_median_decile": float(lens[mid].mean()),
            "moves_all": float(lens.mean())}


def main():
    # the game-per-workgroup launch (one game's whole epoch per workgroup: the
    # tail this script measures); the move-parallel epoch's queue has no
    # per-game workgroups
    os.environ.setdefault("MZGO_MOVE_PARALLEL", "0")
    import mzgo
    from mzgo import _lib
    tag = sys.argv[1] if len(sys.argv) > 1 else "phases"
    N = int(os.environ.get("N", 9))
    G = int(os.environ.get("G", 256))
    S = int(os.environ.get("S", 200))
    C, A = 96, N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    sp = mzgo.SelfPlay(net, G, S, seed=1234)
    fn = _lib.lib.mzgo_debug_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    # one row per tree slot (the move-parallel queue's workgroups at 19x19: one per CU)
    rows = max(G, torch.cuda.get_device_properties(0).multi_processor_count)
    buf = np.zeros((rows, 96), np.uint64)
    sp.reset(epoch=0)
    sp.move(sp.max_moves)                                     # warm-up epoch, stamps dropped
    torch.cuda.synchronize()
    if fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p)) != 0:
        raise RuntimeError("mzgo_debug_stamps failed: load the -DMZGO_STAMPS build (MZGO_LIB)")
    sp.reset(epoch=1)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0 = sp.engine.counters()
    a.record()
    sp.move(sp.max_moves)
    b.record()
    torch.cuda.synchronize()
    c1 = sp.engine.counters()
    ms = a.elapsed_time(b)
    fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p))
    if os.environ.get("MZGO_MOVE_PARALLEL") == "1":
        # the move-parallel epoch: the queue's workgroups have no games; phase
        # shares over every slot row (the boards launch's own slots 83 / 87 too)
        fa = buf.astype(np.float64)
        # the boards launch runs no search: its per-move laps 84-86 and 88-90
        # (representation, root, simulations) hold no interval there
        fa[:, [84, 85, 86, 88, 89, 90]] = 0.0
        tot = {k: float(fa[:, v].sum()) for k, v in PHASES.items()}
        alls = sum(tot.values())
        out = {"tag": tag, "workload": f"{N}x{N} Go self-play, {G} parallel games/GPU, {S} sims/move",
               "schedule": "move-parallel (boards launch + k_search_queue)", "epoch_ms_stamps_build": ms,
               "shares": {k: v / alls for k, v in tot.items()},
               "cycles_per_workgroup": {k: v / rows for k, v in tot.items()},
               "slots_sum": {int(i): float(fa[:, i].sum()) for i in range(fa.shape[1]) if fa[:, i].any()}}
        d = os.path.join(ROOT, "gpurun_out")
        os.makedirs(d, exist_ok=True)
        json.dump(out, open(os.path.join(d, f"{tag}_phases.json"), "w"), indent=1)
        print(json.dumps(out))
        return
    f = buf[:G].astype(np.float64)
    game = f[:, MOVE_SLOTS].sum(1)                            # each game's busy cycles (its whole epoch)
    sims_slots = sorted({s for k, v in PHASES.items() if k not in ("representation", "board") for s in v} - {85})
    tot = {k: float(f[:, v].sum()) for k, v in PHASES.items()}
    alls = sum(tot.values())
    out = {
        "tag": tag, "workload": f"{N}x{N} Go self-play, {G} parallel games/GPU, {S} sims/move",
        "source": "-DMZGO_STAMPS build (s_memtime laps of each game's workgroup), one whole epoch; "
                  "scripts/phases.py",
        "epoch_ms_stamps_build": ms,
        "shares": {k: v / alls for k, v in tot.items()},
        "cycles_per_game": {k: v / G for k, v in tot.items()},
        "simulation_slots_vs_move_stamp": float(f[:, sims_slots].sum() / max(f[:, 86].sum(), 1)),
        "tail": {"mean_game_cycles": float(game.mean()), "max_game_cycles": float(game.max()),
                 "idle_cu_share": float(1 - game.mean() / game.max()),
                 "p10_p50_p90_game_cycles": [float(np.percentile(game, q)) for q in (10, 50, 90)],
                 "what": "1 - mean/max of the games' busy cycles: the CU-time the epoch leaves idle while "
                         "its slowest games finish (one game per CU)"},
        "convs_per_game": float(f[:, 59].mean()),
        "engine_counters": {k: c1[k] - c0[k] for k in ("simulations", "dynamics_convs", "tail_convs")},
        # the 9x9 epoch tail with tail helpers (slots 44-47): the CU-time the
        # epoch leaves idle counts a finished game's workgroup as busy while it
        # computes units for running games
        "tail_helpers": {
            "unit_cycles_per_game": float(f[:, 44].mean()), "units": float(f[:, 45].sum()),
            "jobs_served": float(f[:, 46].sum()), "tail_phase_cycles_per_game": float(f[:, 47].mean()),
            "idle_cu_share_with_helpers": float(1 - (game.sum() + f[:, 44].sum()) / (len(game) * game.max())),
        },
        # what the slowest games (the epoch's tail) spend their cycles on,
        # against the median decile, and how long their games are
        "slowest_decile": _decile(f, game, sp),
        # every slot's mean per game (lap slots: thread 0's partition; others:
        # wave sums / counters, mzgo_common.hpp's map)
        "slots_mean_per_game": {int(i): round(float(f[:, i].mean())) for i in range(f.shape[1]) if f[:, i].any()},
    }
    # (written under gpurun_out/, which the GPU call merges back; copy it to
    # profiles/<tag>_phases.json and profiles/latest_phases.json, which bench.py reads)
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    json.dump(out, open(os.path.join(d, f"{tag}_phases.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
