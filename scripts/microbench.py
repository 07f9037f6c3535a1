"""Per-phase timing of the engine's kernels (development aid).

Times, for 9x9 / C=96 / G=256: batched recurrent_inference (the dynamics conv
+ heads alone), initial_inference, one full search (k_search, S sims) and one
self-play move, each averaged over several launches with HIP events.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]
import torch  # noqa: E402

import mzgo  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    N = int(os.environ.get("N", 9))
    G = int(os.environ.get("G", 256))
    S = int(os.environ.get("S", 200))
    C = 96
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    eng = net.engine()
    lat = torch.rand(G, C, N, N, device="cuda")
    act = torch.randint(0, A, (G,), device="cuda")
    obs = (torch.rand(G, 6, N, N, device="cuda") < 0.2).float()
    obs[:, 2:] = 0
    out = {}
    out["recurrent_inference_ms"] = timeit(lambda: eng.recurrent_inference(lat, act))
    out["initial_inference_ms"] = timeit(lambda: eng.initial_inference(obs))
    seng = net.engine(num_games=G, num_simulations=S)
    out["search_ms"] = timeit(lambda: seng.search(obs), reps=3)
    sp = mzgo.SelfPlay(net, G, S)
    sp.reset()
    out["selfplay_move_ms"] = timeit(sp.move, reps=3)
    out["per_sim_us"] = out["search_ms"] / S * 1e3
    out["conv_share"] = out["recurrent_inference_ms"] / (out["search_ms"] / S)
    print(json.dumps({"N": N, "G": G, "S": S, **out}))


if __name__ == "__main__" and not os.environ.get("STAMPS") and not os.environ.get("MOVE_STAMPS") \
        and not os.environ.get("GAME_STAMPS"):
    main()


def stamps_report():
    """With MZGO_LIB=...libmzgo_stamps.so: cycles per simulation by phase."""
    import ctypes

    import numpy as np
    from mzgo import _lib
    N = int(os.environ.get("N", 9))
    G = int(os.environ.get("G", 256))
    S = int(os.environ.get("S", 200))
    C, A = 96, N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    seng = net.engine(num_games=G, num_simulations=S)
    obs = torch.zeros(G, 6, N, N)
    fn = _lib.lib.mzgo_debug_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    buf = np.zeros((G, 96), np.uint64)
    seng.search(obs)
    torch.cuda.synchronize()
    fn(seng.handle, buf.ctypes.data_as(ctypes.c_void_p))          # drop the warm-up
    ms = timeit(lambda: seng.search(obs), reps=1)
    fn(seng.handle, buf.ctypes.data_as(ctypes.c_void_p))
    names = ["select", "stage", "conv_epilogue", "heads_backup", "p4", "p5", "conv_loop", "conv_sync"]
    allp = buf.astype(np.float64).mean(0) / (2 * S)               # warm-up call inside timeit + 1 rep
    per_sim, waves = allp[:8], allp[8:20]
    total = per_sim.sum()
    print(json.dumps({"N": N, "G": G, "S": S, "search_ms": ms,
                      "cycles_per_sim": {n: round(float(v)) for n, v in zip(names, per_sim) },
                      "share": {n: round(float(v / total), 3) for n, v in zip(names, per_sim)},
                      "wave_conv_loop": [round(float(v)) for v in waves if v > 0],
                      "stage_split": [round(float(v)) for v in allp[20:22]],
                      "select_split_root_deeper": [round(float(v)) for v in allp[22:24]],
                      "root_level_split": [round(float(v)) for v in allp[24:28]],
                      "stage_load_wait": round(float(allp[28])),
                      "stage_detail_scatter0_transform": [round(float(v)) for v in allp[29:31]],
                      "wave_stage_work": [round(float(v)) for v in allp[32:44]],
                      "wave_stage_wait": [round(float(v)) for v in allp[44:56]],
                      "factored_expand_pre_barrier": round(float(allp[56])),
                      "wave1_logits": round(float(allp[57])), "wave1_priors": round(float(allp[58])),
                      "root_conv_loady_expand_total": [round(float(allp[i]) * S) for i in (60, 61, 62)],
                      "expand_per_child_copyE_heads_logits_priors": [round(float(allp[i] / max(allp[68], 1e-9)))
                                                                     for i in (64, 65, 66, 67)],
                      "expanded_children_per_search": float(allp[68] * S),
                      "verify_steps_total": [round(float(allp[i]) * S) for i in (72, 73, 74)],
                      "verify_step2_main_exact": [round(float(allp[i]) * S) for i in (78, 79)],
                      "verify_step2_loop_all_waves": round(float(allp[80]) * S),
                      "parent_materialize_and_conv_tail": [round(float(allp[i]) * S) for i in (81, 82)],
                      "verify_step1_w0_pre_minmax_prefix_reciprocals": [round(float(allp[i]) * S) for i in (75, 76, 77)],
                      "batch_end_barrier_total": round(float(allp[63]) * 2 * S / 2),
                      "batches_per_search": float(buf[:, 31].astype(np.float64).mean() / 2),
                      "batched_sims_per_search": float(buf[:, 28].astype(np.float64).mean() / 2),
                      "batch_detail_total_w0": [round(float(v) * S) for v in allp[69:72]],
                      "conv_slots_total": [round(float(allp[i]) * S) for i in (1, 6, 7, 20, 21, 29, 30)],
                      "slot3_total": round(float(allp[3]) * S),
                      "convs_per_search": float(buf[:, 59].astype(np.float64).mean() / 2),
                      "top_slots_total": sorted([(int(i), round(float(allp[i]) * S)) for i in range(len(allp)) if allp[i] > 0],
                                               key=lambda x: -x[1])[:24],
                      "implied_clock_GHz": total * S / (ms * 1e6)}))


if os.environ.get("STAMPS"):
    stamps_report()


def move_stamps_report():
    """With MZGO_LIB=...libmzgo_stamps.so and MOVE_STAMPS=1: cycles per self-play
    move by phase (k_selfplay_move slots 83-87), averaged over games and moves."""
    import ctypes

    import numpy as np
    from mzgo import _lib
    N = int(os.environ.get("N", 9))
    G = int(os.environ.get("G", 256))
    S = int(os.environ.get("S", 200))
    M = int(os.environ.get("MOVES", 20))
    C, A = 96, N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    sp = mzgo.SelfPlay(net, G, S)
    sp.reset()
    fn = _lib.lib.mzgo_debug_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    buf = np.zeros((G, 96), np.uint64)
    sp.move()
    torch.cuda.synchronize()
    fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p))
    ms = timeit(sp.move, reps=M)
    fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p))
    per = buf[:, 83:88].astype(np.float64).mean(0) / (M + 1)
    rep = buf[:, 88:91].astype(np.float64).mean(0) / (M + 1)
    names = ["board_load_record", "representation", "root_priors_dirichlet", "simulations", "choose_and_step"]
    tot = per.sum()
    print(json.dumps({"N": N, "G": G, "S": S, "move_ms": ms,
                      "cycles_per_move": {n: round(float(v)) for n, v in zip(names, per)},
                      "share": {n: round(float(v / tot), 3) for n, v in zip(names, per)},
                      "representation_conv1_conv2_conv3": [round(float(v)) for v in rep]}))


if os.environ.get("MOVE_STAMPS"):
    move_stamps_report()


def game_stamps_report():
    """With MZGO_LIB=...libmzgo_stamps.so and GAME_STAMPS=1: phase cycles over
    whole self-play games (every slot's stamps summed over all its moves),
    mean over the G games, plus the slowest game's."""
    import ctypes

    import numpy as np
    from mzgo import _lib
    N = int(os.environ.get("N", 9))
    G = int(os.environ.get("G", 256))
    S = int(os.environ.get("S", 200))
    C, A = 96, N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    sp = mzgo.SelfPlay(net, G, S)
    fn = _lib.lib.mzgo_debug_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    buf = np.zeros((G, 96), np.uint64)
    sp.reset()
    sp.move(sp.max_moves)
    torch.cuda.synchronize()
    fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p))      # drop the warm-up game
    sp.reset(epoch=1)
    c0 = sp.engine.counters()
    ms = timeit(lambda: None, reps=1)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    sp.move(sp.max_moves)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b)
    c1 = sp.engine.counters()
    fn(sp.engine.handle, buf.ctypes.data_as(ctypes.c_void_p))
    f = buf.astype(np.float64)
    move_tot = f[:, 83:88].sum(1)
    slow = int(np.argmax(move_tot))
    names = ["board_load_record", "representation", "root_priors_dirichlet", "simulations", "choose_and_step"]
    top = sorted([(int(i), float(f[:, i].mean())) for i in range(83) if f[:, i].mean() > 0], key=lambda x: -x[1])[:16]
    print(json.dumps({"N": N, "G": G, "S": S, "game_ms": ms,
                      "moves": c1["moves"] - c0["moves"], "convs": c1["dynamics_convs"] - c0["dynamics_convs"],
                      "mean_game_cycles": float(move_tot.mean()), "max_game_cycles": float(move_tot.max()),
                      "move_phases_mean": {n: round(float(f[:, 83 + k].mean())) for k, n in enumerate(names)},
                      "move_phases_slowest": {n: round(float(f[slow, 83 + k])) for k, n in enumerate(names)},
                      "search_slots_mean_top": [(i, round(v)) for i, v in top],
                      "convs_slowest_game": float(f[slow, 59]), "convs_mean_game": float(f[:, 59].mean()),
                      "wall_slots_mean": {i: round(float(f[:, i].mean())) for i in
                                          (0, 2, 3, 4, 5, 22, 23, 24, 25, 26, 27, 40, 41, 42, 43, 52, 53, 54, 62, 63, 69, 70,
                                           71, 72, 73, 74, 75, 76, 77, 78, 79, 81, 82)},
                      "selects_per_game": float(f[:, 92].mean()), "deep_levels_per_game": float(f[:, 91].mean()),
                      "mean_leaf_depth": float(f[:, 95].sum() / max(f[:, 92].sum(), 1)),
                      "batches_per_game": float(f[:, 31].mean()), "batched_sims_per_game": float(f[:, 28].mean()),
                      "seq_replay_batches_per_game": float(f[:, 93].mean()),
                      "seq_replay_sims_per_game": float(f[:, 94].mean()),
                      "expand_slots_64_68_total": [round(float(f[:, i].mean())) for i in (64, 65, 66, 67, 68)]}))


if os.environ.get("GAME_STAMPS"):
    game_stamps_report()
