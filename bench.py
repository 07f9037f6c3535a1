"""Benchmark: MCTS simulations/sec + self-play moves/sec, 9x9 Go, 200 sims/move.

BASELINE.json's metric on configs[1]: 256 parallel self-play games per GPU,
200 simulations per move, the reference network (latent_dim 96) with
deterministic random-init weights, fp32.  One *step* = one whole self-play
epoch: all 256 games from the empty board until
every one has ended.  Under compat "reference" (the bench's protocol, SURVEY
§0.6: the action is a uniform draw over the legal moves, never read from the
search) an epoch is the move-parallel pair: k_selfplay_boards records and
steps every game's boards without their searches, then k_search_queue runs
every recorded move's search (representation + root priors, 200 simulations
of select / dynamics + prediction / expand / backup, the root value) from one
queue on one workgroup per CU.  MZGO_MOVE_PARALLEL=0 times the
game-per-workgroup launch instead (one fused k_selfplay_move launch playing
each game's moves back to back on its CU); the records are byte-identical.

Multi-GPU, one process per GPU: ``bench.py --gpus N`` starts the N rank
processes itself (or runs under torch.distributed.run with --nproc-per-node
N).  Games are sharded by global id (rank * G + slot); the only collective is
the RCCL gather of every rank's packed game records to rank 0 after every
epoch, inside the timed region (BASELINE config 3's trajectory gather);
value = all ranks' simulations / the max over ranks of the timed span;
scaling "weak".

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

def mfma_per_conv(N, cin, cout):
    """16x16x4 f32 MFMAs of one 3x3 conv of one board (Winograd at 9x9 / 19x19)."""
    if N == 9:
        return 20 * (cout // 16) * (cin // 4)
    if N == 19:
        return 5 * 20 * (cout // 16) * (cin // 4)
    return 9 * (cin // 4) * (cout // 16) * ((N * N + 15) // 16)


def cpu_baseline(N, C, S, budget_s=12.0, blocks=None, threads=1):
    """The oracle (CPU restatement of self_play.py's MCTS, batch-1 torch net,
    object tree) timed on this host with ``threads`` intra-op threads (1: the
    per-process leg), on a bounded sample.
    blocks: the residual-tower network of config 5 (oracle/resnet.py, fp32)."""
    import numpy as np

    from oracle.mcts import MCTS
    from oracle.net import OracleNet
    from oracle.rng import SearchHooks, injected_noise
    from oracle.weights import deterministic_state_dict
    from oracle import gogame

    torch.set_num_threads(threads)
    A = N * N + 1
    if blocks is None:
        net = OracleNet(deterministic_state_dict(C, A, 0))
    else:
        from mzgo.weights import deterministic_res_state_dict
        from oracle.resnet import OracleResNet
        net = OracleResNet(deterministic_res_state_dict(C, A, blocks, 0), blocks)
    st = gogame.init_state(N)
    sims, moves, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        hooks = SearchHooks(1234, 0, moves)
        noise = injected_noise(1234, 0, moves, A)
        # a search cut short at the budget counts the simulations it ran
        left = budget_s - (time.perf_counter() - t0)
        m = MCTS(net, A, S, choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
                 noise=lambda p, a, e: (1 - e) * p + e * noise)
        if blocks is not None:
            m.num_simulations = S if left > 60 else max(1, min(S, int(left / 0.3)))
        with torch.no_grad():
            m.run(st)
        sims += m.num_simulations
        legal = np.flatnonzero(gogame.invalid_moves(st) == 0)
        st = gogame.next_state(st, int(legal[moves % len(legal)]))
        moves += 1
        if gogame.game_ended(st):
            st = gogame.init_state(N)
    dt = time.perf_counter() - t0
    net_name = "batch-1 net" if blocks is None else f"{blocks}-block residual net (fp32), batch 1"
    return {"value": sims / dt, "unit": "sims/s", "cores": threads, "kind": "port",
            "sample": f"{moves} moves, {sims} sims, {N}x{N}, one game, {threads} thread(s), {dt:.1f} s "
                      f"(oracle MCTS + torch-CPU {net_name}; host has {os.cpu_count()} cpus)"}


def cpu_share(cgroup_cpu_max="/sys/fs/cgroup/cpu.max"):
    """(cores, source): the CPU share this process may use for the baseline --
    the cgroup's CPU quota if one is set, else the per-GPU share the GPU box
    exports as OMP_NUM_THREADS (16 per GPU; the box's affinity mask and
    os.cpu_count() show the whole machine), else the affinity mask
    (scripts/cpu_scaling.py -> profiles/r6_cpu_scaling.json: what the box
    reports and how the baseline scales past the share)."""
    try:
        with open(cgroup_cpu_max) as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period))), f"cgroup cpu.max {quota} {period}"
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) <= aff:
        return int(omp), f"OMP_NUM_THREADS={omp} (the box's per-GPU CPU share; affinity mask {aff} cpus)"
    return aff, f"affinity mask ({aff} cpus)"


def _cpu_worker(a):
    return cpu_baseline(*a)


def _cpu_worker_threads(a):
    return cpu_baseline(*a[:4], blocks=a[4], threads=a[5])


def cpu_baseline_procs(N, C, S, budget_s, procs, blocks=None):
    """P independent single-thread oracle processes (the
    reference's own parallelism is one game per process), sims/s summed.
    Must run before this process touches the GPU (spawned children)."""
    import multiprocessing as mp
    if procs <= 1:
        return cpu_baseline(N, C, S, budget_s, blocks)
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(N, C, S, budget_s, blocks)] * procs)
    # BASELINE.md's other CPU row: ONE process using every thread of the
    # share (the reference run as-is: one game, torch's intra-op threads)
    with mp.get_context("spawn").Pool(1) as pool:
        one = pool.map(_cpu_worker_threads, [(N, C, S, budget_s / 2, blocks, procs)])[0]
    total = sum(r["value"] for r in res)
    return {"value": total, "unit": "sims/s", "cores": procs, "kind": "port",
            "single_core_value": res[0]["value"],
            "one_process_all_threads": {"value": one["value"], "threads": procs, "sample": one["sample"]},
            "sample": f"{procs} processes x 1 thread, each one {N}x{N} game at {S} sims/move for "
                      f"{budget_s:.0f} s (oracle MCTS + torch-CPU batch-1 net; host has {os.cpu_count()} cpus)"}


# MI355X peaks (MI355X_MICROARCH.md): HBM 8 TB/s; fp32 MFMA 157.3 TF/s; VALU
# issue 2 wave-instructions / clk / CU (4 SIMD-32, a wave64 instruction takes
# 2 cycles); LDS 128-256 B/clk/CU (the LDS array: one lane group per cycle).
PEAK_HBM_GBPS = 8000.0
PEAK_FP32_MFMA_TFLOPS = 157.3
CUS, PEAK_CLK_GHZ = 256, 2.4


def pmc_summary(workload, dynamics, moves_per_launch, n_gpus=1, kernel="k_selfplay_move"):
    """Per-launch PMC means of k_selfplay_move from rocprofv3 passes of this
    same bench command (scripts/pmc.sh -> profiles/<tag>_pmc.json);
    only a profile of the same workload, launch structure and GPU count
    counts (the passes are 1-GPU runs: an N > 1 line gets none)."""
    import glob
    for path in [os.path.join(ROOT, "profiles", "latest_pmc.json")] + \
            sorted(glob.glob(os.path.join(ROOT, "profiles", "latest_pmc_*.json"))):
        p = json.load(open(path))
        if (p.get("workload") == workload and p.get("dynamics") == dynamics
                and p.get("moves_per_launch", 1) == moves_per_launch and p.get("n_gpus", 1) == n_gpus
                and kernel in p.get("kernel", "k_selfplay_move")):
            return p
    return None


def phases_summary(workload, moves_per_launch):
    """Per-phase shares of an epoch (select / expand / conv /
    replay / root / board / representation) and the epoch's tail, from the
    -DMZGO_STAMPS build of the same workload (scripts/phases.py ->
    profiles/<tag>_phases.json; in the timed kernel no stamp executes)."""
    path = os.path.join(ROOT, "profiles", "latest_phases.json")
    if moves_per_launch != 0 or not os.path.exists(path):
        return None
    p = json.load(open(path))
    if p.get("workload") != workload:
        return None
    out = {"shares": {k: round(v, 4) for k, v in p["shares"].items()},
           "tail_idle_cu_share": round(p["tail"]["idle_cu_share"], 4),
           "source": f"profiles/{p['tag']}_phases.json"}
    th = p.get("tail_helpers")
    if th:
        # ended games' workgroups computing running games' parent convs count as busy
        out["tail_idle_cu_share_with_helpers"] = round(th["idle_cu_share_with_helpers"], 4)
        out["tail_convs_share"] = round(p["engine_counters"]["tail_convs"] /
                                        max(1, p["engine_counters"]["dynamics_convs"]), 4)
    sd = p.get("slowest_decile")
    if sd:
        # the epoch's slowest games against the median decile, per phase (the tail's make-up)
        out["slowest_decile_vs_median"] = {k: round(v / max(sd["cycles_median_decile"][k], 1.0), 3)
                                           for k, v in sd["cycles_slowest"].items()}
        out["moves_per_game"] = {"slowest_decile": sd["moves_slowest"], "all": sd["moves_all"]}
    return out


def roofline(N, C, S, G, counts, avg_kern_s, dynamics, workload, moves_per_launch, n_gpus=1,
             kernel="k_selfplay_move"):
    """Roofline of the dominant kernel, per launch: k_selfplay_move (the
    game-per-workgroup launch) or, in the move-parallel epoch, k_search_queue
    (every search of the launch; the boards launch before it records and
    steps the boards and is timed beside it).

    Executed MFMA work: the dynamics convs the searches ran (Winograd GEMMs at
    9x9 / 19x19) + the representation per move.  HBM: the factored algorithm's
    own bytes (E[a] rows are an L2-resident table and are not charged).  The
    PMC counters (when profiles/latest_pmc.json is of this workload) give the
    issue-side units: VALU wave-instructions and LDS-array cycles per launch
    against their per-CU peaks at the measured clock.  ``bound`` is the unit
    with the largest fraction."""
    A, CELLS = N * N + 1, N * N
    L = counts["launches"]
    sims_l, moves_l, convs_l = counts["sims"] / L, counts["moves"] / L, counts["convs"] / L
    ct = (CELLS + 15) // 16
    mfma_l = 2048 * (convs_l * mfma_per_conv(N, C, C) + moves_l * (
        9 * 2 * 4 * ct + mfma_per_conv(N, 64, 64) + mfma_per_conv(N, 64, C)))
    mfma_tf = mfma_l / avg_kern_s / 1e12
    CS = (CELLS + 15) // 16 * 16
    if dynamics == "factored":
        # per prior row formed (engine counter: eager expansions, and lazily
        # expanded nodes a select reached -- the lazy policy head writes no row
        # for the others) the node's prior and child rows; per conv its input
        # read (the parent's Y, or the root latent: the rebuilt latent is
        # formed inside the input transform, never stored) and its Y written;
        # per move the representation's three conv outputs (64, 64, C channels)
        # written and read back, and the record (planes, policy, scalars)
        rows_l = counts.get("rows", counts["sims"]) / L
        hbm_l = (rows_l * 2 * A * 4 + convs_l * 2 * CELLS * C * 4
                 + moves_l * (2 * (128 + C) * CS * 4 + 2 * CELLS + A * 8 + 32))
    else:
        hbm_l = sims_l * (2 * C * CS * 4 + A * 4) + moves_l * ((6 * CELLS + 2 * C * CS) * 4 + A * 8)
    units = {
        "mfma": {"achieved": mfma_tf, "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                 "frac": mfma_tf / PEAK_FP32_MFMA_TFLOPS, "per_launch": mfma_l,
                 "what": "executed v_mfma_f32_16x16x4_f32 FLOPs (parent convs + representation)"},
        "hbm": {"achieved": hbm_l / avg_kern_s / 1e9, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                "frac": hbm_l / avg_kern_s / 1e9 / PEAK_HBM_GBPS, "per_launch": hbm_l,
                "what": "algorithmic HBM bytes of the factored search (E[a] table and weights L2-resident, "
                        "not charged; a parent's Y read from the LDS copy still charged)"},
    }
    pmc = pmc_summary(workload, dynamics, moves_per_launch, n_gpus, kernel)
    traffic = None
    if pmc is not None:
        c = pmc["counters"]
        dur = pmc["avg_duration_ms"] / 1e3
        clk = c["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9 if "GRBM_GUI_ACTIVE" in c else PEAK_CLK_GHZ
        clk = min(clk, PEAK_CLK_GHZ)
        if "SQ_INSTS_VALU" in c:
            peak = CUS * 2 * clk * 1e9          # wave-instructions / s
            ach = c["SQ_INSTS_VALU"] / dur
            units["valu"] = {"achieved": ach / 1e12, "peak": peak / 1e12, "unit": "Twave-instr/s",
                             "frac": ach / peak, "per_launch": c["SQ_INSTS_VALU"],
                             "what": "VALU wave-instructions issued (SQ_INSTS_VALU, MFMA excluded)"}
        if "SQ_LDS_IDX_ACTIVE" in c:
            peak = CUS * clk * 1e9              # LDS-array cycles / s
            ach = c["SQ_LDS_IDX_ACTIVE"] / dur
            units["lds"] = {"achieved": ach / 1e12, "peak": peak / 1e12, "unit": "Tcycles/s",
                            "frac": ach / peak, "per_launch": c["SQ_LDS_IDX_ACTIVE"],
                            "what": "LDS-array busy cycles (SQ_LDS_IDX_ACTIVE) per CU-cycle"}
        if "hbm_bytes_per_launch" in pmc:
            traffic = pmc["hbm_bytes_per_launch"]
        units["pmc_source"] = f"profiles/{pmc['tag']}_pmc.json"
        units["clock_GHz"] = clk
    bound = max((k for k in ("mfma", "hbm", "valu", "lds") if k in units), key=lambda k: units[k]["frac"])
    u = units[bound]
    return {"bound": bound, "kernel": kernel, "achieved": u["achieved"], "peak": u["peak"],
            "unit": u["unit"], "frac": u["frac"], "traffic": traffic,
            "avg_launch_ms": avg_kern_s * 1e3, "sims_per_launch": sims_l,
            "dynamics_convs_per_move": convs_l / max(moves_l, 1e-9),
            "prior_rows_per_move": counts.get("rows", counts["sims"]) / L / max(moves_l, 1e-9), "units": units,
            "algorithm": "factored dynamics (conv once per parent, children relu(Y + E[a])), batched + "
                         "replayed expansions" if dynamics == "factored" else
                         "a Winograd / implicit-GEMM dynamics conv per simulation"}


PEAK_BF16_MFMA_TFLOPS = 2500.0   # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def tower_roofline(N, C, blocks, G, sims, tower_ms, board_towers, evaluated):
    """Config 5's dominant kernel: the tower conv (one 3x3 conv of a batch of
    boards, bf16 MFMA).  Algorithmic FLOPs per board and conv = 2 x N^2 x 9 x
    C^2 (the conv as the network defines it; the kernel also multiplies the
    16-row tiles' pad rows: executed x 16*ceil(N^2/16) / N^2).  The timed
    towers (HIP events on the launch stream around each batched step's tower,
    or every 16th one-leaf step's) covered ``board_towers`` boards x L convs in
    ``tower_ms``, so achieved = board_towers x L x FLOP per board-conv / time
    (inter-launch gaps included).  ``evaluated`` = towers run (the engine's
    counter, speculative entries that were dropped included) over ``sims``."""
    L = 2 * blocks + 1
    per_bt_s = tower_ms / 1e3 / max(board_towers, 1)      # one board through the whole tower
    alg = 2 * N * N * 9 * C * C
    exe = 2 * 16 * ((N * N + 15) // 16) * 9 * C * C
    ach = alg * L / per_bt_s / 1e12
    batched = os.environ.get("MZGO_TOWER_BATCH", "0") != "0"
    chain = not batched and os.environ.get("MZGO_TCONV_CHAIN") != "0" and G * (C // 64) <= 256
    kname = "k_tconv_chain" if chain else "k_tconv_ks"
    out = {"bound": "mfma", "kernel": f"{kname}<{N}>", "achieved": ach, "peak": PEAK_BF16_MFMA_TFLOPS,
           "unit": "TFLOP/s", "frac": ach / PEAK_BF16_MFMA_TFLOPS, "traffic": None,
           "us_per_board_conv": per_bt_s / L * 1e6, "us_per_64_board_conv": per_bt_s / L * 64e6,
           "board_towers_timed": board_towers, "convs_per_tower": L,
           "flops_per_board_conv": alg, "executed_flops_per_board_conv": exe,
           "mfma_executed_tflops": exe * L / per_bt_s / 1e12,
           "towers_per_simulation": evaluated / max(sims, 1),
           # one leaf per game per step: a conv launch (a chain launch's layer) covers G boards
           "avg_launch_ms": per_bt_s / L * G * 1e3, "boards_per_launch": G, "flops_per_launch": alg * G,
           "steps": "batched (k_tbatch: root children + speculative leaf batches)" if batched else "one leaf per game",
           "what": "algorithmic conv FLOPs (2 N^2 9 C^2 per board and conv) x boards x L / the timed towers' "
                   "HIP-event spans (gaps included)"}
    path = os.path.join(ROOT, "profiles", "latest_tower_pmc.json")
    if os.path.exists(path):
        p = json.load(open(path))
        if p.get("workload") == f"{N}x{N}/C{C}/B{blocks}/G{G}" and ("chain" in p.get("kernel", "")) == chain:
            per = L if chain else 1                     # (the chain's counters cover L convs)
            out["traffic"] = p.get("hbm_bytes_per_launch") / per if p.get("hbm_bytes_per_launch") else None
            out["traffic_per"] = "conv launch (a chain launch's counters / its L convs)"
            out["pmc_source"] = f"profiles/{p['tag']}_pmc.json"
            out["pmc"] = p.get("derived")
            clk = (p.get("derived") or {}).get("in_kernel_clock_GHz")
            if clk:
                # the chip holds ~2.2 GHz under this kernel's bf16 MFMA load:
                # the fraction of the dense peak at the clock it actually runs
                out["frac_at_in_kernel_clock"] = ach / (PEAK_BF16_MFMA_TFLOPS * clk / 2.4)
    pw = os.path.join(ROOT, "profiles", "r3_power_clock.json")
    if os.path.exists(pw):
        summ = json.load(open(pw)).get("summary", {})
        for k, v in summ.items():
            if k.startswith("config 5"):
                out["power"] = dict(v, source="profiles/r3_power_clock.json (rocm-smi during the bench; cap 1400 W)")
    return out


def tower_main(args, world, rank, local, cpu_ref):
    """BASELINE config 5: 19x19, 20-block residual nets (C=256), 1600
    simulations per move, 64 games per GPU (mzgo.ResMuZeroNet on the tower
    engine).  A step = one move of every game (1600 simulations each); whole
    games (up to 361 moves) are out of a bench's time budget at this size."""
    import mzgo
    N, C, S, G, B = args.board_size, args.latent_dim, args.sims, args.games, args.blocks
    A = N * N + 1
    net = mzgo.ResMuZeroNet(C, A, B).to(f"cuda:{local}").eval()
    if rank == 0:
        net.load_state_dict(mzgo.deterministic_res_state_dict(C, A, B, 0))
    if world > 1:
        from mzgo import distributed as mdist
        mdist.broadcast_weights(net)
    planes = None
    live = None
    if args.start_move > 0:
        # mid-game (untimed): every game fast-forwarded to move ``start_move`` by
        # self-play at 8 simulations per move on a second engine of the same
        # network, its boards then loaded into the timed engine's slots.  A
        # game that ended during the fast-forward (two passes) is not loaded:
        # its slot plays from the empty board (games_live_at_start counts the
        # others) -- the board load carries the position, not a finished game
        ff = mzgo.SelfPlay(net, G, 8, seed=4321, game_base=rank * G)
        ff.reset(epoch=0)
        ff.move(args.start_move)
        planes = ff.engine.board_planes().cpu().numpy()
        live = [ff.engine.record(g)["status"] == 0 for g in range(G)]
        del ff
        torch.cuda.empty_cache()
    sp = mzgo.SelfPlay(net, G, S, seed=1234, game_base=rank * G)
    eng = sp.engine
    sp.reset(epoch=0)
    if planes is not None:
        for g in range(G):
            if live[g]:
                eng.board_set(g, planes[g])
    for _ in range(args.warmup):
        sp.move()
    torch.cuda.synchronize()
    eng.tower_timing(True)
    c0 = eng.counters()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sp.move(args.moves_per_step)
    if world > 1:
        from mzgo import distributed as mdist
        mdist.gather_packed(mdist.pack_engine(eng), to_host=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    tower_ms, towers = eng.tower_timing(False)
    c1 = eng.counters()
    sims = c1["simulations"] - c0["simulations"]
    moves = c1["moves"] - c0["moves"]
    evaluated = c1["dynamics_convs"] - c0["dynamics_convs"]      # tower engines: towers evaluated
    sims_local = sims
    if world > 1:
        t = torch.tensor([dt, float(sims), float(moves)], dtype=torch.float64,
                         device=f"cuda:{local}" if dist.get_backend() == "nccl" else "cpu")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, sims, moves = tmax[0].item(), t[1].item(), t[2].item()
    if rank == 0:
        workload = f"{N}x{N} Go self-play, {B}-block residual nets (C={C}), {G} parallel games/GPU, {S} sims/move"
        mps = args.moves_per_step
        roof = tower_roofline(N, C, B, G, sims_local, tower_ms, towers, evaluated)
        # the towers' share of the step: timed tower spans / wall time (batched
        # steps time every tower; one-leaf steps every 16th, scaled up)
        roof["share_of_step"] = (tower_ms / 1e3 * (1.0 if os.environ.get("MZGO_TOWER_BATCH", "0") != "0" else 16.0)) / dt
        out = {
            "metric": f"MCTS simulations/sec (whole node) + self-play moves/sec, {N}x{N} Go, {B}-block residual "
                      f"nets, {S} sims/move (BASELINE config 5)",
            "value": sims / dt, "unit": "sims/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (deterministic random-init weights, self-play from empty boards)",
            "moves_per_s": moves / dt,
            "config": {"workload": workload, "step": (f"{mps} consecutive moves" if mps > 1 else "one move")
                                                     + f" of {G} games/GPU ({S} simulations each; "
                                                     f"{2 * B + 1} convs per simulation)"
                                                     + (f", from move {args.start_move}" if args.start_move else ""),
                       "moves_per_step": mps,
                       "board_size": N, "latent_dim": C, "res_blocks": B, "games_per_gpu": G,
                       "sims_per_move": S, "parallelism": f"game-sharded x{world}", "compat": "reference",
                       "precision": "bf16 MFMA operands, fp32 accumulation, bf16 activations",
                       "start_move": args.start_move,
                       "stones_at_start": None if planes is None else
                       float(sum((planes[g, 0] + planes[g, 1]).sum() for g in range(G) if live[g])
                             / max(sum(live), 1)),
                       "games_live_at_start": None if live is None else int(sum(live))},
            "roofline": roof,
        }
        if cpu_ref is not None:
            out["cpu_baseline"] = cpu_ref
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def refill_main(args, net, world, rank, local, cpu_ref):
    """Refill configuration (the epoch tail): R engines of G game
    slots each, engine r on HIP stream r; step i plays one whole epoch of G
    games on engine i % R.  Kernels on different streams run concurrently, so
    the workgroups of epoch i + 1 start on the CUs that epoch i's finished
    games free (one game workgroup fills a CU's LDS), instead of those CUs
    idling until epoch i's slowest game ends; stream order keeps each
    engine's epochs sequential.  Same games, kernel and records as the
    headline (game ids (rank * R + r) * G + slot, epoch keys distinct); value
    = all simulations / wall time."""
    import mzgo
    N, C, S, G, R = args.board_size, args.latent_dim, args.sims, args.games, args.refill
    # the epoch tail's helpers keep a finished game's workgroup on its CU (it
    # serves running games' convs), which is exactly the CU the next engine's
    # epoch would start on: refill and tail helpers exclude each other
    # (same-call A/B: 106.2 M with them off, 95.6 M on)
    os.environ["MZGO_TAIL_HELPERS"] = "0"
    # refill is the game-per-workgroup launch's answer to the epoch tail (the
    # move-parallel epoch is the other): its epochs are k_selfplay_move
    os.environ["MZGO_MOVE_PARALLEL"] = "0"
    sps = [mzgo.SelfPlay(net, G, S, seed=1234, game_base=(rank * R + r) * G, dynamics=args.dynamics)
           for r in range(R)]
    M = sps[0].max_moves
    streams = [torch.cuda.Stream() for _ in range(R)]
    ev = []
    gathers = []
    step_no = [0]

    def one_epoch(record):
        i = step_no[0]
        r = i % R
        with torch.cuda.stream(streams[r]):
            if record:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(streams[r])
            sps[r].reset(epoch=i)
            sps[r].move(M)
            if record:
                b.record(streams[r])
                ev.append((a, b))
                if world > 1:
                    # every timed epoch's records to rank 0 (RCCL, ordered after this stream's epoch)
                    from mzgo import distributed as mdist
                    gathers.append(mdist.gather_packed(mdist.pack_engine(sps[r].engine), async_op=True))
        step_no[0] += 1

    for _ in range(max(args.warmup, R)):
        one_epoch(False)
    torch.cuda.synchronize()
    c0 = [sp.engine.counters() for sp in sps]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_epoch(True)
    for work, _ in gathers:
        work.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    c1 = [sp.engine.counters() for sp in sps]
    sims = sum(b["simulations"] - a["simulations"] for a, b in zip(c0, c1))
    moves = sum(b["moves"] - a["moves"] for a, b in zip(c0, c1))
    convs = sum(b["dynamics_convs"] - a["dynamics_convs"] for a, b in zip(c0, c1))
    rows = sum(b["prior_rows"] - a["prior_rows"] for a, b in zip(c0, c1))
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    if world > 1:
        t = torch.tensor([dt, float(sims), float(moves)], dtype=torch.float64,
                         device=f"cuda:{local}" if dist.get_backend() == "nccl" else "cpu")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, sims, moves = tmax[0].item(), t[1].item(), t[2].item()
    if rank == 0:
        workload = f"{N}x{N} Go self-play, {G} parallel games/GPU, {S} sims/move"
        counts = dict(launches=len(kern_ms), sims=sims / world, moves=moves / world, convs=convs, rows=rows)
        # R engines' epochs overlap on R streams, so an epoch's own event span
        # includes the time it shares the GPU: the roofline is taken on wall
        # time instead (all epochs' work / dt, i.e. dt / epochs per launch)
        roof = roofline(N, C, S, G, counts, dt / len(kern_ms), args.dynamics, workload + f", refill {R}", 0, world)
        roof["avg_launch_ms_basis"] = "wall time / epochs (overlapping streams)"
        roof["epoch_event_span_ms"] = sum(kern_ms) / len(kern_ms)
        out = {
            "metric": f"MCTS simulations/sec (whole node) + self-play moves/sec, {N}x{N} Go, {S} sims/move "
                      f"(refill configuration)",
            "value": sims / dt, "unit": "sims/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (deterministic random-init weights, self-play from empty boards)",
            "moves_per_s": moves / dt,
            "config": {"workload": workload, "step": f"one whole self-play epoch of {G} games/GPU, epochs on "
                                                     f"{R} engines / HIP streams overlapping (refill)",
                       "board_size": N, "latent_dim": C, "games_per_gpu": G, "sims_per_move": S,
                       "parallelism": f"game-sharded x{world}", "compat": "reference", "dynamics": args.dynamics,
                       "refill": R},
            "roofline": roof,
        }
        if cpu_ref is not None:
            out["cpu_baseline"] = cpu_ref
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def _launch_module():
    """mzgo/launch.py loaded by file path (standard library only): the parent
    of ``--gpus N`` never imports the mzgo package, so it never loads
    libmzgo.so."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_mzgo_launch", os.path.join(ROOT, "muzero-go_amd", "mzgo",
                                                                             "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2, choices=[2, 5],
                    help="2: 9x9 / 256 games / 200 sims (the headline, BASELINE configs[1]); "
                         "5: 19x19 / 20-block residual nets / 1600 sims / 64 games (BASELINE configs[4])")
    ap.add_argument("--blocks", type=int, default=20, help="residual blocks (config 5)")
    ap.add_argument("--moves-per-step", type=int, default=1,
                    help="config 5: a step = this many consecutive moves of every game (a game segment)")
    ap.add_argument("--start-move", type=int, default=0,
                    help="config 5: time moves from this move on (every game fast-forwarded there first by "
                         "untimed self-play at 8 simulations per move)")
    ap.add_argument("--gpus", type=int, default=1)
    # defaults per config (2: 10 / 1 / 9 / 256 / 200 / 96; 5: 2 / 1 / 19 / 64 / 1600 / 256), filled below
    # only where the option is not given
    ap.add_argument("--steps", type=int, default=None, help="timed steps (config 2: whole self-play epochs)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps")
    ap.add_argument("--board-size", type=int, default=None)
    ap.add_argument("--games", type=int, default=None, help="parallel games per GPU")
    ap.add_argument("--sims", type=int, default=None)
    ap.add_argument("--latent-dim", type=int, default=None)
    ap.add_argument("--dynamics", choices=["factored", "direct"], default="factored",
                    help="factored: one conv per parent, children as relu(Y + E[a]) (mzgo_expand.hpp); "
                         "direct: a dynamics conv per simulation, as the reference computes it")
    ap.add_argument("--moves-per-launch", type=int, default=0,
                    help="moves of every game per k_selfplay_move launch (0 = whole games)")
    ap.add_argument("--refill", type=int, default=0,
                    help="R >= 2: a separate configuration (not the headline): R engines of G slots on R HIP "
                         "streams play consecutive epochs, so CUs a finished game frees start the next epoch's "
                         "games instead of idling while the epoch's slowest games finish (the epoch tail)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--cpu-procs", type=int, default=None,
                    help="oracle processes for cpu_baseline (default: this host's CPU share, cpu_share())")
    args = ap.parse_args()
    defaults = {2: dict(board_size=9, games=256, sims=200, latent_dim=96, steps=20, warmup=3),
                5: dict(board_size=19, games=64, sims=1600, latent_dim=256, steps=2, warmup=1)}[args.config]
    for k, v in defaults.items():
        if getattr(args, k) is None:
            setattr(args, k, v)

    share, share_src = cpu_share()
    if args.cpu_procs is None:
        args.cpu_procs = share
    blocks = args.blocks if args.config == 5 else None
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # --gpus N without a launcher: N fresh rank processes (RANK / LOCAL_RANK /
        # WORLD_SIZE / MASTER_* as torch.distributed.run sets them), started
        # before anything here loads libmzgo.so or touches a GPU; rank 0 prints
        # the line, this process exits with the ranks' status.  The CPU
        # baseline runs here first (this process never touches a GPU) and
        # reaches rank 0's line through the environment.
        if not args.no_cpu_baseline:
            ref = cpu_baseline_procs(args.board_size, args.latent_dim, args.sims, args.cpu_budget, args.cpu_procs,
                                     blocks)
            ref["measured_in"] = "launcher process, before the ranks started (no GPU work running)"
            ref["cores_source"] = share_src if args.cpu_procs == share else "--cpu-procs"
            os.environ["MZGO_CPU_BASELINE"] = json.dumps(ref)
        sys.exit(_launch_module().spawn_ranks(
            args.gpus, [sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={world}: run `bench.py --gpus N` alone (it starts N ranks) "
                 f"or under torch.distributed.run with --nproc-per-node N")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N>1 path on a one-GPU box (never the driver's runs):
    # MZGO_SHARE_DEVICE=1 puts every rank on cuda:0, MZGO_DIST_BACKEND=gloo
    # replaces RCCL (which refuses two ranks on one GPU)
    backend = os.environ.get("MZGO_DIST_BACKEND", "nccl")
    if os.environ.get("MZGO_SHARE_DEVICE") == "1":
        local = 0
    cpu_ref = None
    if rank == 0 and not args.no_cpu_baseline:
        if "MZGO_CPU_BASELINE" in os.environ:        # (bench.py --gpus N's own launcher measured it)
            cpu_ref = json.loads(os.environ["MZGO_CPU_BASELINE"])
        else:
            # before the GPU is initialised (the baseline spawns worker
            # processes); under torch.distributed.run the other ranks wait for
            # rank 0 in init_process_group meanwhile
            cpu_ref = cpu_baseline_procs(args.board_size, args.latent_dim, args.sims, args.cpu_budget,
                                         args.cpu_procs, blocks)
            cpu_ref["cores_source"] = share_src if args.cpu_procs == share else "--cpu-procs"
            if world > 1:
                cpu_ref["measured_in"] = "rank 0, before GPU initialisation (the other ranks waiting)"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if args.config == 5:
        tower_main(args, world, rank, local, cpu_ref)
        return

    import mzgo
    from mzgo import distributed as mdist

    N, C, S, G = args.board_size, args.latent_dim, args.sims, args.games
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).to(f"cuda:{local}").eval()
    if rank == 0:
        net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    if world > 1:
        mdist.broadcast_weights(net)                      # one RCCL broadcast, untimed
    if args.refill >= 2:
        refill_main(args, net, world, rank, local, cpu_ref)
        return
    sp = mzgo.SelfPlay(net, G, S, seed=1234, game_base=rank * G, dynamics=args.dynamics)
    eng = sp.engine
    M = sp.max_moves
    stream = torch.cuda.current_stream()

    # One step = one whole self-play epoch: every
    # slot starts a new game from the empty board and plays until it ends
    # (double pass, or the N*N move cap).  ``--moves-per-launch`` moves of
    # every game run in one k_selfplay_move launch (default: the whole game,
    # so each CU plays its game's moves back to back); the epoch index keys
    # the RNG, so every epoch plays new games.
    epoch_no = 0
    per = M if args.moves_per_launch <= 0 else args.moves_per_launch
    chunks = [min(per, M - j) for j in range(0, M, per)]

    def one_epoch(evs=None):
        nonlocal epoch_no
        sp.reset(epoch=epoch_no)
        for j, k in enumerate(chunks):
            if evs is not None:
                evs[j][0].record(stream)
            sp.move(k)
            if evs is not None:
                evs[j][1].record(stream)
        epoch_no += 1

    for _ in range(args.warmup):
        one_epoch()
    torch.cuda.synchronize()
    c0 = eng.counters()

    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in chunks]
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # The trajectory gather of config 3 (RCCL, the only collective on the
    # data path): every timed epoch's records are packed on the device into
    # their own slice of a rank-local HBM staging buffer (a D2D copy on the
    # launch stream, 17 MB per epoch at 9x9 / 256 games), and the staged
    # epochs go to rank 0's HBM in ONE gather at the end of the timed loop.
    # A gather per epoch would share the chip with the next epoch: RCCL moves
    # data with kernels, an epoch puts one workgroup on every CU at ~159 KiB
    # of LDS, and a collective kernel resident while it waits for the
    # slowest rank displaces a game's workgroup for that long -- measured
    # with a stand-in kernel waiting 20 ms: +11 ms per 49 ms epoch overlapped,
    # +2.4 ms even when gated until the next epoch is resident
    # (scripts/rccl_standin.py).  One large collective at the end
    # never overlaps an epoch, and 288 GB of HBM holds the staging easily.
    gathers, staged = [], None
    if world > 1:
        per_epoch = mdist.pack_engine(eng).numel()
        staged = torch.empty(args.steps * per_epoch, dtype=torch.uint8, device=f"cuda:{local}")
        torch.cuda.synchronize()

    eng.launch_timing(True)        # move-parallel epochs: HIP events around both launches
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_epoch(ev[i])
        if world > 1:
            mdist.pack_engine(eng, out=staged[i * per_epoch:(i + 1) * per_epoch])
    if world > 1:
        gathers.append(mdist.gather_packed(staged, async_op=True))
    for work, _ in gathers:
        work.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    c1 = eng.counters()
    sims = c1["simulations"] - c0["simulations"]
    moves = c1["moves"] - c0["moves"]
    # launch durations (HIP events on the launch stream), all launches of every
    # timed epoch: k_selfplay_move, or in the move-parallel epoch (compat
    # "reference") the boards launch + k_search_queue, whose own
    # durations the engine's events give
    kern_ms = [a.elapsed_time(b) for e in ev for a, b in e]
    boards_ms, queue_ms = eng.launch_timing(False)
    launches = len(kern_ms)
    kernel = "k_search_queue" if queue_ms else "k_selfplay_move"
    if queue_ms:
        assert len(queue_ms) == launches, (len(queue_ms), launches)
        avg_kern_s = sum(queue_ms) / launches / 1e3
    else:
        avg_kern_s = sum(kern_ms) / launches / 1e3

    if world > 1:
        t = torch.tensor([dt, float(sims), float(moves)], dtype=torch.float64,
                         device=f"cuda:{local}" if dist.get_backend() == "nccl" else "cpu")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, sims, moves = tmax[0].item(), t[1].item(), t[2].item()

    if rank == 0:
        workload = f"{N}x{N} Go self-play, {G} parallel games/GPU, {S} sims/move"
        counts = dict(launches=launches, sims=sims / world, moves=moves / world,
                      convs=(c1["dynamics_convs"] - c0["dynamics_convs"]),
                      rows=(c1["prior_rows"] - c0["prior_rows"]))
        roof = roofline(N, C, S, G, counts, avg_kern_s, args.dynamics, workload, args.moves_per_launch, world,
                        kernel)
        if queue_ms:
            roof["boards_launch_ms"] = sum(boards_ms) / launches
            roof["epoch_launches_ms"] = sum(kern_ms) / launches
        out = {
            "metric": f"MCTS simulations/sec (whole node) + self-play moves/sec, {N}x{N} Go, {S} sims/move",
            "value": sims / dt,
            "unit": "sims/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (deterministic random-init weights, self-play from empty boards)",
            "moves_per_s": moves / dt,
            "config": {"workload": workload, "step": f"one whole self-play epoch: {G} games/GPU from the "
                                                     f"empty board to their end ({len(chunks)} launch(es) "
                                                     f"of up to {per} moves)",
                       "board_size": N, "latent_dim": C, "games_per_gpu": G, "sims_per_move": S,
                       "parallelism": f"game-sharded x{world}", "compat": "reference",
                       "dynamics": args.dynamics,
                       "schedule": ("move-parallel: boards launch + k_search_queue (every move's search from "
                                    "one queue, one workgroup per CU)") if queue_ms else
                                   "game-per-workgroup k_selfplay_move"},
            "roofline": roof,
        }
        if world > 1:
            out["gather"] = {"collective": f"{dist.get_backend()} gather to rank 0", "count": len(gathers),
                             "epochs_per_gather": args.steps, "bytes_per_rank": int(staged.numel()),
                             "bytes_per_epoch_per_rank": int(per_epoch),
                             "schedule": "every timed epoch's records packed into a rank-local HBM staging slice; "
                                         "one gather of all of them at the end of the timed loop (inside it): no "
                                         "collective kernel shares the chip with an epoch"}
        # (the stamps build is profiled on one GPU: phase shares only on 1-GPU lines)
        # (the stamps build profiles the game-per-workgroup launch: MZGO_MOVE_PARALLEL=0 lines only)
        ph = phases_summary(workload, args.moves_per_launch) if (args.dynamics == "factored" and world == 1
                                                                 and not queue_ms) else None
        if ph is not None:
            out["phases"] = ph
        if cpu_ref is not None:
            out["cpu_baseline"] = cpu_ref
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
