"""Benchmark: MCTS simulations/sec + self-play moves/sec, 9x9 Go, 200 sims/move.

BASELINE.json's metric on configs[1]: 256 parallel self-play games per GPU,
200 simulations per move, the reference network (latent_dim 96) with
deterministic random-init weights, fp32.  One *step* = one self-play move of
every game on the GPU: one launch of the fused k_selfplay_move kernel
(observation record, representation + root priors, 200 simulations of
select / dynamics+prediction (MFMA) / expand / backup, action choice, board
step).  Games restart (new epoch) every max_moves steps, so any --steps works.

Multi-GPU (torchrun, one process per GPU): games are sharded by global id
(rank * G + slot); the only collective is the end-of-run RCCL gather of every
rank's game records to rank 0 (inside the timed region); scaling "weak".

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

FLOPS_PER_SIM_9x9 = None  # filled from the geometry below


def algorithmic_flops(N, C, S):
    """Per-simulation and per-move (root) FLOPs of the reference network.

    sim:  dynamics 3x3 conv 2*9*C*C*N^2 + three 1x1 heads 3*2*C*N^2 + embedding add C*N^2
    root: representation 2*9*N^2*(6*64 + 64*64 + 64*C) + two 1x1 heads 2*2*C*N^2
    (FCs and softmax are O(A) and omitted.)
    """
    cells = N * N
    sim = 2 * 9 * C * C * cells + 3 * 2 * C * cells + C * cells
    root = 2 * 9 * cells * (6 * 64 + 64 * 64 + 64 * C) + 2 * 2 * C * cells
    return sim, root


def algorithmic_bytes(N, C, G):
    """SURVEY.md §8(d)'s algorithmic bytes per simulation (fp32): parent latent
    read + child latent write 2*C*N^2*4, tree traffic at depth d = 2 (A child
    priors / ids / visits / value sums, 20 B each, + 12 B backup per level),
    the new node's priors A*4, and the weights amortised over G games."""
    A = N * N + 1
    return 2 * C * N * N * 4 + 2 * A * 20 + 2 * 12 + A * 4 + (9 * C * C + 3 * C + A * C) * 4 // G


def mfma_per_conv(N, cin, cout):
    """16x16x4 f32 MFMAs of one 3x3 conv of one board (Winograd at 9x9 / 19x19)."""
    if N == 9:
        return 20 * (cout // 16) * (cin // 4)
    if N == 19:
        return 5 * 20 * (cout // 16) * (cin // 4)
    return 9 * (cin // 4) * (cout // 16) * ((N * N + 15) // 16)


def cpu_baseline(N, C, S, budget_s=12.0):
    """The oracle (CPU restatement of self_play.py's MCTS, batch-1 torch net,
    object tree) timed on this host with one thread, on a bounded sample."""
    import numpy as np

    from oracle.mcts import MCTS
    from oracle.net import OracleNet
    from oracle.rng import SearchHooks, injected_noise
    from oracle.weights import deterministic_state_dict
    from oracle import gogame

    torch.set_num_threads(1)
    A = N * N + 1
    net = OracleNet(deterministic_state_dict(C, A, 0))
    st = gogame.init_state(N)
    sims, moves, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        hooks = SearchHooks(1234, 0, moves)
        noise = injected_noise(1234, 0, moves, A)
        m = MCTS(net, A, S, choice=lambda seq, sim: seq[hooks.choice_index(len(seq), sim)],
                 noise=lambda p, a, e: (1 - e) * p + e * noise)
        with torch.no_grad():
            m.run(st)
        sims += S
        legal = np.flatnonzero(gogame.invalid_moves(st) == 0)
        st = gogame.next_state(st, int(legal[moves % len(legal)]))
        moves += 1
        if gogame.game_ended(st):
            st = gogame.init_state(N)
    dt = time.perf_counter() - t0
    return {"value": sims / dt, "unit": "sims/s", "cores": 1, "kind": "port",
            "sample": f"{moves} moves x {S} sims, {N}x{N}, one game, 1 thread, {dt:.1f} s "
                      f"(oracle MCTS + torch-CPU batch-1 net; host has {os.cpu_count()} cpus)"}


def _cpu_worker(a):
    return cpu_baseline(*a)


def cpu_baseline_procs(N, C, S, budget_s, procs):
    """P independent single-thread oracle processes (the
    reference's own parallelism is one game per process), sims/s summed.
    Must run before this process touches the GPU (spawned children)."""
    import multiprocessing as mp
    if procs <= 1:
        return cpu_baseline(N, C, S, budget_s)
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(N, C, S, budget_s)] * procs)
    total = sum(r["value"] for r in res)
    return {"value": total, "unit": "sims/s", "cores": procs, "kind": "port",
            "single_core_value": res[0]["value"],
            "sample": f"{procs} processes x 1 thread, each one {N}x{N} game at {S} sims/move for "
                      f"{budget_s:.0f} s (oracle MCTS + torch-CPU batch-1 net; host has {os.cpu_count()} cpus)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--board-size", type=int, default=9)
    ap.add_argument("--games", type=int, default=256, help="parallel games per GPU")
    ap.add_argument("--sims", type=int, default=200)
    ap.add_argument("--latent-dim", type=int, default=96)
    ap.add_argument("--dynamics", choices=["factored", "direct"], default="factored",
                    help="factored: one conv per parent, children as relu(Y + E[a]) (mzgo_expand.hpp); "
                         "direct: a dynamics conv per simulation, as the reference computes it")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--cpu-procs", type=int, default=min(16, os.cpu_count() or 1),
                    help="oracle processes for cpu_baseline (the GPU box's CPU share is 16)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu_ref = None
    if world == 1 and not args.no_cpu_baseline:
        # before the GPU is initialised: the baseline spawns worker processes
        cpu_ref = cpu_baseline_procs(args.board_size, args.latent_dim, args.sims, args.cpu_budget, args.cpu_procs)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import mzgo

    N, C, S, G = args.board_size, args.latent_dim, args.sims, args.games
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).to(f"cuda:{local}").eval()
    if rank == 0:
        net.load_state_dict(mzgo.deterministic_state_dict(C, A, 0))
    if world > 1:
        from mzgo import distributed as mdist
        mdist.broadcast_weights(net)                      # one RCCL broadcast, untimed
    sp = mzgo.SelfPlay(net, G, S, seed=1234, game_base=rank * G, dynamics=args.dynamics)
    eng = sp.engine
    M = sp.max_moves
    stream = torch.cuda.current_stream()

    step_no = 0

    def one_step():
        nonlocal step_no
        if step_no % M == 0:
            sp.reset(epoch=step_no // M)
        sp.move()
        step_no += 1

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    c0 = eng.counters()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if step_no % M == 0:
            sp.reset(epoch=step_no // M)
        ev[i][0].record(stream)
        sp.move()
        ev[i][1].record(stream)
        step_no += 1
    if world > 1:
        # the trajectory gather of config 3: every rank's packed game records
        # to rank 0's HBM over RCCL (the only collective on the data path)
        from mzgo import distributed as mdist
        mdist.gather_packed(mdist.pack_engine(eng), to_host=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    c1 = eng.counters()
    sims = c1["simulations"] - c0["simulations"] if c1["simulations"] >= c0["simulations"] else c1["simulations"]
    moves = c1["moves"] - c0["moves"] if c1["moves"] >= c0["moves"] else c1["moves"]
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    avg_kern_s = sum(kern_ms) / len(kern_ms) / 1e3

    if world > 1:
        t = torch.tensor([dt, float(sims), float(moves)], dtype=torch.float64, device=f"cuda:{local}")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, sims, moves = tmax[0].item(), t[1].item(), t[2].item()

    if rank == 0:
        sim_f, root_f = algorithmic_flops(N, C, S)
        per_launch_moves = moves / world / args.steps
        per_launch_sims = sims / world / args.steps
        launch_flops = per_launch_moves * (S * sim_f + root_f)
        equiv_tflops = launch_flops / avg_kern_s / 1e12      # the reference formulation's FLOP rate
        convs = c1["dynamics_convs"] - c0["dynamics_convs"]
        ct = (N * N + 15) // 16
        # executed MFMA work: the dynamics convs the searches ran + the
        # representation (conv1 direct, conv2/conv3 latent convs) per move
        mfma_launch = 2048 * (convs / args.steps * mfma_per_conv(N, C, C) + per_launch_moves * (
            9 * 2 * 4 * ct + mfma_per_conv(N, 64, 64) + mfma_per_conv(N, 64, C)))
        mfma_exec = mfma_launch / avg_kern_s / 1e12
        peak_mfma = 157.3
        bytes_sim = algorithmic_bytes(N, C, G)
        gbps_8d = per_launch_sims * bytes_sim / avg_kern_s / 1e9
        peak_hbm = 8000.0
        if args.dynamics == "factored":
            # The factored algorithm's own HBM bytes: per simulation the child's
            # E[a] row (9 C f32) and its prior and child-id rows (2 A x 4 B); per
            # parent conv the rebuilt latent (written, read) and its Y (written,
            # read into LDS); per move the representation's input and latent and
            # the record.  (SURVEY §8(d)'s direct-formulation bytes and FLOPs per
            # simulation are reported beside it: the factored kernel runs past
            # both of those rooflines because it no longer does that work.)
            CS = (N * N + 15) // 16 * 16
            launch_convs = convs / args.steps
            fact_bytes = (per_launch_sims * (9 * C * 4 + 2 * A * 4)
                          + launch_convs * (2 * C * CS * 4 + 2 * N * N * C * 4)
                          + per_launch_moves * ((6 * N * N + 2 * C * CS) * 4 + 2 * N * N + A * 8 + 32))
            gbps = fact_bytes / avg_kern_s / 1e9
            roof = {"bound": "hbm", "kernel": "k_selfplay_move", "achieved": gbps, "peak": peak_hbm,
                    "unit": "GB/s", "frac": gbps / peak_hbm, "traffic": None,
                    "algorithmic_bytes_per_launch": fact_bytes, "sims_per_launch": per_launch_sims,
                    "avg_launch_ms": avg_kern_s * 1e3,
                    "survey_8d_bytes_per_sim": bytes_sim, "equiv_survey_8d_gbps": gbps_8d,
                    "equiv_direct_conv_tflops": equiv_tflops,
                    "equiv_direct_conv_frac_of_fp32_mfma": equiv_tflops / peak_mfma,
                    "dynamics_convs_per_move": convs / max(1.0, moves / world),
                    "mfma_executed": mfma_exec, "mfma_executed_frac": mfma_exec / peak_mfma,
                    "note": "not HBM-bound: batched expansions are VALU-bound, parent/representation convs fp32-MFMA-bound, the rest per-game latency; see DESIGN.md section 5",
                    "algorithm": "factored dynamics (conv once per parent, children relu(Y + E[a])), "
                                 "batched + replayed expansions"}
        else:
            roof = {"bound": "mfma", "kernel": "k_selfplay_move", "achieved": equiv_tflops,
                    "peak": peak_mfma, "unit": "TFLOP/s", "frac": equiv_tflops / peak_mfma, "traffic": None,
                    "flops_per_launch": launch_flops, "avg_launch_ms": avg_kern_s * 1e3,
                    # what the MFMA pipes actually execute (Winograd issues fewer
                    # MFMA FLOPs than the direct conv's algorithmic count)
                    "mfma_executed": mfma_exec, "mfma_executed_frac": mfma_exec / peak_mfma,
                    "algorithm": "winograd F(2,3)xF(3,3)" if N in (9, 19) else "direct implicit GEMM"}
        out = {
            "metric": "MCTS simulations/sec (whole node) + self-play moves/sec, 9x9 Go, 200 sims/move",
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
            "config": {"workload": f"{N}x{N} Go self-play, {G} parallel games/GPU, {S} sims/move",
                       "board_size": N, "latent_dim": C, "games_per_gpu": G, "sims_per_move": S,
                       "parallelism": f"game-sharded x{world}", "compat": "reference",
                       "dynamics": args.dynamics},
            "roofline": roof,
        }
        prof = os.path.join(ROOT, "profiles", "latest_summary.json")
        if os.path.exists(prof):
            p = json.load(open(prof))
            if (p.get("workload") == out["config"]["workload"] and "k_selfplay_move" in p.get("kernel", "")
                    and p.get("dynamics", "direct") == args.dynamics):
                # HBM bytes per launch from rocprofv3 PMC passes of this same command
                # (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; scripts/summarize_profile.py)
                out["roofline"]["traffic"] = p["hbm_bytes_per_launch"]
                out["roofline"]["traffic_source"] = f"profiles/{p['tag']}_summary.json"
        if cpu_ref is not None:
            out["cpu_baseline"] = cpu_ref
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
