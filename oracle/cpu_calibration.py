"""CPU-baseline calibration (TEST INFRASTRUCTURE ONLY; runs in the build
container, where /root/reference exists): SURVEY.md §8(d) asks to time the
restatement (oracle.mcts.MCTS, bench.py's cpu_baseline) against the real
reference MCTS.run on the same host and report the ratio, plus the
"1 process x all threads" row.  Writes profiles/cpu_calibration.json.

Usage: python -m oracle.cpu_calibration [budget_s]
"""
import json
import os
import sys
import time

import numpy as np
import torch

from oracle import gogame
from oracle.make_golden import _ref_net, import_reference
from oracle.mcts import MCTS
from oracle.net import OracleNet
from oracle.weights import deterministic_state_dict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _time(make_search, N, S, budget):
    st = gogame.init_state(N)
    sims, moves, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget:
        with torch.no_grad():
            make_search().run(st)
        sims += S
        legal = np.flatnonzero(gogame.invalid_moves(st) == 0)
        st = gogame.next_state(st, int(legal[moves % len(legal)]))
        moves += 1
        if gogame.game_ended(st):
            st = gogame.init_state(N)
    dt = time.perf_counter() - t0
    return sims / dt, moves, dt


def main(budget=20.0, N=9, S=200, C=96):
    sp = import_reference()
    A = N * N + 1
    sd = deterministic_state_dict(C, A, 0)
    ref_net = _ref_net(sp, sd, C, A)
    ora_net = OracleNet(sd)
    rows = {}
    for threads in (1, os.cpu_count()):
        torch.set_num_threads(threads)
        ref, rm, rdt = _time(lambda: sp.MCTS(ref_net, A, S), N, S, budget)
        ora, om, odt = _time(lambda: MCTS(ora_net, A, S), N, S, budget)
        rows[f"{threads}_thread"] = {
            "threads": threads, "reference_sims_per_s": ref, "oracle_sims_per_s": ora,
            "oracle_over_reference": ora / ref, "reference_moves": rm, "oracle_moves": om,
            "seconds": [rdt, odt]}
        print(threads, "thread(s): reference", round(ref, 1), "oracle", round(ora, 1), "ratio", round(ora / ref, 3))
    out = {"workload": f"{N}x{N}, {S} sims/move, latent_dim {C}, one game, batch-1 torch-CPU net",
           "host_cpus": os.cpu_count(), "budget_s_per_row": budget, "rows": rows,
           "note": "bench.py's cpu_baseline runs the oracle as P single-thread processes on the GPU box; "
                   "divide it by oracle_over_reference (1 thread) for the reference-equivalent rate"}
    with open(os.path.join(REPO, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 20.0)
