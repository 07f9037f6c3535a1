"""Does a collective's CU-resident kernel, issued between two epochs, delay
the next epoch?  (VERDICT r4 "what's weak" 5)

bench.py --gpus N overlaps each epoch's RCCL gather with the next epoch:
the gather is ordered after epoch i's kernel (and the record pack) on RCCL's
stream while epoch i + 1's whole-game launch is already queued on the launch
stream.  RCCL moves data with kernels; the epoch kernel puts one workgroup
on every CU at ~159 KiB of LDS.  If the collective's kernel is dispatched
first, the workgroups it displaces start late -- by the time it stays
resident, which on a peer rank is the inter-rank skew.

One GPU cannot run RCCL with two ranks, so a stand-in kernel
(tools/standin.hip: W workgroups of one wave with L KiB of LDS spinning for T
us) plays the collective: per epoch, the same command sequence as bench.py
(reset, whole-game move, record pack) on the launch stream, an event, and on
a second stream a wait on it and the stand-in.  Modes, alternating, same
process:
  none     -- no stand-in (the epoch alone)
  overlap  -- the stand-in as bench.py orders the gather (after epoch i, beside
              epoch i + 1's launch)
  ordered  -- the launch stream also waits for the stand-in before epoch
              i + 1 (the design that never overlaps: the gather's own time is
              then on the critical path)
  gated    -- bench.py's schedule: epoch i's stand-in issued after epoch
              i + 1's launch behind Engine.wait_started (it can take a CU only
              once all of epoch i + 1's workgroups are resident)
Per epoch: the launch stream's event span of reset + move (ms).

Usage (GPU box): python scripts/rccl_standin.py [W] [LDS_KB] [T_US] -> one JSON line
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import mzgo
    from mzgo import distributed as mdist
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    LKB = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    TUS = float(sys.argv[3]) if len(sys.argv) > 3 else 2000.0
    reps = int(os.environ.get("REPS", 4))
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libstandin.so"))
    lib.standin_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]
    N, C, S, G = 9, 96, 200, 256
    net = mzgo.MuZeroNet(C, N * N + 1).to("cuda").eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, N * N + 1, 0))
    sp = mzgo.SelfPlay(net, G, S, seed=1234)
    M = sp.max_moves
    a = torch.cuda.current_stream()
    b = torch.cuda.Stream()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    cycles = int(TUS * 100)                       # s_memrealtime: 100 MHz (MI355X_MICROARCH.md)
    def run(mode, k, base):
        # epochs base .. base + k - 1 (the RNG key): every mode plays the same games
        evs = []
        torch.cuda.synchronize()
        started = sp.engine.counters()["workgroups_started"]
        pend = None
        for i in range(k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(a)
            sp.reset(epoch=base + i)
            sp.move(M)
            e1.record(a)
            started += G
            mdist.pack_engine(sp.engine)          # the gather's input, as bench.py packs it
            if mode == "gated":
                # bench.py's schedule: epoch i - 1's stand-in after epoch i's launch, behind the gate
                if pend is not None:
                    b.wait_event(pend)
                    sp.engine.wait_started(started, b)
                    assert lib.standin_launch(W, LKB, cycles, ctypes.c_void_p(sink.data_ptr()),
                                              ctypes.c_void_p(b.cuda_stream)) == 0
                pend = torch.cuda.Event()
                pend.record(a)
            elif mode != "none":
                done = torch.cuda.Event()
                done.record(a)
                b.wait_event(done)
                assert lib.standin_launch(W, LKB, cycles, ctypes.c_void_p(sink.data_ptr()),
                                          ctypes.c_void_p(b.cuda_stream)) == 0
                if mode == "ordered":
                    fin = torch.cuda.Event()
                    fin.record(b)
                    a.wait_event(fin)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        return [x.elapsed_time(y) for x, y in evs]

    run("none", 2, 0)                             # warmup
    res = {m: [] for m in ("none", "overlap", "ordered", "gated")}
    for r in range(reps):
        for m in res:
            # the first epoch of a run follows no stand-in: only epochs 2.. count
            res[m] += run(m, 5, 100 + 5 * r)[1:]
    out = {"what": "epoch (reset + whole-game move) event span on the launch stream, ms; 9x9/256/200",
           "standin": {"workgroups": W, "lds_kb": LKB, "spin_us": TUS},
           "epochs_per_mode": len(res["none"])}
    for m, v in res.items():
        out[m] = {"mean_ms": float(np.mean(v)), "min_ms": float(np.min(v)), "max_ms": float(np.max(v))}
    # the same epochs (games) in every mode: per-epoch differences
    for m in ("overlap", "ordered", "gated"):
        d = np.array(res[m]) - np.array(res["none"])
        out[f"{m}_delay_ms"] = {"mean": float(d.mean()), "min": float(d.min()), "max": float(d.max())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
