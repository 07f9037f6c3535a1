"""Summarise a scripts/pmc.sh run into profiles/<tag>_pmc.json (and
profiles/latest_pmc.json, which bench.py reads) + profiles/<tag>_kernel_stats.csv.

Per-launch means over every dispatch of the kernel (the trace's average
duration; each counter's mean over its pass).  HBM bytes follow
MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE from separate passes (KB),
FETCH_SIZE doubled on gfx950, WRITE_SIZE as is.
"""
import csv
import collections
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "9x9 Go self-play, 256 parallel games/GPU, 200 sims/move"
dynamics = sys.argv[3] if len(sys.argv) > 3 else "factored"
kernel = sys.argv[4] if len(sys.argv) > 4 else "k_selfplay_move"
moves_per_launch = int(sys.argv[5]) if len(sys.argv) > 5 else 0   # bench.py --moves-per-launch (0: whole games)
latest = sys.argv[6] if len(sys.argv) > 6 else "latest_pmc.json"       # the file bench.py reads
in_clk = float(sys.argv[7]) if len(sys.argv) > 7 else 0.0   # in-kernel clock (GHz) from a stamps build, optional
src = os.path.join("gpurun_out", f"pmc_{tag}")
os.makedirs("profiles", exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join("profiles", f"{tag}_kernel_stats.csv"))
stats = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))) if kernel in r["Name"]][0]

counters = collections.defaultdict(list)
for d in ("p1", "p2", "fetch", "write"):
    f = os.path.join(src, d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kernel in r["Kernel_Name"]:
            per[(r["Counter_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))] += float(r["Counter_Value"])
    for (name, _), v in per.items():
        counters[name].append(v)
mean = {k: statistics.mean(v) for k, v in counters.items()}
out = {
    "tag": tag, "workload": workload, "dynamics": dynamics, "moves_per_launch": moves_per_launch,
    "kernel": stats["Name"], "calls": int(stats["Calls"]),
    "avg_duration_ms": float(stats["AverageNs"]) / 1e6,
    "counters": mean, "dispatches_per_counter": {k: len(v) for k, v in counters.items()},
}
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    out["hbm_bytes_per_launch"] = 2 * mean["FETCH_SIZE"] * 1024 + mean["WRITE_SIZE"] * 1024
    out["hbm_GBps"] = out["hbm_bytes_per_launch"] / (out["avg_duration_ms"] / 1e3) / 1e9
    out["hbm_accounting"] = ("2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE doubled on gfx950, "
                             "calibrated on 16-B/lane streaming reads; an upper bound for narrower reads)")
    # the same command's memory-side requests by size (scripts/pmc_tcc.sh -> summarize_tcc.py), if run
    tcc = os.path.join("profiles", f"{tag}_tcc.json")
    if os.path.exists(tcc):
        t = json.load(open(tcc))
        out["hbm_bytes_per_launch_requests_x_size"] = t["hbm_bytes_per_launch"]
        out["tcc"] = {k: t[k] for k in ("read_requests", "write_requests", "l2_hit_rate")}
        out["tcc"]["source"] = f"profiles/{tag}_tcc.json"
c = mean
dur = out["avg_duration_ms"] / 1e3
if "GRBM_GUI_ACTIVE" in c:
    # GRBM_GUI_ACTIVE / 8 XCDs / duration reads HIGH on dispatches shorter
    # than ~0.3 ms (MI355X_MICROARCH.md, DVFS give-back): k_tconv's 26 us
    # launches gave 3.12 GHz.  The clock used is that quotient only for
    # dispatches >= 0.3 ms, and never above the chip's 2.4 GHz maximum; for
    # shorter ones it is 2.4 GHz, so every busy fraction below is a LOWER
    # bound (the in-kernel s_memtime clock, ~2.1 GHz on k_tconv, would give
    # fractions ~14 % higher).
    grbm_clk = c["GRBM_GUI_ACTIVE"] / 8 / dur
    clk = min(grbm_clk, 2.4e9) if dur >= 0.3e-3 else 2.4e9
    cu_cycles = 256 * clk * dur
    out["derived"] = {
        "effective_clock_GHz": clk / 1e9,
        "grbm_quotient_GHz": grbm_clk / 1e9,
        "clock_source": ("GRBM_GUI_ACTIVE / 8 / duration (dispatch >= 0.3 ms), capped at 2.4 GHz"
                         if dur >= 0.3e-3 else "2.4 GHz (dispatch < 0.3 ms: the GRBM quotient reads high)"),
        "valu_issue_frac": c.get("SQ_INSTS_VALU", 0) / (2 * cu_cycles),
        "mfma_busy_frac": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (4 * cu_cycles),
        "mfma_insts_per_launch": c.get("SQ_INSTS_MFMA", 0),
        "lds_array_busy_frac": c.get("SQ_LDS_IDX_ACTIVE", 0) / cu_cycles,
        "lds_bank_conflict_share": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0)),
        "wave_wait_any_share": c.get("SQ_WAIT_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0)),
        "wave_issue_stall_share": c.get("SQ_WAIT_INST_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0)),
        "wave_active_share": c.get("SQ_ACTIVE_INST_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0)),
        **({"in_kernel_clock_GHz": in_clk,
            "mfma_busy_frac_at_in_kernel_clock": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (4 * 256 * in_clk * 1e9 * dur),
            "in_kernel_clock_source": "s_memtime / s_memrealtime deltas of a -DMZGO_TCONV_STAMPS build "
                                      "(scripts/tconv_stamps.py), same workload"} if in_clk > 0 else {}),
        "note": "fractions of CU-cycles at effective_clock_GHz (see clock_source); "
                "VALU peak 2 wave-instr/clk/CU, MFMA busy summed over 4 SIMDs, LDS array one cycle/clk/CU; "
                "wave shares of SQ_WAVE_CYCLES (quad-cycles, as the SQ_WAIT_*/ACTIVE_* counters)",
    }
json.dump(out, open(os.path.join("profiles", f"{tag}_pmc.json"), "w"), indent=1)
json.dump(out, open(os.path.join("profiles", latest), "w"), indent=1)
print(json.dumps(out, indent=1))
