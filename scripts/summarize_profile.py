"""Summarise a scripts/profile.sh run into profiles/<tag>_*.{csv,json}.

HBM traffic per launch of the dominant kernel follows MI355X_MICROARCH.md's
rocprofv3 recipe: FETCH_SIZE and WRITE_SIZE are collected in separate passes
(kilobytes); on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
reads, so it is doubled; WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else "k_selfplay_move"
src = os.path.join("gpurun_out", f"prof_{tag}")
dst = "profiles"
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))


def per_launch(name):
    rows = [r for r in csv.DictReader(open(os.path.join(src, name, "run_counter_collection.csv")))
            if kernel in r["Kernel_Name"]]
    return [float(r["Counter_Value"]) * 1024 for r in rows]


fetch = per_launch("fetch")
write = per_launch("write")
stats = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))
         if kernel in r["Name"]][0]
out = {
    "kernel": stats["Name"],
    "calls": int(stats["Calls"]),
    "avg_duration_ms": float(stats["AverageNs"]) / 1e6,
    "fetch_bytes_per_launch_raw": statistics.median(fetch),
    "fetch_bytes_per_launch_corrected_x2": 2 * statistics.median(fetch),
    "write_bytes_per_launch": statistics.median(write),
    "hbm_bytes_per_launch": 2 * statistics.median(fetch) + statistics.median(write),
}
out["hbm_GBps"] = out["hbm_bytes_per_launch"] / (out["avg_duration_ms"] / 1e3) / 1e9
out["tag"] = tag
out["workload"] = sys.argv[3] if len(sys.argv) > 3 else "9x9 Go self-play, 256 parallel games/GPU, 200 sims/move"
out["dynamics"] = sys.argv[4] if len(sys.argv) > 4 else "factored"
json.dump(out, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1)
json.dump(out, open(os.path.join(dst, "latest_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
