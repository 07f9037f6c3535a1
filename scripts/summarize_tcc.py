"""Summarise a scripts/pmc_tcc.sh run of k_selfplay_move into
profiles/<tag>_tcc.json: memory-side read / write requests by size, bytes
under each accounting, L2 hit rate, per launch (means over the dispatches).

Read bytes: 128 B per TCC_BUBBLE (a 128-B request), 32 B per _32B request,
64 B for the rest (rocprofv3's FETCH_SIZE expression); write bytes: 64 B per
_64B request, 32 B for the rest (WRITE_SIZE's).  Beside them the bench's old
accounting (2 x FETCH_SIZE + WRITE_SIZE: MI355X_MICROARCH.md's doubling,
calibrated on 16-B/lane streaming reads only)."""
import collections
import csv
import json
import os
import statistics
import sys

tag = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else "k_selfplay_move"
src = os.path.join("gpurun_out", f"tcc_{tag}")
stats = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))) if kernel in r["Name"]][0]
c = collections.defaultdict(list)
for d in ("rd", "wr", "l2"):
    f = os.path.join(src, d, "run_counter_collection.csv")
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kernel in r["Kernel_Name"]:
            per[(r["Counter_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))] += float(r["Counter_Value"])
    for (name, _), v in per.items():
        c[name].append(v)
m = {k: statistics.mean(v) for k, v in c.items()}
rd, r32, bub = m["TCC_EA0_RDREQ_sum"], m["TCC_EA0_RDREQ_32B_sum"], m["TCC_BUBBLE_sum"]
wr, w64 = m["TCC_EA0_WRREQ_sum"], m["TCC_EA0_WRREQ_64B_sum"]
read_b = bub * 128 + (rd - bub - r32) * 64 + r32 * 32
write_b = w64 * 64 + (wr - w64) * 32
fetch_kb = read_b / 1024
out = {
    "tag": tag, "kernel": kernel, "avg_duration_ms": float(stats["AverageNs"]) / 1e6,
    "dispatches": int(stats["Calls"]), "counters": m,
    "read_requests": {"all": rd, "128B": bub, "32B": r32, "64B": rd - bub - r32},
    "write_requests": {"all": wr, "64B": w64, "32B": wr - w64},
    "hbm_bytes_per_launch": read_b + write_b,
    "read_bytes": read_b, "write_bytes": write_b,
    "dram_read_requests_share": m.get("TCC_EA0_RDREQ_DRAM_sum", 0) / max(rd, 1),
    "old_accounting_bytes": 2 * read_b + write_b,
    "l2_hit_rate": m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1),
    "l2_requests": {"read": m.get("TCC_READ_sum"), "write": m.get("TCC_WRITE_sum")},
    "what": "memory-side (TCC_EA0) requests of one launch by size; bytes = 128/64/32 B per read request by size "
            "(FETCH_SIZE's expression), 64/32 B per write request (WRITE_SIZE's)",
}
os.makedirs("profiles", exist_ok=True)
json.dump(out, open(os.path.join("profiles", f"{tag}_tcc.json"), "w"), indent=1)
print(json.dumps({k: out[k] for k in ("avg_duration_ms", "read_requests", "write_requests", "hbm_bytes_per_launch",
                                       "old_accounting_bytes", "l2_hit_rate", "dram_read_requests_share")}))
