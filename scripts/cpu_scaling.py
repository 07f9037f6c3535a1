"""CPU baseline scaling on the GPU box (cpu_baseline's core count).

Runs bench.py's cpu_baseline_procs (P single-thread oracle processes, sims/s
summed) at several P and records what the host reports about its CPUs: the
cgroup's CPU quota (cpu.max), the affinity mask, os.cpu_count().  Never
touches the GPU.

    python scripts/cpu_scaling.py --procs 16 32 64 --budget 6 > profiles/r6_cpu_scaling.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-go_amd")]


def cgroup_cpus():
    """The cgroup v2 CPU quota as a CPU count (None when unlimited or absent)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
    except (OSError, ValueError):
        return None, None
    raw = f"{quota} {period}"
    if quota == "max":
        return None, raw
    return int(quota) / int(period), raw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, nargs="+", default=[16, 32, 64])
    ap.add_argument("--budget", type=float, default=6.0)
    args = ap.parse_args()
    import bench
    q, raw = cgroup_cpus()
    host = {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_cpu_max": raw,
            "cgroup_cpus": q, "share": bench.cpu_share()}
    rows = []
    for p in args.procs:
        r = bench.cpu_baseline_procs(9, 96, 200, args.budget, p)
        rows.append({"procs": p, "sims_per_s": r["value"], "per_proc": r["value"] / p,
                     "single_core_value": r["single_core_value"],
                     "one_process_all_threads": r["one_process_all_threads"]["value"]})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"host": host, "workload": "9x9, 200 sims/move, oracle MCTS + torch-CPU batch-1 net (C=96)",
                      "budget_s_per_proc": args.budget, "rows": rows}))


if __name__ == "__main__":
    main()
