#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-launch counters of the rollout kernel.

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [--json out.json]

Prints per-wave instruction counts (SQ_* / SQ_WAVES), the issue/wait split, the kernel-trace
average duration, and FETCH_SIZE / WRITE_SIZE per launch.  FETCH_SIZE / WRITE_SIZE are
rocprofv3's derived TCC counters in KB; per MI355X_MICROARCH.md §HBM, FETCH_SIZE counts 64 B
per memory-side read request (half the bytes of a wide 128-B request) -- reported raw and
with the ×2 correction; our reads are narrow (dword / dwordx2 per lane), where the guide calls
the scale uncalibrated.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "rollout_kernel"


def counters(path):
    """{counter: [value per dispatch]} for the rollout kernel."""
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(path, "run_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if KERNEL not in row["Kernel_Name"]:
                    continue
                per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: [v[d] for d in sorted(v, key=int)] for k, v in per.items()}


def main():
    root = sys.argv[1]
    out = {}
    with open(os.path.join(root, "stats", "run_kernel_stats.csv")) as fh:
        for row in csv.DictReader(fh):
            if KERNEL in row["Name"]:
                out["kernel"] = row["Name"]
                out["calls"] = int(row["Calls"])
                out["avg_ms"] = float(row["AverageNs"]) * 1e-6
    allc = {}
    for sub in ("pmc_issue", "pmc_valu", "pmc_lds", "pmc_fetch", "pmc_write"):
        p = os.path.join(root, sub)
        if os.path.isdir(p):
            for k, v in counters(p).items():
                allc[k] = v[-1]          # last dispatch (after warmup)
    waves = allc.get("SQ_WAVES", float("nan"))
    out["waves_per_launch"] = waves
    per_wave = {k: v / waves for k, v in allc.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
    out["per_wave"] = per_wave
    if "SQ_WAVE_CYCLES" in allc:
        wc = allc["SQ_WAVE_CYCLES"]
        out["split"] = {k: allc[k] / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY") if k in allc}
    if "FETCH_SIZE" in allc:
        out["fetch_kb"] = allc["FETCH_SIZE"]
    if "WRITE_SIZE" in allc:
        out["write_kb"] = allc["WRITE_SIZE"]
    for k, v in sorted(out.items()):
        if k == "per_wave":
            print("per wave:")
            for kk, vv in sorted(v.items()):
                print(f"  {kk:28s} {vv:14.1f}")
        else:
            print(f"{k}: {v}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
