#!/usr/bin/env python3
"""profiles/traffic_<tag>.json from one tools/profile.sh run: HBM bytes per rollout launch from the
FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 --pmc runs), FETCH_SIZE doubled for gfx950
(MI355X_MICROARCH.md, HBM section: it counts 64 B per 128-B read request).  bench.py reads the file
of its workload tag at run time into roofline.traffic, so regenerate it whenever the kernel changes.

usage: python tools/traffic_json.py gpurun_out/prof_<tag> <config tag, e.g. C3 or C3_ell0.7211> [note]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    tmp = os.path.join(prof, "pmc_summary.json")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), prof, "--json", tmp],
                          stdout=subprocess.DEVNULL)
    s = json.load(open(tmp))
    fetch = 2.0 * s["fetch_kb"] * 1024.0
    write = s["write_kb"] * 1024.0
    out = {"config": tag, "kernel": s["kernel"],
           "source": f"{os.path.relpath(prof, ROOT)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                     "tools/profile.sh; last dispatch = the timed launch)",
           "fetch_size_kb_raw": s["fetch_kb"], "write_size_kb": s["write_kb"],
           "correction": "FETCH_SIZE x2 (gfx950 counts 64 B per 128-B read request, MI355X_MICROARCH.md HBM "
                         "section); WRITE_SIZE as reported; KB = 1024 B",
           "bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
           "kernel_avg_ms_under_profiler": s.get("avg_ms"), "note": note}
    path = os.path.join(ROOT, "profiles", f"traffic_{tag}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, out["bytes_per_launch"])


if __name__ == "__main__":
    main()
