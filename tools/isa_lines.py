#!/usr/bin/env python3
"""Static VALU/LDS/SALU instruction counts of a kernel's ISA, attributed to source lines.

usage: python tools/isa_lines.py <kernel.s> [--site LINE] [--file mrbo_rollout.hip] [--top 40]
The .s must be compiled with -gline-tables-only.  Each instruction is attributed to the
innermost location in --file (default mrbo_rollout.hip) of its inlining chain; --site keeps only
instructions whose chain passes through that line of --file (e.g. one inlined evaluate call site).
"""
import collections
import re
import sys

def main():
    path = sys.argv[1]
    args = sys.argv[2:]
    site = int(args[args.index("--site") + 1]) if "--site" in args else None
    fname = args[args.index("--file") + 1] if "--file" in args else "mrbo_rollout.hip"
    top = int(args[args.index("--top") + 1]) if "--top" in args else 40
    chain = []
    cnt = collections.Counter()
    kinds = collections.defaultdict(collections.Counter)
    for l in open(path):
        if "\t.loc\t" in l or l.lstrip().startswith(".loc"):
            locs = re.findall(r"([\w./-]+):(\d+):\d+", l)
            chain = [(f.split("/")[-1], int(n)) for f, n in locs]
            continue
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if site is not None and (fname, site) not in chain:
            continue
        inner = next(((f, n) for f, n in chain if f == fname), None)
        if inner is None:
            continue
        k = "valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else "salu" if op.startswith("s_") else "mem"
        cnt[inner[1]] += 1
        kinds[inner[1]][k] += 1
    tot = collections.Counter()
    for ln, c in kinds.items():
        tot.update(c)
    print("total", dict(tot))
    for ln, c in sorted(cnt.items(), key=lambda x: -x[1])[:top]:
        print(f"{ln:6d} {c:6d}  {dict(kinds[ln])}")

main()
