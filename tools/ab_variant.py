#!/usr/bin/env python3
"""Fast A/B variants of the N ≤ 64 rollout kernel (C2/C3): one kernel unit (d, FMAX = 4) compiled
with -DMRBO_AB_MIN (RPL = 1, the specialised kernel only: seconds instead of minutes) and extra
flags, linked with the main build's host-API and GP-fit objects into mrbo/variants/libmrbo_<name>.so.
Plans of other shapes fail to create in such a library.

usage: python tools/ab_variant.py name:"-DFLAG ..." [name:"..."] ... [--dims 6] [--fmax 4] [--rpl 1]
(C5: --dims 8 --fmax 6 --rpl 4)
Run __graft_entry__.build() first (the api / gpfit objects come from its object directory).
"""
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402


def main():
    args = sys.argv[1:]
    dims, fmax, rpl = [6], 4, 1
    if "--dims" in args:
        i = args.index("--dims")
        dims = [int(x) for x in args[i + 1].split(",")]
        del args[i:i + 2]
    if "--rpl" in args:
        i = args.index("--rpl")
        rpl = int(args[i + 1])
        del args[i:i + 2]
    if "--fmax" in args:
        i = args.index("--fmax")
        fmax = int(args[i + 1])
        del args[i:i + 2]
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    vdir = os.path.join(g.PKG, "mrbo", "variants")
    os.makedirs(vdir, exist_ok=True)
    base = [os.path.join(g.OBJDIR, "api.o"), os.path.join(g.OBJDIR, "gpfit.o"), os.path.join(g.OBJDIR, "order.o")]
    for b in base:
        if not os.path.exists(b):
            raise SystemExit(f"{b} missing: run __graft_entry__.build() first")
    procs = []
    for spec in args:
        name, _, flags = spec.partition(":")
        objs = []
        for d in dims:
            obj = os.path.join(vdir, f"{name}_k{d}_f{fmax}.o")
            defs = [f"-DMRBO_D={d}", "-DMRBO_AB_MIN", f"-DMRBO_AB_RPL={rpl}"] + ([f"-DMRBO_FMAX={fmax}"] if fmax != 6 else [])
            unit = g.UNIT_FLAGS + (g.F4_FLAGS if fmax == 4 else [])   # as the main build's units
            cmd = [hipcc] + g.HIPCC_FLAGS + unit + shlex.split(flags) + defs + \
                  ["-c", "-o", obj, os.path.join(g.CSRC, "mrbo_kernels.hip")]
            procs.append((subprocess.Popen(cmd, stderr=subprocess.DEVNULL), name))
            objs.append(obj)
        if True:   # a fresh host API with the variant's flags (stamp counters, queue layout, ...)
            api = os.path.join(vdir, f"{name}_api.o")
            cmd = [hipcc] + g.HIPCC_FLAGS + shlex.split(flags) + ["-c", "-o", api, os.path.join(g.CSRC, "mrbo_api.hip")]
            procs.append((subprocess.Popen(cmd, stderr=subprocess.DEVNULL), name))
            objs.append(api)
        procs.append((None, (name, objs)))
    pending = []
    for p, info in procs:
        if p is None:
            name, objs = info
            out = os.path.join(vdir, f"libmrbo_{name}.so")
            pending.append((name, objs, out))
            continue
        if p.wait() != 0:
            raise SystemExit(f"variant {info}: compile failed")
    for name, objs, out in pending:
        bo = base if not any(o.endswith("_api.o") for o in objs) else base[1:]
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs + bo)
        print("built", out)


if __name__ == "__main__":
    main()
