#!/usr/bin/env python3
"""List the names the reference defines at top level of `Main` into tests/golden/julia_ref_names.json.

The reference is not a Julia package: rollout_bayesian_optimization.jl:15-30 `include`s its files
into `Main`, so every top-level function, type and constant of those files is a `Main` binding.
tests/test_julia_binding.py checks that julia/MRBO.jl (a `module`, which sees only Base/Core
unless told otherwise) brings every such name it uses into scope from `Main`, and `import`s the
ones it adds methods to.  Data only (names and the file:line that defines each), read from the
reference's sources as text.  Run here, where /root/reference exists; the JSON travels with the repo.
usage: python tests/golden/make_julia_names.py [--reference /root/reference]
"""
import argparse
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
IDENT = r"[A-Za-z_¡-￿][A-Za-z0-9_!¡-￿]*"
DEFS = [
    re.compile(rf"^function\s+({IDENT})\s*[({{]"),             # function f(…) / function f{T}(…)
    re.compile(rf"^(?:mutable\s+)?struct\s+({IDENT})"),        # struct T / mutable struct T
    re.compile(rf"^abstract\s+type\s+({IDENT})"),
    re.compile(rf"^const\s+({IDENT})\s*="),
    re.compile(rf"^({IDENT})\s*\([^=]*\)\s*(?:where\s+[^=]+)?=[^=]"),   # one-line method f(x) = …
    re.compile(rf"^({IDENT})\s*=[^=]"),                         # global assignment
]


def included_files(ref):
    entry = os.path.join(ref, "rollout_bayesian_optimization.jl")
    files = []
    for line in open(entry, encoding="utf-8"):
        m = re.match(r'\s*include\("([^"]+)"\)', line)
        if m:
            files.append(m.group(1))
    return entry, files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    entry, files = included_files(args.reference)
    names = {}
    for f in files:
        for ln, line in enumerate(open(os.path.join(args.reference, f), encoding="utf-8"), 1):
            for rx in DEFS:
                m = rx.match(line)
                if m:
                    names.setdefault(m.group(1), f"{f}:{ln}")
                    break
    packages = []
    for line in open(entry, encoding="utf-8"):
        m = re.match(rf"\s*using\s+({IDENT})", line)
        if m:
            packages.append(m.group(1))
    out = {"source": "rollout_bayesian_optimization.jl:1-30 includes (top-level definitions)",
           "included": files, "packages": packages, "names": dict(sorted(names.items()))}
    path = os.path.join(HERE, "julia_ref_names.json")
    with open(path, "w", encoding="utf-8") as fh:
        json.dump(out, fh, indent=1, ensure_ascii=False)
    print(f"{len(names)} names from {len(files)} files -> {path}")


if __name__ == "__main__":
    main()
