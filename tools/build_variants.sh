#!/bin/bash
# Build A/B variants of libmrbo.so (one input dimension, default d=6) into mrbo/variants/ for timing
# on the GPU box.  usage: [MRBO_VARIANT_DIMS=8] tools/build_variants.sh name:"-DFLAG ..." [name:"..."] ...   (default: base + stamps)
set -e
cd "$(dirname "$0")/.."
mkdir -p rollout-bayesian-optimization_amd/mrbo/variants
[ $# -eq 0 ] && set -- "base:" "stamps:-DMRBO_STAMPS"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  python3 - "$name" "$flags" <<'PY' &
import shlex, sys
import __graft_entry__ as g
name, flags = sys.argv[1], sys.argv[2]
import os
dims = [int(x) for x in os.environ.get("MRBO_VARIANT_DIMS", "6").split(",")]
g.compile_lib(f"{g.PKG}/mrbo/variants/libmrbo_{name}.so", extra=shlex.split(flags), dims=dims, jobs=2)
PY
done
wait
ls -la rollout-bayesian-optimization_amd/mrbo/variants
