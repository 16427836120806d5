#!/bin/bash
# Build A/B variants of libmrbo.so (d=6 only) into mrbo/variants/ for timing on the GPU box.
# usage: tools/build_variants.sh name:"-DFLAG ..." [name:"..."] ...   (default: base + stamps)
set -e
cd "$(dirname "$0")/../rollout-bayesian-optimization_amd"
mkdir -p mrbo/variants
[ $# -eq 0 ] && set -- "base:" "stamps:-DMRBO_STAMPS"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMRBO_ONLY_D=6 $flags \
    -o mrbo/variants/libmrbo_$name.so csrc/mrbo_api.hip &
done
wait
ls -la mrbo/variants
