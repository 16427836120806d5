#!/bin/bash
# Build A/B variants of libmrbo.so (d=6 only) into mrbo/variants/ for timing on the GPU box.
set -e
cd "$(dirname "$0")/../rollout-bayesian-optimization_amd"
build() { name=$1; shift; hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMRBO_ONLY_D=6 "$@" -o mrbo/variants/libmrbo_$name.so csrc/mrbo_api.hip & }
build base
build inl -DMRBO_INLINE_TRANSCENDENTALS
build inl_nolicm -DMRBO_INLINE_TRANSCENDENTALS -mllvm -disable-machine-licm
build w1 -DMRBO_WAVES_PER_SIMD=1
wait
ls -la mrbo/variants
