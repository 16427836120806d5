#!/bin/bash
# A/B timing of d=8 library variants on the C5 row (N=256, 256 MC x 512 restarts per launch).
# usage: MRBO_VARIANT_DIMS=8 tools/build_variants.sh name:"-D..." ... ; bash tools/ab_run_c5.sh name ...
V=${GRAFT_REPO_ROOT:-$PWD}/rollout-bayesian-optimization_amd/mrbo/variants
mkdir -p gpurun_out
for v in "$@"; do
  MRBO_LIB=$V/libmrbo_$v.so timeout -k 10 200 python bench.py --config C5 --mc-per-gpu 256 --steps 2 --warmup 1 \
    --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "variant $v failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value']), d['roofline']['kernel_ms'])"
done
