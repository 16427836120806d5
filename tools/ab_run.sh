#!/bin/bash
# A/B timing of library variants on the GPU box: bench.py per variant (+ stamps where built).
# usage: [BENCH_ARGS="--mle"] bash tools/ab_run.sh base inl ...   (variants from tools/build_variants.sh)
V=${GRAFT_REPO_ROOT:-$PWD}/rollout-bayesian-optimization_amd/mrbo/variants
mkdir -p gpurun_out
for v in "$@"; do
  MRBO_LIB=$V/libmrbo_$v.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS \
    > gpurun_out/ab_$v$AB_TAG.json 2> gpurun_out/ab_$v$AB_TAG.err || { echo "variant $v failed"; exit 1; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
lines = [l for l in open(f"gpurun_out/ab_{v}.json") if l.startswith("{")]
d = json.loads(lines[-1])
print(f"{v:12s} {d['value']:12.0f} traj/s  kernel {d['roofline']['kernel_ms']:.2f} ms  frac {d['roofline']['frac']:.4f}")
PY
  grep "mrbo stamps" gpurun_out/ab_$v$AB_TAG.err | head -30
done
