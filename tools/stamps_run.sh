#!/bin/bash
# Per-phase cycle shares (MRBO_STAMPS variant) of the C3 kernel at ℓ = 1 and at the MLE ℓ.
root=${GRAFT_REPO_ROOT:-$PWD}
V=$root/rollout-bayesian-optimization_amd/mrbo/variants
out=$root/gpurun_out/stamps
mkdir -p $out
cd $root
MRBO_LIB=$V/libmrbo_stamps.so timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > $out/c3.json 2> $out/c3.err && \
MRBO_LIB=$V/libmrbo_stamps.so timeout -k 10 120 python -u bench.py --mle --steps 2 --warmup 1 --no-cpu-baseline \
  > $out/c3_mle.json 2> $out/c3_mle.err
rc=$?
grep "mrbo stamps" $out/c3.err | tail -17
echo ---
grep "mrbo stamps" $out/c3_mle.err | tail -17
exit $rc
