#!/bin/bash
# per-trajectory wall times + work counters (MRBO_TAIL variant, MRBO_TAIL_DUMP) for the schedule's
# work weights: C3 and C3-MLE, index order (launch 1 = warm-up ... ), into gpurun_out/tail_dump/
root=${GRAFT_REPO_ROOT:-$PWD}; cd "$root"
out=gpurun_out/tail_dump; mkdir -p $out; rm -f $out/*.bin
L=rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_tail.so
MRBO_TAIL_DUMP=$out/c3.bin MRBO_LIB=$L timeout -k 10 150 python -u bench.py --steps 2 --warmup 1 --schedule index --no-cpu-baseline > $out/c3.json 2> $out/c3.err || exit 1
MRBO_TAIL_DUMP=$out/c3mle.bin MRBO_LIB=$L timeout -k 10 150 python -u bench.py --mle --steps 2 --warmup 1 --schedule index --no-cpu-baseline > $out/c3mle.json 2> $out/c3mle.err || exit 1
MRBO_TAIL_DUMP=$out/c3mle_lf.bin MRBO_LIB=$L timeout -k 10 150 python -u bench.py --mle --steps 3 --warmup 1 --no-cpu-baseline > $out/c3mle_lf.json 2> $out/c3mle_lf.err || exit 1
ls -la $out; grep -h "mrbo tail" $out/*.err
