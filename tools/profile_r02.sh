#!/bin/bash
# Round-2 profiles: the headline bench line (with the CPU baseline), the C3 profile (kernel-trace
# stats + separate PMC passes, tools/profile.sh), and kernel-trace stats of every bench row
# (C3 at the MLE lengthscale, C4 / C4-MLE, C5 / C5 at ℓ = 20 / C5 with NonUniformCost).
# Outputs under gpurun_out/r02p/; the summaries worth keeping are copied to profiles/r02/.
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/r02p
mkdir -p $out
cd $root
timeout -k 10 240 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 1
bash tools/profile.sh c3_r02 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
export TMPDIR=/tmp
row() {  # row <name> <bench args...>
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$name -o run -- \
    python3 $root/bench.py "$@" --no-cpu-baseline > $out/$name.json 2> $out/$name.err)
}
row c3_mle --mle --steps 3 --warmup 1 && \
row c4 --config C4 --mc-per-gpu 1024 --steps 3 --warmup 1 && \
row c4_mle --config C4 --mc-per-gpu 1024 --mle --steps 3 --warmup 1 && \
row c5 --config C5 --mc-per-gpu 2048 --steps 2 --warmup 1 && \
row c5_l20 --config C5 --mc-per-gpu 64 --restarts 64 --ell 20 --steps 2 --warmup 1 && \
row c5_cost --config C5 --mc-per-gpu 256 --cost --steps 2 --warmup 1 && \
row c2 --config C2 --steps 3 --warmup 1
rc=$?
python tools/pmc_summary.py $root/gpurun_out/prof_c3_r02 --json $out/pmc_summary_c3.json > $out/pmc_summary_c3.txt
echo "rows rc=$rc"
exit $rc
