#!/bin/bash
# GP-fit A/B on one box: the default library against variant libraries (mrbo/variants/<name>.so),
# interleaved twice; then the -DMRBO_GPFIT_STAMPS variants' phase stamps.
# usage: bash tools/ab_gpfit.sh <tag> "<variant names>" "<stamp variant names>" [N list]
tag=$1; vars=$2; svars=$3; ns=${4:-128,256,384,512}
out=gpurun_out/$tag
mkdir -p "$out"
V=$PWD/rollout-bayesian-optimization_amd/mrbo/variants
for rep in 1 2; do
  for v in default $vars; do
    lib=""; [ "$v" != default ] && lib=$V/$v.so
    MRBO_LIB=$lib timeout -k 10 200 python -u tools/bench_rows.py --rows gp_fit --gpfit-n $ns --cpu-seconds 0.05 \
      > "$out/rows_${v}_$rep.jsonl" 2> "$out/rows_${v}_$rep.err" || exit 1
    python -c "
import sys, json
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(sys.argv[2], d['config']['workload'][:6], round(d['kernel_ms'], 4), 'ms kernel')" "$out/rows_${v}_$rep.jsonl" "$v/$rep"
  done
done
for v in $svars; do
  MRBO_LIB=$V/$v.so timeout -k 10 200 python -u tools/bench_rows.py --rows gp_fit --gpfit-n $ns --cpu-seconds 0.05 \
    > "$out/stamps_$v.jsonl" 2> "$out/stamps_$v.err" || exit 1
  grep -h "gpfit_tile" "$out/stamps_$v.jsonl" "$out/stamps_$v.err" | sort -t= -k2 -n | awk 'NR%6==1' | sed "s/^/$v: /"
done
