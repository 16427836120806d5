#!/bin/bash
# C2 launch A/B on the GPU box: the default library against variants/libmrbo_<v>.so, index order and
# longest-first (bench.py --schedule auto), 10 steps each.  usage: bash tools/ab_c2.sh <tag> <variant>...
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
V=$PWD/rollout-bayesian-optimization_amd/mrbo/variants
for v in base "$@"; do
  for sch in index auto; do
    if [ "$v" = base ]; then lib=""; else lib="$V/libmrbo_$v.so"; fi
    MRBO_LIB=$lib timeout -k 10 120 python -u bench.py --config C2 --steps 10 --warmup 2 --no-cpu-baseline --schedule $sch \
      > "$out/c2_${v}_$sch.json" 2> "$out/c2_${v}_$sch.err" || { echo "$v $sch failed"; tail -5 "$out/c2_${v}_$sch.err"; exit 1; }
    python -c "
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], round(d['value']), 'traj/s; kernel', round(d['roofline']['kernel_ms'], 4), 'ms; step', round(d['ms_per_step'], 4), 'ms; frac', round(d['roofline']['frac'], 4), d['roofline']['launch'])" "$out/c2_${v}_$sch.json" $v $sch
  done
done
