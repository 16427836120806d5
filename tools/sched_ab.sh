#!/bin/bash
# A/B of the trajectory schedule on the main library (C3 by default, BENCH_ARGS for others):
# index order vs longest-first (round-robin over the per-XCD chunks), REPS interleaved rounds;
# then the MRBO_TAIL variant (mrbo/variants/libmrbo_tail.so) once per schedule for the idle tail.
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/sched_ab${TAG:+_$TAG}
mkdir -p "$out"
cd "$root"
for rep in $(seq 1 "${REPS:-3}"); do
  for s in index longest-first; do
    timeout -k 10 150 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --schedule $s $BENCH_ARGS \
      > "$out/${s}_$rep.json" 2> "$out/${s}_$rep.err" || { echo "$s rep $rep failed"; tail -5 "$out/${s}_$rep.err"; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], round(d['value']), 'traj/s kernel', round(d['roofline']['kernel_ms'],3), 'ms step', round(d['ms_per_step'],3))" "$out/${s}_$rep.json" $s $rep
  done
done
if [ -f rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_tail.so ]; then
  for s in index longest-first; do
    MRBO_LIB=rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_tail.so timeout -k 10 150 python -u bench.py --steps 3 --warmup 2 \
      --no-cpu-baseline --schedule $s $BENCH_ARGS > "$out/tail_$s.json" 2> "$out/tail_$s.err" || exit 1
    echo "tail $s"; grep "mrbo tail" "$out/tail_$s.err" | tail -3
  done
fi
