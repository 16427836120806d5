#!/bin/bash
# Interleaved A/B of library variants (mrbo/variants/libmrbo_<v>.so) on the GPU box: REPS rounds,
# each running every variant once (bench.py C3, or BENCH_ARGS), so that clock drift between boxes
# and over time falls on all variants alike.  Prints kernel ms per run and the per-variant median.
# usage: [REPS=3] [BENCH_ARGS="--mle"] [TAG=x] bash tools/ab_rep.sh base fold ...
# A variant lib+VAR=value runs libmrbo_<lib>.so with VAR=value in its environment; lib "main" is
# the main build (mrbo/libmrbo.so).
root=${GRAFT_REPO_ROOT:-$PWD}
V=$root/rollout-bayesian-optimization_amd/mrbo/variants
out=$root/gpurun_out/ab_rep${TAG:+_$TAG}
mkdir -p "$out"
cd "$root"
REPS=${REPS:-3}
for rep in $(seq 1 "$REPS"); do
  for v in "$@"; do
    f=$out/${v}_$rep
    lib=${v%%+*}; envs=""
    [[ $v == *+* ]] && envs=${v#*+}
    so=$V/libmrbo_$lib.so
    [[ $lib == main ]] && so=$root/rollout-bayesian-optimization_amd/mrbo/libmrbo.so
    env $envs MRBO_LIB=$so timeout -k 10 120 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline $BENCH_ARGS \
      > "$f.json" 2> "$f.err" || { echo "variant $v rep $rep failed"; tail -5 "$f.err"; exit 1; }
    python - "$f.json" "$v" "$rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:14s} rep {sys.argv[3]}  {d['value']:12.0f} traj/s  kernel {d['roofline']['kernel_ms']:.3f} ms  "
      f"frac {d['roofline']['frac']:.4f}  work {d['work_per_traj']}", flush=True)
PY
    grep "mrbo stamps" "$f.err" | grep -v " 0.00%" | tail -24
  done
done
python - "$out" "$@" <<'PY'
import glob, json, statistics, sys
out, names = sys.argv[1], sys.argv[2:]
for v in names:
    ks = []
    for f in sorted(glob.glob(f"{out}/{v}_*.json")):
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
        ks.append(d["roofline"]["kernel_ms"])
    print(f"median {v:14s} kernel {statistics.median(ks):.3f} ms  runs {['%.3f' % k for k in ks]}")
PY
