#!/bin/bash
# Round-3 GPU session: a chain of steps, each under its own time limit, stopping at the first
# failure.  usage (on the box, from the repo root): bash tools/gpu_r03.sh <tag> step [step ...]
#   tests     pytest -m gpu (all GPU tests; parity statistics -> parity.json)
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py (the driver's default line, C3)
#   rows      bench rows: C3 at the MLE ℓ, C4 at ℓ = 0.5 and MLE, C2 (no CPU baseline)
#   prof      rocprofv3 --kernel-trace --stats of the default bench (1 step) + FETCH_SIZE / WRITE_SIZE
#             passes (tools/profile.sh), C3 and C3-MLE
# Outputs under gpurun_out/<tag>/.
root=${GRAFT_REPO_ROOT:-$PWD}
tag=$1; shift
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
export MRBO_PARITY_REPORT=$out/parity.json
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > "$out/pytest.log" 2>&1
      rc=$?; tail -5 "$out/pytest.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
      rc=$?; tail -3 "$out/smoke.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$out/bench_c3.json" 2> "$out/bench_c3.err"
      rc=$?; tail -c 600 "$out/bench_c3.json" ;;
    rows)
      timeout -k 10 200 python -u bench.py --mle --no-cpu-baseline > "$out/bench_c3_mle.json" 2> "$out/bench_c3_mle.err" && \
      timeout -k 10 200 python -u bench.py --config C4 --mc-per-gpu 1024 --steps 3 --warmup 1 --ell 0.5 --no-cpu-baseline \
        > "$out/bench_c4_l05.json" 2> "$out/bench_c4_l05.err" && \
      timeout -k 10 200 python -u bench.py --config C4 --mc-per-gpu 1024 --steps 3 --warmup 1 --mle --no-cpu-baseline \
        > "$out/bench_c4_mle.json" 2> "$out/bench_c4_mle.err" && \
      timeout -k 10 200 python -u bench.py --config C2 --no-cpu-baseline > "$out/bench_c2.json" 2> "$out/bench_c2.err"
      rc=$?
      for f in "$out"/bench_*.json; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['work_per_traj'])" "$f"
      done ;;
    prof)
      bash tools/profile.sh "${tag}_c3" && bash tools/profile.sh "${tag}_c3mle" --steps 1 --warmup 1 --no-cpu-baseline --mle
      rc=$? ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "== $step rc=$rc $(date +%T)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
