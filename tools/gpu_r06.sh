#!/bin/bash
# Round-6 GPU session: a chain of steps, each under its own time limit, stopping at the first
# failure.  usage (on the box, from the repo root): bash tools/gpu_r06.sh <tag> step [step ...]
#   tests     pytest -m gpu (all GPU tests; parity statistics -> parity.json)
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py (the driver's default line, C3)
#   rows      bench rows: C3 at the MLE ℓ, C4 at ℓ = 0.5 and MLE, C2 (no CPU baseline)
#   ab        A/B of the library variants in mrbo/variants (AB_VARIANTS, default "old new oldst newst")
#   gpfit     tools/bench_rows.py gp_fit rows (N = 64 .. 512, 256 lengthscales per launch)
#   bo        tools/bo_compare.py, BO_TRIALS (40) trials per case, BO_CASES (default: the asserted
#             set; a comma list of tools/bo_compare.py SETTINGS keys) -> bo_compare.jsonl
#   sharded   C3 bench over the multi-rank path at one rank (--sharded: RCCL all-gather, device merge)
#             beside the plain line, 10 steps each, no CPU baseline
#   shim      tools/shim_rate.py at C3 (the Julia drop-in's call patterns)
#   c2        C2 bench line (20 steps)
#   myopic    myopic BO diagnostics: seeds, solve margins, no-repeat pick (4 cases, 60 trials)
#   c5        C5 at ℓ = 1 (2 048 × 512) and ℓ = 20 (64 × 64)
#   c5cost    C5 + NonUniformCost at M = 256, R = 128 (one step)
#   ab6       A/B: this library vs mrbo/variants/libmrbo_r6old.so (C3, C3-MLE)
#   ab6c5     the same for C5 + NonUniformCost (256 × 128)
#   prof      rocprofv3 --kernel-trace --stats of the default bench (20 steps after 3 warm-up) + the PMC
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
    sharded)
      timeout -k 10 200 python -u bench.py --sharded --steps 10 --no-cpu-baseline > "$out/bench_c3_sharded.json" 2> "$out/bench_c3_sharded.err" && \
      timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > "$out/bench_c3_plain.json" 2> "$out/bench_c3_plain.err"
      rc=$?
      for f in "$out"/bench_c3_sharded.json "$out"/bench_c3_plain.json; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" "$f"
      done ;;
    prof)
      bash tools/profile.sh "${tag}_c3" --steps 40 --warmup 5 --no-cpu-baseline && bash tools/profile.sh "${tag}_c3mle" --steps 5 --warmup 2 --no-cpu-baseline --mle
      rc=$? ;;
    ab)
      AB_TAG="" timeout -k 10 400 bash tools/ab_run.sh ${AB_VARIANTS:-old new oldst newst} > "$out/ab.log" 2>&1
      rc=$?; cp gpurun_out/ab_*.json gpurun_out/ab_*.err "$out/" 2>/dev/null; grep -v "^\[mrbo stamps\] .* 0.00%" "$out/ab.log" | tail -60 ;;
    gpfit)
      timeout -k 10 400 python -u tools/bench_rows.py --rows gp_fit --gpfit-n ${GPFIT_N:-64,128,256,384,512} --cpu-seconds 2 > "$out/gpfit_rows.jsonl" 2> "$out/gpfit_rows.err"
      rc=$?; python -c "
import sys, json
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(d['config']['workload'], round(d['value']), 'fits/s;', round(d['kernel_ms'], 3), 'ms kernel; frac', round(d['roofline']['frac'], 4))" "$out/gpfit_rows.jsonl" ;;
    bo)
      timeout -k 10 ${BO_TIMEOUT:-1000} python -u tools/bo_compare.py --trials ${BO_TRIALS:-40} --cases ${BO_CASES:-asserted} ${BO_ARGS:-} \
        --out "$out/bo_compare.jsonl" > /dev/null 2> "$out/bo_compare.err"
      rc=$?; grep "final gap" "$out/bo_compare.err" ;;
    shim)
      timeout -k 10 300 python -u tools/shim_rate.py --config C3 > "$out/shim_rate_c3.json" 2> "$out/shim_rate_c3.err"
      rc=$?; cat "$out/shim_rate_c3.json" ;;
    c2)
      timeout -k 10 200 python -u bench.py --config C2 --no-cpu-baseline --steps 20 > "$out/bench_c2.json" 2> "$out/bench_c2.err"
      rc=$?; tail -c 400 "$out/bench_c2.json" ;;
    myopic)
      # the myopic rows that closed less in round 4 (+ the Hartmann-6 EI control): other seeds,
      # interior solves (margins) and the no-repeat pick, 60 trials each
      cases=myopic_hartmann6d_poi,myopic_hartmann6d_lcb,myopic_sixhump_poi,myopic_hartmann6d_ei
      rc=0
      for v in "seed 1" "seed 2" "seed 3" "margin 0.01" "margin 0.05" "norepeat"; do
        set -- $v
        case $1 in
          seed) args="--seed $2"; vt=seed$2 ;;
          margin) args="--solve-margin $2"; vt=margin$2 ;;
          norepeat) args="--no-repeat"; vt=norepeat ;;
        esac
        timeout -k 10 300 python -u tools/bo_compare.py --trials 60 --cases $cases $args \
          --out "$out/bo_myopic_$vt.jsonl" > /dev/null 2> "$out/bo_myopic_$vt.err" || { rc=$?; break; }
        grep "final gap" "$out/bo_myopic_$vt.err"
      done ;;
    c5)
      timeout -k 10 300 python -u bench.py --config C5 --mc-per-gpu 2048 --steps 2 --warmup 1 --no-cpu-baseline \
        > "$out/bench_c5.json" 2> "$out/bench_c5.err" && \
      timeout -k 10 300 python -u bench.py --config C5 --mc-per-gpu 64 --restarts 64 --ell 20 --steps 3 --warmup 1 --no-cpu-baseline \
        > "$out/bench_c5_l20.json" 2> "$out/bench_c5_l20.err"
      rc=$?
      for f in "$out"/bench_c5.json "$out"/bench_c5_l20.json; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['work_per_traj'])" "$f"
      done ;;
    c5cost)
      timeout -k 10 400 python -u bench.py --config C5 --cost --mc-per-gpu 256 --restarts 128 --steps 1 --warmup 1 --no-cpu-baseline \
        > "$out/bench_c5_cost.json" 2> "$out/bench_c5_cost.err"
      rc=$?; tail -c 400 "$out/bench_c5_cost.json" ;;
    ab6)
      # the round-6 library against the round's starting C3 kernel (mrbo/variants/libmrbo_r6old.so),
      # interleaved on one box: C3 and C3-MLE
      REPS=3 TAG=c3 timeout -k 10 400 bash tools/ab_rep.sh r6old ${AB6_VARIANTS:-} main > "$out/ab_c3.log" 2>&1 && \
      REPS=2 TAG=c3mle BENCH_ARGS="--mle" timeout -k 10 500 bash tools/ab_rep.sh r6old ${AB6_VARIANTS:-} main > "$out/ab_c3mle.log" 2>&1
      rc=$?; cat "$out/ab_c3.log" "$out/ab_c3mle.log" | grep -v "mrbo stamps" | tail -24 ;;
    ab6c5)
      # C5 + NonUniformCost (the bench row's shape, 256 × 128 per launch): this library vs r6old
      REPS=2 STEPS=1 TAG=c5cost BENCH_ARGS="--config C5 --cost --mc-per-gpu 256 --restarts 128" \
        timeout -k 10 600 bash tools/ab_rep.sh ${AB6C5_VARIANTS:-r6old main} > "$out/ab_c5cost.log" 2>&1
      rc=$?; grep -v "mrbo stamps" "$out/ab_c5cost.log" | tail -8 ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "== $step rc=$rc $(date +%T)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
