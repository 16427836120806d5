#!/bin/bash
# round-6 session 2: GPU tests, default bench, tail vs steps (sort once / re-sort every step)
root=${GRAFT_REPO_ROOT:-$PWD}; cd "$root"
out=gpurun_out/r6j; mkdir -p $out
export MRBO_PARITY_REPORT=$out/parity.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $out/bench_c3.json
L=rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_tail.so
for rs in 0 1; do
  MRBO_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --resort $rs --no-cpu-baseline > $out/tail20_rs$rs.json 2> $out/tail20_rs$rs.err || exit 1
  echo "resort $rs"; grep "mrbo tail" $out/tail20_rs$rs.err | awk '{print $9, $10, $11, $12, $13}' | tr '\n' ';'; echo
done
timeout -k 10 200 python -u bench.py --mle --no-cpu-baseline > $out/bench_c3_mle.json 2> $out/bench_c3_mle.err || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mle', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $out/bench_c3_mle.json
L8=rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_tail8.so
for s in index longest-first; do
  MRBO_LIB=$L8 timeout -k 10 400 python -u bench.py --config C5 --cost --mc-per-gpu 256 --restarts 128 --steps 1 --warmup 1 --schedule $s --no-cpu-baseline \
    > $out/c5cost_$s.json 2> $out/c5cost_$s.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5cost', sys.argv[2], d['value'], d['roofline']['kernel_ms'])" $out/c5cost_$s.json $s
  grep "mrbo tail" $out/c5cost_$s.err | tail -1
done
