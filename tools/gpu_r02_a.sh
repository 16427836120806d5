#!/bin/bash
# Round-2 GPU session A: GPU test suite (incl. full-size parity), then the bench rows.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/r02a
mkdir -p $out
cd $root
export MRBO_PARITY_REPORT=$out/parity.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
tail -5 $out/pytest.log
timeout -k 10 240 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err && \
timeout -k 10 120 python -u bench.py --mle --no-cpu-baseline > $out/bench_c3_mle.json 2> $out/bench_c3_mle.err && \
timeout -k 10 120 python -u bench.py --config C4 --mc-per-gpu 1024 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_c4.json 2> $out/bench_c4.err && \
timeout -k 10 120 python -u bench.py --config C4 --mc-per-gpu 1024 --steps 3 --warmup 1 --mle --no-cpu-baseline > $out/bench_c4_mle.json 2> $out/bench_c4_mle.err && \
timeout -k 10 120 python -u bench.py --config C5 --mc-per-gpu 2048 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err && \
timeout -k 10 120 python -u bench.py --config C5 --mc-per-gpu 64 --restarts 64 --steps 2 --warmup 1 --ell 20 --no-cpu-baseline > $out/bench_c5_l20.json 2> $out/bench_c5_l20.err && \
timeout -k 10 120 python -u bench.py --config C5 --mc-per-gpu 256 --steps 2 --warmup 1 --cost --no-cpu-baseline > $out/bench_c5_cost.json 2> $out/bench_c5_cost.err
echo "bench rc=$?"
for f in $out/bench_*.json; do echo "$f"; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['work_per_traj'], d['config'].get('kernel'))" $f; done
