#!/bin/bash
# GP-fit: GPU tests (tests/test_mle.py) then the gp_fit bench rows (N = 64 / 128 / 256).
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/gpfit
mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_mle.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?
tail -25 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_rows.py --rows gp_fit --cpu-seconds 2 > $out/rows.jsonl 2> $out/rows.err
rc=$?
cat $out/rows.jsonl | python -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(d['config']['workload'], round(d['value']), 'fits/s call;', round(d['kernel_fits_per_s']), 'fits/s kernel;', d['kernel_ms'], 'ms; frac', round(d['roofline']['frac'], 4))"
exit $rc
