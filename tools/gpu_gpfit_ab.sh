#!/bin/bash
# GP-fit check on the GPU box: test_mle.py (device fits vs the oracle), then the gp_fit rows of the
# default library and the phase stamps of the -DMRBO_GPFIT_STAMPS variant (variants/libmrbo_gpst.so).
# usage: bash tools/gpu_gpfit_ab.sh <tag>
tag=${1:-gpfit}
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_mle.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$out/pytest_mle.log" 2>&1 || { tail -30 "$out/pytest_mle.log"; exit 1; }
tail -2 "$out/pytest_mle.log"
timeout -k 10 300 python -u tools/bench_rows.py --rows gp_fit --cpu-seconds 0.5 > "$out/gpfit_rows.jsonl" 2> "$out/gpfit_rows.err" || exit 1
python -c "
import sys, json
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(d['config']['workload'], round(d['value']), 'fits/s per call;', round(d['kernel_ms'], 3), 'ms kernel; frac', round(d['roofline']['frac'], 4))" "$out/gpfit_rows.jsonl"
MRBO_LIB=$PWD/rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_gpst.so timeout -k 10 200 python -u tools/bench_rows.py --rows gp_fit --gpfit-n 96,128,192,256 --cpu-seconds 0.2 > "$out/gpfit_stamps.jsonl" 2> "$out/gpfit_stamps.err" || exit 1
grep -h "gpfit_tile" "$out/gpfit_stamps.jsonl" "$out/gpfit_stamps.err" | sort -t= -k2 -n | awk 'NR%6==1'
