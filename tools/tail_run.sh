set -e
mkdir -p gpurun_out/tail
L=rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_tail.so
MRBO_LIB=$L timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tail/c3.json 2> gpurun_out/tail/c3.err
MRBO_LIB=$L timeout -k 10 120 python -u bench.py --mle --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tail/c3mle.json 2> gpurun_out/tail/c3mle.err
MRBO_LIB=$L timeout -k 10 120 python -u bench.py --mc-per-gpu 2048 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tail/c3m2048.json 2> gpurun_out/tail/c3m2048.err
grep "mrbo tail" gpurun_out/tail/*.err
