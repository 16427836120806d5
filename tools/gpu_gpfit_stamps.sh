mkdir -p gpurun_out/r4f
MRBO_LIB=$PWD/rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_gpst.so timeout -k 10 200 python -u tools/bench_rows.py --rows gp_fit --gpfit-n 96,128,192,256 --cpu-seconds 0.5 > gpurun_out/r4f/gpfit_stamps.jsonl 2> gpurun_out/r4f/gpfit_stamps.err; echo rc=$?
grep -h "gpfit_tile" gpurun_out/r4f/gpfit_stamps.jsonl gpurun_out/r4f/gpfit_stamps.err | sort | uniq -c | head -20
