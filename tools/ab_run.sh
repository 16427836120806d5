set -e
export TMPDIR=/tmp
for v in base inl inl_nolicm w1; do
  MRBO_LIB=$PWD/rollout-bayesian-optimization_amd/mrbo/variants/libmrbo_$v.so timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null
done
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1
