set -e
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/r6a; mkdir -p $out
cd $root
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench_plain.json 2> $out/bench_plain.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 $root/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench_prof.json 2> $out/bench_prof.err
echo done
