set -e
# Kernel-trace stats of the non-headline rows (C4, C5, C2) under rocprofv3, beside tools/profile.sh.
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/prof_rows
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c4 -o run -- python3 $root/bench.py --config C4 --mc-per-gpu 1024 --steps 2 --warmup 1 --no-cpu-baseline > $out/c4.json 2> $out/c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c5 -o run -- python3 $root/bench.py --config C5 --mc-per-gpu 256 --steps 2 --warmup 1 --no-cpu-baseline > $out/c5.json 2> $out/c5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c2 -o run -- python3 $root/bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > $out/c2.json 2> $out/c2.err
echo rows done
