#!/bin/bash
# WRITE_SIZE / FETCH_SIZE passes (separate rocprofv3 --pmc runs) of the C3 bench for library variants.
# usage (on the box, repo root): bash tools/wr_pass.sh <variant> [<variant> ...]   -> gpurun_out/wr_<v>_{write,fetch}/
root=${GRAFT_REPO_ROOT:-$PWD}
V=$root/rollout-bayesian-optimization_amd/mrbo/variants
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  for c in WRITE_SIZE FETCH_SIZE; do
    MRBO_LIB=$V/libmrbo_$v.so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$root/gpurun_out/wr_${v}_$c" -o run \
      -- python3 "$root/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$root/gpurun_out/wr_${v}_$c.log" 2>&1 || exit 1
  done
  python3 - "$root/gpurun_out" "$v" <<'PY'
import csv, glob, sys
out, v = sys.argv[1], sys.argv[2]
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    vals = []
    for f in glob.glob(f"{out}/wr_{v}_{c}/**/run_counter_collection.csv", recursive=True) + glob.glob(f"{out}/wr_{v}_{c}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "rollout_kernel" in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    print(v, c, "KB per launch (per dispatch sums):", sorted(set(round(x, 1) for x in vals)))
PY
done
