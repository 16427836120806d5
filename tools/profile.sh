#!/bin/bash
# Profile the headline bench on the GPU box: kernel-trace stats + separate PMC passes.
# Usage (on the box, from the repo root): bash tools/profile.sh <tag> [bench args...]
# Outputs under gpurun_out/prof_<tag>/ ; copy the summaries worth keeping into profiles/.
set -e
tag=${1:-run}; shift || true
args=${*:-"--steps 1 --warmup 1 --no-cpu-baseline"}
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
run() {  # run <name> <rocprofv3 options...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$out/$name" -o run -- \
    python3 "$root/bench.py" $args > "$out/$name.log" 2>&1
}
run stats --kernel-trace --stats
run pmc_issue --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
run pmc_valu --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU
run pmc_lds --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_CVT
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
echo "profile $tag done: $out"
