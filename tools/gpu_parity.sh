#!/bin/bash
# GPU parity suite only (tests/test_gpu_parity.py), report JSON under gpurun_out/<tag>/.
root=${GRAFT_REPO_ROOT:-$PWD}
out=$root/gpurun_out/${1:-parity}
mkdir -p $out
cd $root
export MRBO_PARITY_REPORT=$out/parity.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?
tail -15 $out/pytest.log
exit $rc
