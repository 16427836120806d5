#!/bin/bash
# within-chunk longest-first: schedule tests, C3 A/B (index vs longest-first) + tail, write traffic
root=${GRAFT_REPO_ROOT:-$PWD}; cd "$root"
out=gpurun_out/r6l; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu.py -k "schedule or order or stochastic" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -ne 0 ] && { grep FAILED $out/pytest.log; exit $rc; }
TAG=r6l bash tools/sched_ab.sh || exit 1
bash tools/profile.sh r6l_c3 --steps 40 --warmup 5 --no-cpu-baseline || exit 1
