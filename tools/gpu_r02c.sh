#!/bin/bash
# Round-2 session C: full GPU suite, the C3 bench line (with CPU baseline), C3 rocprof profile.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r18.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_r18.log
timeout -k 10 600 bash tools/profile.sh r02 resnet18 > /dev/null || exit $?
echo profiled
