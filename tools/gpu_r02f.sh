#!/bin/bash
# Round-2 session F/I (part 1, final tree): full GPU suite, then the rocprofv3 kernel-trace + PMC
# profiles of C3 / C4 / C5 (tools/profile.sh). Part 2 (tools/gpu_r02e.sh) runs the bench
# lines once the traffic files are regenerated from these profiles.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for m in resnet18 resnet50 llama7b; do
  timeout -k 10 300 bash tools/profile.sh r02f $m > gpurun_out/profile_$m.log 2>&1 || exit $?
  echo "profiled $m"
done
