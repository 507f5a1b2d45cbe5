#!/bin/bash
# Round-2 GPU session: reference parity tests, one bench line, then the C3 rocprof profile.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_reference.py -q -rf --timeout 120 --timeout-method thread \
  > gpurun_out/ref_tests.log 2>&1
rc=$?; echo "ref tests rc=$rc"; tail -5 gpurun_out/ref_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r18.log 2>&1 || exit $?
tail -c 1500 gpurun_out/bench_r18.log
timeout -k 10 900 bash tools/profile.sh r02 resnet18
