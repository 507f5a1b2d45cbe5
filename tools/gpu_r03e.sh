#!/bin/bash
# Round-3 session E: fp32 GEMM fragment double-buffering (sched_group_barrier) A/B on C3.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "c3_resnet18 and fp32" > gpurun_out/e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/e_r18.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e_ktrace -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/e_ktrace.log 2>&1 || exit $?
echo done
