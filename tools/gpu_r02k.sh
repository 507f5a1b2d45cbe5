#!/bin/bash
# Round-2 session K: register-staged 64x64 solve tiles: GPU parity suite, then the C3 and C4
# bench lines (no CPU leg) for the A/B against session H.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_k.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k_r18.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench_k_r18.log
timeout -k 10 300 python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k_r50.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_k_r50.log
