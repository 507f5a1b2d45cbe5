#!/bin/bash
# Round-2 session P: XCD row-panel placement for multi-round 64x64 launches (C4): GPU parity
# suite, then the C4 and C5 bench lines (no CPU leg) against session M.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_p.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_p_r50.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_p_r50.log
timeout -k 10 400 python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_p_llama.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_p_llama.log
