#!/bin/bash
# Round-2 session N: GPU parity suite, then the C5 bench line (no CPU leg) for the A/B of the
# prefetching multi-unit search against session M.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_n.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_n.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n_llama.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_n_llama.log
