#!/bin/bash
# Round-2 session Q: paired threshold probes in the stage-1 insert: GPU parity suite, then the
# C3 and C5 bench lines (no CPU leg) against the v5 lines.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_q.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q_r18.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_q_r18.log
timeout -k 10 400 python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q_llama.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_q_llama.log
