#!/bin/bash
# Round-2 session G: full GPU suite, then C3 and C5 bench lines (no CPU leg) for an A/B
# against the session-F profiles (thin-solve sc1 hand-off, XCD row-panel wide-tile order).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_g.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_g_r18.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench_g_r18.log
timeout -k 10 400 python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_g_llama.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench_g_llama.log
