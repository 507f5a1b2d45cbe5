#!/bin/bash
# Round-3 session L: the persistent thin-factor loop (k_thin_loop) and the canonical-order
# thin solve (k_thin_solve): focused parity tests, the full GPU suite, C3 bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 120 --timeout-method thread \
  -k "thin or timeout or batched_equals_single or iteration_count or max_iter_one" > gpurun_out/l_thin.log 2>&1
rc=$?; tail -3 gpurun_out/l_thin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/l_r18.log 2>&1 || exit $?
tail -c 300 gpurun_out/l_r18.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/l_tests.log 2>&1; rc=$?; tail -2 gpurun_out/l_tests.log; [ $rc -eq 0 ] || exit $rc
echo done
