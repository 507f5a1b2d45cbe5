#!/bin/bash
# Round-3 session J: fused finalize with several units per block (C4's 48-layer batch):
# parity (fused == separate, forced small budgets; fault repair), then C4 / C3 bench lines.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fused or timeout" tests/test_gpu_configs.py -k "c4 or fused or timeout" \
  > gpurun_out/j_tests.log 2>&1; rc=$?; tail -2 gpurun_out/j_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/j_r50.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/j_r18.log 2>&1 || exit $?
echo done
