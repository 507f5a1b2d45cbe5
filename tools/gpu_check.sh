#!/bin/bash
# One GPU box session: parity tests, then (only if no fault/timeout) a short bench.
# Usage: tools/gpu_check.sh [pytest-args...]   (outputs under gpurun_out/)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -c 3000 gpurun_out/bench.log
exit $brc
