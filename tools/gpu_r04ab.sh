#!/bin/bash
# Round-4 session AB: forced multi-candidate selection (sel_widen) gives the same bits;
# parity / configs suites and a C3 bench on the tree with the switch.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "ab_widen|300|python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k widened" \
  "ab_tests|600|python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread" \
  "ab_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
