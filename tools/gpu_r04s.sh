#!/bin/bash
# Round-4 session S: the EPC multiplier on the device (no per-step host sync), the
# library eigensolver restored: EPC tests + timing, low-rank tests + bench.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "s_tests|400|python -u -m pytest tests/test_gpu_epc.py tests/test_gpu_panel.py tests/test_gpu_lowrank.py -x -v --timeout 200 --timeout-method thread -s" \
  "s_lrb|200|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0"
