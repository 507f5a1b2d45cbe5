#!/bin/bash
# Round-4 session R: the one-workgroup Jacobi eigensolver (Rayleigh-Ritz of the rank
# projection, EPC's R x R eigensolves): tests, (f)3 and (f)2 timings.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "r_tests|300|python -u -m pytest tests/test_gpu_panel.py tests/test_gpu_lowrank.py tests/test_gpu_epc.py -x -v --timeout 120 --timeout-method thread -s" \
  "r_lrb|200|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0" \
  "r_f3|300|python -u tools/lowrank_bench.py --svd-sample 0"
