#!/bin/bash
# Round-3 session X: fused search finalize re-reading H_T / U (no stage-1 registers held
# through the search) with per-group stores: parity tests of the fused path, C3 bench,
# search phase timeline.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "x_tests|600|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k 'fused or c3 or timeout or batched or step'" \
  "x_r18|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "x_hist0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6"
