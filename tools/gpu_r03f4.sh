#!/bin/bash
# Round-3 session F4: half tiles for CU balance (split_for_balance; same bits): the GPU
# configs / parity suites incl. the staging-forms bit-equality test, C3 A/B against whole
# tiles (ADMMQ_HALF_TILES=0), GEMM timeline of C3 mode 0, emulated 8-GPU shards.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "f4_tests|600|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py" \
  "f4_r18|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "f4_r18_whole|300|ADMMQ_HALF_TILES=0 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "f4_tl0|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "f4_emu18|300|python -u bench.py --emulate-world 8 --steps 1 --warmup 1"
