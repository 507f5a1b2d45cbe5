#!/bin/bash
# Round-4 session AI: stage-1 level reads batched before their compares (QMAX <= 8) in the
# thin loop and the legacy stage 1 - thin / search tests, thin-loop phases, C3 bench.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "ai_tests|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread" \
  "ai_tl|200|ADMMQ_LIB=$T python -u tools/thin_loop_timeline.py" \
  "ai_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
