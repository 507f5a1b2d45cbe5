#!/bin/bash
# Round-3 session F9: fp32 64x64 tiles with the MFMA bursts at raised issue priority
# (ADMMQ_GEMM_F32_STAGE=4, same bits) against the default: C3 config tests under stage 4,
# C3 / C4 bench A/B.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "f9_tests4|400|ADMMQ_GEMM_F32_STAGE=4 python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k 'c3 or staging'" \
  "f9_r18_s4|300|ADMMQ_GEMM_F32_STAGE=4 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "f9_r18_s3|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "f9_r50_s4|300|ADMMQ_GEMM_F32_STAGE=4 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "f9_r50_s3|300|python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline"
