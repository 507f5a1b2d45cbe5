#!/bin/bash
# Round-3 session Z: fp32 64x64 staging ring depth on C4 (2-deep ring: 32 KB per workgroup,
# 4 workgroups per CU for its 2-round launches) and C5 / C3 for reference.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "z_r50_s2|300|ADMMQ_GEMM_F32_STAGE=2 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "z_r50_s3|300|ADMMQ_GEMM_F32_STAGE=3 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "z_r18_s2|300|ADMMQ_GEMM_F32_STAGE=2 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline"
