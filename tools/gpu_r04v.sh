#!/bin/bash
# Round-4 session V: the paired-K-step GEMM ring (gemm stage 5) - same-bits tests, then
# A/B against stage 3 at C3, C4 and the lone layer4 shard.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "v_tests|300|python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k 'staging_forms or ksplit'" \
  "v_c3_s3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --gemm-stage 3" \
  "v_c3_s5|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --gemm-stage 5" \
  "v_c4_s3|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --gemm-stage 3" \
  "v_c4_s5|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --gemm-stage 5" \
  "v_emu_s5|200|python -u bench.py --emulate-world 8 --model resnet50 --emulate-only 0,3 --steps 2 --warmup 1 --gemm-stage 5"
