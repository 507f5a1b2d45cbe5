#!/bin/bash
# Round-4 session A: K-split solve tiles - GEMM parity tests, C3 A/B, emulated 8-GPU C4 / C3.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "a_pytest|400|python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k 'ksplit or staging or wide or c3_batched or c3_resnet18 or c4_batched'" \
  "a_bench_ks1|240|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit 1" \
  "a_bench_ks0|240|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit 0" \
  "a_emu50|400|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1" \
  "a_emu18|300|python -u bench.py --emulate-world 8 --steps 2 --warmup 1"
