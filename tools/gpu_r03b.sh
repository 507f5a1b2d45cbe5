#!/bin/bash
# Round-3 session B: persistent fp32 solve (k_gemm_f32p): GPU parity on the solve / config
# tests, then C3 bench lines for the tile rules (9 = the previous k_gemm), C4 for 1 and 9.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q -rf \
  --timeout 300 --timeout-method thread > gpurun_out/b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/b_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 9 0 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --f32-tiles $r > gpurun_out/b_r18_t$r.log 2>&1 || exit $?
done
for r in 9 1; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline --f32-tiles $r > gpurun_out/b_r50_t$r.log 2>&1 || exit $?
done
echo done
