#!/bin/bash
# Round-3 session H: fp32 solve with one tile per workgroup and per-problem tile rows
# (k_gemm_f32t, 2-stage ring, 3 workgroups/CU) against k_gemm at C3 / C4 / C5.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in "0 0" "2 3" "2 0" "2 1"; do
  set -- $k
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --f32-kernel $1 --f32-tiles $2 \
    > gpurun_out/h_r18_k$1_t$2.log 2>&1 || exit $?
done
for k in "0 0" "2 3"; do
  set -- $k
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline --f32-kernel $1 \
    --f32-tiles $2 > gpurun_out/h_r50_k$1_t$2.log 2>&1 || exit $?
done
echo done
