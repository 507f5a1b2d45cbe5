#!/bin/bash
# Round-3 session C: the new GPU tests (fault repair, channel KATs, C5 full-layer batch,
# Krylov projection on flat iterates, F7 21/21), fp32 C3 rocprof evidence (kernel trace +
# PMC passes), the two-stream probe, and the (f)3 low-rank timing with the exact-agreeing
# projection.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_fused_finalize_timeout_reported_and_repaired \
  tests/test_gpu_parity.py::test_channel_schemes_reference_kats tests/test_gpu_configs.py::test_c5_llama_full_layer_batch \
  tests/test_gpu_lowrank.py tests/test_gpu_reference.py tests/test_torch_ops.py \
  > gpurun_out/c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/c_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh r03a resnet18 > gpurun_out/c_profile.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/two_stream_probe.py 201 fused > gpurun_out/c_2s_fused.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/two_stream_probe.py 201 nofused > gpurun_out/c_2s_nofused.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/lowrank_bench.py > gpurun_out/c_lowrank.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --gemm-ks 2 > gpurun_out/c_r18_ks2.log 2>&1 || exit $?
echo done
