#!/bin/bash
# Round-3 session N: 64-column loop teams (parity), finer phase breakdown of k_thin_loop.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 120 --timeout-method thread \
  -k "thin or timeout or batched_equals_single" > gpurun_out/n_thin.log 2>&1
rc=$?; tail -3 gpurun_out/n_thin.log; [ $rc -eq 0 ] || exit $rc
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 300 python -u tools/thin_loop_timeline.py \
  > gpurun_out/n_tl_r18.log 2>&1 || exit $?
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 300 python -u tools/thin_loop_timeline.py --model resnet50 \
  > gpurun_out/n_tl_r50.log 2>&1 || exit $?
cat gpurun_out/n_tl_r18.log gpurun_out/n_tl_r50.log
echo done
