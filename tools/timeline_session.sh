#!/bin/bash
# Phase timelines of the search kernels (diagnostics) with the `make TRACE=1` library
# built into tools/tracelib/ (make -C admm-quantization_amd/csrc TRACE=1 OBJDIR=../../build/objt
# OUT=../../tools/tracelib/libadmmq.so OPS_OUT=../../tools/tracelib/libadmmq_torch.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so
mkdir -p gpurun_out
( timeout -k 10 120 python -u tools/hist_timeline.py --mode 0 --iters 6 && \
  timeout -k 10 120 python -u tools/small_timeline.py --mode 2 ) > gpurun_out/timeline.log 2>&1
rc=$?; cat gpurun_out/timeline.log; exit $rc
