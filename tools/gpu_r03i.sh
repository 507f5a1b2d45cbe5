#!/bin/bash
# Round-3 session I: phase timelines of the fused search (mode 0) and the small-job kernel (mode 2), fp32 solve.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so
timeout -k 10 120 python -u tools/hist_timeline.py --mode 0 --iters 6 > gpurun_out/i_hist0.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/small_timeline.py --mode 2 > gpurun_out/i_small2.log 2>&1 || exit $?
echo done
