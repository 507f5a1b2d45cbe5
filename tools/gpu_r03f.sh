#!/bin/bash
# Round-3 session F: per-workgroup timeline of the fp32 solve GEMM (TRACE library) at C3 modes 0 and 1.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so
timeout -k 10 120 python -u tools/gemm_timeline.py --mode 0 --iters 6 > gpurun_out/f_tl0.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/gemm_timeline.py --mode 1 --iters 6 > gpurun_out/f_tl1.log 2>&1 || exit $?
echo done
