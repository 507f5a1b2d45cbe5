#!/bin/bash
# Round-3 session G: what bounds the fp32 solve GEMM per CU: timeline of the full kernel,
# of its K-loop without MFMAs (diaglib1) and without global -> LDS staging (diaglib2).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in tracelib diaglib1 diaglib2; do
  ADMMQ_LIB=$PWD/tools/$v/libadmmq.so timeout -k 10 120 python -u tools/gemm_timeline.py --mode 0 --iters 6 \
    > gpurun_out/g_$v.log 2>&1 || exit $?
done
echo done
