#!/bin/bash
# Round-3 session R: rocprofv3 evidence for the fp32-solve C3 bench (kernel trace + PMC
# passes), then the fp32 GEMM per-workgroup timeline: full kernel, K-loop without MFMAs
# (diaglib1), K-loop without global -> LDS staging (diaglib2).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile.sh r03r resnet18 || exit $?
for v in tracelib diaglib1 diaglib2; do
  ADMMQ_LIB=$PWD/tools/$v/libadmmq.so timeout -k 10 120 python -u tools/gemm_timeline.py --mode 0 --iters 6 \
    > gpurun_out/r_gemm_$v.log 2>&1 || exit $?
done
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 120 python -u tools/hist_timeline.py --mode 0 --iters 6 \
  > gpurun_out/r_hist.log 2>&1 || exit $?
echo done
