#!/bin/bash
# Round-3 session S (re-entry 3): what bounds the fp32 solve GEMM per CU (timeline of the full
# kernel, of its K-loop without MFMAs (diaglib1) and without global -> LDS staging (diaglib2)),
# and the phase timeline of the fused search at C3 mode 0 in the fp32 form.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "s_gemm_full|120|ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "s_gemm_nomfma|120|ADMMQ_LIB=$PWD/tools/diaglib1/libadmmq.so python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "s_gemm_nostage|120|ADMMQ_LIB=$PWD/tools/diaglib2/libadmmq.so python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "s_hist0|120|ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so python -u tools/hist_timeline.py --mode 0 --iters 6"
